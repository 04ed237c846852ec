// host_copy.h -- the host runtime's multi-threaded staging copies (pageable
// payload -> pinned staging buffer), kept free of HIP so the CPU test-suite
// can run them under ThreadSanitizer (tests/sanitize/host_tsan.cpp).
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace hdfs_crc {

// Host threads for the staging copy of pageable payloads: one memcpy thread
// moves ~24 GB/s on the GPU box's EPYC, under half the PCIe link (config 2
// from pageable memory: 28 / 38 / 42 / 45 GiB/s with 1 / 2 / 4 / 8 threads).
// Default 8 (at most half the hardware threads); $HDFS_CRC32C_COPY_THREADS
// = 1..32 overrides.
inline unsigned copy_threads() {
    static const unsigned v = [] {
        const char *e = std::getenv("HDFS_CRC32C_COPY_THREADS");
        if (e && std::atoi(e) >= 1 && std::atoi(e) <= 32) return unsigned(std::atoi(e));
        const unsigned hw = std::thread::hardware_concurrency();
        return std::max(1u, std::min(8u, hw / 2));
    }();
    return v;
}

// Runs f(begin, end) over [0, n) items split evenly on up to copy_threads()
// threads (the calling thread takes the first part); `bytes` is the work
// size, and below 8 MiB everything stays on the calling thread.
template <class F>
void parallel_copy(size_t n, size_t bytes, F f) {
    const unsigned t = bytes < (8u << 20) ? 1u : unsigned(std::min<size_t>(copy_threads(), n ? n : 1));
    if (t <= 1) {
        f(size_t(0), n);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(t - 1);
    for (unsigned k = 1; k < t; ++k) th.emplace_back(f, n * k / t, n * (k + 1) / t);
    f(size_t(0), n / t);
    for (auto &x : th) x.join();
}

// memcpy of a large range on parallel_copy's threads (64-byte pieces).
inline void copy_range(uint8_t *dst, const uint8_t *src, size_t n) {
    const size_t lines = (n + 63) / 64;
    parallel_copy(lines, n, [=](size_t b, size_t e) {
        const size_t lo = b * 64, hi = std::min(n, e * 64);
        if (hi > lo) std::memcpy(dst + lo, src + lo, hi - lo);
    });
}

// Staging copy of a large range in pieces: copy_threads() threads each copy
// their share of piece 0, 1, ... in turn; when every share of piece p is in,
// the calling thread (also a copier) hands the piece to ready(offset, size),
// which queues its H2D copy.  Threads are started once per call.
template <class R>
void copy_range_pipelined(uint8_t *dst, const uint8_t *src, size_t n, size_t piece, R ready) {
    const unsigned t = n < (8u << 20) ? 1u : copy_threads();
    const size_t npieces = (n + piece - 1) / piece;
    std::vector<std::atomic<unsigned>> done(npieces);
    for (auto &d : done) d.store(0, std::memory_order_relaxed);
    auto work = [&](unsigned k) {
        for (size_t p = 0; p < npieces; ++p) {
            const size_t b = p * piece, e = std::min(n, b + piece);
            const size_t lines = (e - b + 63) / 64;
            const size_t lo = b + lines * k / t * 64, hi = std::min(e, b + lines * (k + 1) / t * 64);
            if (hi > lo) std::memcpy(dst + lo, src + lo, hi - lo);
            done[p].fetch_add(1, std::memory_order_release);
        }
    };
    std::vector<std::thread> th;
    th.reserve(t - 1);
    for (unsigned k = 1; k < t; ++k) th.emplace_back(work, k);
    // the calling thread: its own share, then publish pieces as they complete
    size_t next = 0;
    for (size_t p = 0; p < npieces; ++p) {
        const size_t b = p * piece, e = std::min(n, b + piece);
        const size_t lines = (e - b + 63) / 64;
        const size_t hi = std::min(e, b + lines / t * 64);
        if (hi > b) std::memcpy(dst + b, src + b, hi - b);
        done[p].fetch_add(1, std::memory_order_release);
        for (; next <= p && done[next].load(std::memory_order_acquire) == t; ++next)
            ready(next * piece, std::min(n, next * piece + piece) - next * piece);
    }
    for (; next < npieces; ++next) {
        while (done[next].load(std::memory_order_acquire) != t) std::this_thread::yield();
        ready(next * piece, std::min(n, next * piece + piece) - next * piece);
    }
    for (auto &x : th) x.join();
}

}  // namespace hdfs_crc
