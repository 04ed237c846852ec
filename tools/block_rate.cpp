// block_rate.cpp -- diagnostic: concurrent 4 MiB block writes from C, the
// shape of libfuse's worker threads each running hadoop_fuse_write_block
// (src/fuse.c:336-449, many threads: fuse.c:1771).  Every thread checksums
// one device-resident 4 MiB block (64 x 64 KiB packets, bpc 512) per
// iteration and waits for it, T threads at once; prints one JSON line per
// mode with the wall time per block over all threads:
//   single  -- one crc32c_plan_exec per block on the thread's own stream, then
//              a stream synchronisation (what a caller does without batching)
//   queue   -- crc32c_block_checksums through one crc32c_blocks queue
//              (group commit into multi-block launches), one block in flight
//              per thread
//   queue2  -- the same with two blocks in flight per thread (submit the next,
//              then wait for the previous)
//   kernel  -- one thread issuing crc32c_plan_exec_blocks of B blocks back to
//              back: the GPU's time per block in a multi-block launch (events)
//   rqueue, rqueue2 -- the queue's resident mode (crc32c_blocks_create_resident:
//              a resident kernel, no launch per block), one / two blocks in
//              flight per thread, every block checked against the queue's
//              checksums of the same buffer
//   resident, resident2 -- the debug library's A/B shapes of that kernel
//              (crc32c_debug_resident_*, HDFS_CRC32C_RESIDENT_WAVES)
// Every line has cpu_us_per_block: the process's CPU time (getrusage) per
// block -- the submitting threads' and the queue worker's spinning included;
// queue lines also the worker thread's own (worker_cpu_us_per_block, and
// worker_busy = its CPU seconds per wall second).
//
//   rqueue_mixed, rqueue2_mixed, queue2_mixed -- (mixed = 1) every other block
//              of a thread is the first block of an append at an unaligned
//              offset (hadoop_fuse_do_write, src/fuse.c:488-574: write_block at
//              blockoffset > 0, the first packet trimmed to a chunk boundary,
//              hadooprpc.c:832-840) through crc32c_block_submit_plan with its own
//              plan, the payload off 16-byte alignment; checked against
//              crc32c_plan_exec of the same plan and bytes
//
//   tools/block_rate [threads=16] [iterations=400] [max_blocks=16] [window_us=30]
//                    [max_depth=2] [queue_modes_only=0] [mixed=0: 1 = the mixed modes only]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/resource.h>
#include <thread>
#include <string>
#include <vector>

#include "hdfs_crc32c.h"
#include "hdfs_crc32c_debug.h"

#define CHECK(x)                                                                      \
    do {                                                                              \
        if (!(x)) {                                                                   \
            std::fprintf(stderr, "block_rate: %s failed (line %d): %s\n", #x, __LINE__, \
                         crc32c_last_error());                                        \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

using Clock = std::chrono::steady_clock;

// The cgroup's CPU throttling so far (cgroup v2 cpu.stat; -1 if unreadable)
// and the process's CPU time: a run that spins more threads than the
// container's CPU quota is throttled, which shows here.
static long long throttled_usec() {
    FILE *f = std::fopen("/sys/fs/cgroup/cpu.stat", "r");
    if (!f) return -1;
    char key[64];
    long long v, r = -1;
    while (std::fscanf(f, "%63s %lld", key, &v) == 2)
        if (!std::strcmp(key, "throttled_usec")) r = v;
    std::fclose(f);
    return r;
}
static double cpu_seconds() {
    rusage u{};
    getrusage(RUSAGE_SELF, &u);
    return double(u.ru_utime.tv_sec + u.ru_stime.tv_sec) + 1e-6 * double(u.ru_utime.tv_usec + u.ru_stime.tv_usec);
}

static double seconds(Clock::time_point a, Clock::time_point b) {
    return std::chrono::duration<double>(b - a).count();
}

int main(int argc, char **argv) {
    std::setvbuf(stdout, nullptr, _IOLBF, 0);  // (lines survive a crash when stdout is a file)
    const int nthreads = argc > 1 ? std::atoi(argv[1]) : 16;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 400;
    const uint32_t max_blocks = argc > 3 ? uint32_t(std::atoi(argv[3])) : 16u;
    const uint32_t window_us = argc > 4 ? uint32_t(std::atoi(argv[4])) : 30u;
    constexpr size_t kBlock = 4u << 20;
    constexpr int kPkts = 64;
    std::vector<crc32c_packet> pk(kPkts);
    for (int i = 0; i < kPkts; ++i) pk[i] = crc32c_packet{uint64_t(i) * 65536u, uint64_t(i) * 128u, 65536u, 512u};
    const size_t nout = kPkts * 128;

    crc32c_ctx *ctx = nullptr;
    CHECK(crc32c_ctx_create(0, &ctx) == 0);
    crc32c_plan *plan = nullptr;
    CHECK(crc32c_plan_create(ctx, pk.data(), pk.size(), 0, &plan) == 0);
    const int maxdepth = argc > 5 ? std::atoi(argv[5]) : 2;  // blocks in flight per thread (queue modes)
    const bool sweep_only = argc > 6 && std::atoi(argv[6]) != 0;  // only the queue modes
    const int nbuf = std::max(2, maxdepth) * nthreads;
    std::vector<uint8_t *> bufs(nbuf);
    std::vector<uint32_t *> outs(nbuf);
    for (int i = 0; i < nbuf; ++i) {
        CHECK(hipMalloc(&bufs[i], kBlock) == hipSuccess);
        CHECK(hipMemset(bufs[i], i * 37 + 1, kBlock) == hipSuccess);
        CHECK(hipMalloc(&outs[i], nout * 4) == hipSuccess);
    }
    CHECK(hipDeviceSynchronize() == hipSuccess);
    const bool mixed_only = argc > 7 && std::atoi(argv[7]) != 0;

    auto run = [&](const char *mode, auto body) {
        std::atomic<int> ready{0};
        std::atomic<bool> go{false};
        std::vector<std::thread> th;
        Clock::time_point t0, t1;
        for (int k = 0; k < nthreads; ++k)
            th.emplace_back([&, k] {
                ready++;
                while (!go.load()) std::this_thread::yield();
                body(k);
            });
        while (ready.load() < nthreads) std::this_thread::yield();
        const long long th0 = throttled_usec();
        const double c0 = cpu_seconds();
        t0 = Clock::now();
        go = true;
        for (auto &t : th) t.join();
        t1 = Clock::now();
        const double s = seconds(t0, t1);
        const double cpus = (cpu_seconds() - c0) / s;
        const long long th1 = throttled_usec();
        const double blocks = double(nthreads) * iters;
        std::printf("{\"mode\": \"%s\", \"threads\": %d, \"blocks\": %.0f, \"us_per_block\": %.3f, \"gib_s\": %.1f, "
                    "\"cpus_busy\": %.2f, \"cpu_us_per_block\": %.3f, \"throttled_us\": %lld",
                    mode, nthreads, blocks, s / blocks * 1e6, blocks * kBlock / s / double(1 << 30), cpus,
                    cpus * s / blocks * 1e6, th0 < 0 || th1 < 0 ? -1ll : th1 - th0);
    };

    // single: one launch per block
    std::vector<hipStream_t> streams(nthreads);
    for (auto &s : streams) CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess);

    if (mixed_only) {
        // thread k's unaligned shape: an append of 4 MiB - off at block offset
        // off (its own file), payload skewed off 16-byte alignment
        std::vector<crc32c_plan *> uplans(nthreads);
        std::vector<int> skew(nthreads);
        for (int k = 0; k < nthreads; ++k) {
            const uint64_t off = 100 + 4099ull * uint64_t(k), len = kBlock - off;
            const int64_t np = crc32c_packetize(len, off, 65536, 512, nullptr, 0);
            CHECK(np > 0);
            std::vector<uint64_t> lens(static_cast<size_t>(np));
            CHECK(crc32c_packetize(len, off, 65536, 512, lens.data(), size_t(np)) == np);
            std::vector<crc32c_packet> up;
            uint64_t po = 0, oi = 0;
            for (uint64_t l : lens) {
                up.push_back(crc32c_packet{po, oi, uint32_t(l), 512u});
                po += l;
                oi += crc32c_nchunks(l, 512);
            }
            CHECK(oi <= nout);
            CHECK(crc32c_plan_create(ctx, up.data(), up.size(), 0, &uplans[k]) == 0);
            skew[k] = 1 + (k * 5) % 15;
        }
        // expected: block b of thread k, kind 0 (whole block) or 1 (its append)
        std::vector<std::vector<uint32_t>> want(2 * size_t(nbuf), std::vector<uint32_t>(nout));
        auto expect = [&](int b, int kind, int k) {
            std::vector<uint32_t> &w = want[2 * size_t(b) + size_t(kind)];
            // (on the launch stream: the streams are non-blocking, so a memset on
            // the null stream could land after the launch)
            CHECK(hipMemsetAsync(outs[b], 0, nout * 4, streams[0]) == hipSuccess);
            if (kind == 0)
                CHECK(crc32c_plan_exec(plan, bufs[b], outs[b], streams[0]) == 0);
            else
                CHECK(crc32c_plan_exec(uplans[k], bufs[b] + skew[k], outs[b], streams[0]) == 0);
            CHECK(hipStreamSynchronize(streams[0]) == hipSuccess);
            CHECK(hipMemcpy(w.data(), outs[b], nout * 4, hipMemcpyDeviceToHost) == hipSuccess);
        };
        const std::pair<bool, int> modes[3] = {{true, 1}, {true, 2}, {false, 2}};  // (resident, depth)
        for (const auto &md : modes) {
                const bool res = md.first;
                const int depth = md.second;
                for (int k = 0; k < nthreads; ++k)
                    for (int slot = 0; slot < depth; ++slot) {
                        const int b = depth * k + slot;
                        const int last = ((iters - 1 - slot) / depth) * depth + slot;  // last i of this slot
                        expect(b, last % 2, k);
                    }
                for (int w = 0; w < 2; ++w) {
                    for (int i = 0; i < nbuf; ++i) CHECK(hipMemset(outs[i], 0, nout * 4) == hipSuccess);
                    CHECK(hipDeviceSynchronize() == hipSuccess);
                    crc32c_blocks *q = nullptr;
                    if (res)
                        CHECK(crc32c_blocks_create_resident(plan, 2000, &q) == 0);
                    else
                        CHECK(crc32c_blocks_create(plan, max_blocks, window_us, &q) == 0);
                    const char *name = res ? (depth == 1 ? "rqueue_mixed" : "rqueue2_mixed") : "queue2_mixed";
                    run(name, [&](int k) {
                        std::vector<uint64_t> ring(depth);
                        for (int i = 0; i < iters; ++i) {
                            const int slot = i % depth;
                            if (i >= depth) CHECK(crc32c_block_wait(q, ring[slot]) == 0);
                            const int b = depth * k + slot;
                            if (i % 2 == 0)
                                CHECK(crc32c_block_submit(q, bufs[b], outs[b], &ring[slot]) == 0);
                            else
                                CHECK(crc32c_block_submit_plan(q, uplans[k], bufs[b] + skew[k], outs[b], &ring[slot]) == 0);
                            if (depth == 1) CHECK(crc32c_block_wait(q, ring[slot]) == 0);
                        }
                        if (depth > 1)
                            for (int i = std::max(0, iters - depth); i < iters; ++i)
                                CHECK(crc32c_block_wait(q, ring[i % depth]) == 0);
                    });
                    uint64_t launches = 0, blocks = 0;
                    CHECK(crc32c_blocks_stats(q, &launches, &blocks) == 0);
                    CHECK(crc32c_blocks_destroy(q) == 0);
                    // (the last block of each slot, over its own checksums: a slot
                    // that alternates shapes keeps the longer one's tail)
                    int bad = 0, bad_unaligned = 0;
                    std::vector<uint32_t> got(nout);
                    for (int k = 0; k < nthreads; ++k)
                        for (int slot = 0; slot < depth; ++slot) {
                            const int b = depth * k + slot;
                            const int last = ((iters - 1 - slot) / depth) * depth + slot;
                            const size_t nc = size_t(crc32c_plan_nchecksums(last % 2 ? uplans[k] : plan));
                            CHECK(hipMemcpy(got.data(), outs[b], nout * 4, hipMemcpyDeviceToHost) == hipSuccess);
                            const std::vector<uint32_t> &w = want[2 * size_t(b) + size_t(last % 2)];
                            const bool wrong = !std::equal(got.begin(), got.begin() + nc, w.begin());
                            bad += wrong;
                            bad_unaligned += wrong && (last % 2);
                            if (wrong) {  // (diagnostic: where, and the host's crc32c of that chunk)
                                size_t j = 0, nw = 0;
                                for (size_t x = 0; x < nc; ++x) nw += got[x] != w[x];
                                while (got[j] == w[j]) ++j;
                                const uint64_t off = 100 + 4099ull * uint64_t(k);
                                const size_t first = (last % 2) ? 512 - off % 512 : 512;
                                std::vector<uint8_t> chunk(j == 0 ? first : 512, uint8_t(b * 37 + 1));
                                std::fprintf(stderr, "wrong: mode %s depth %d thread %d slot %d kind %d: %zu of %zu checksums "
                                             "differ, first at %zu: got %08x want %08x host %08x\n",
                                             res ? "resident" : "queue", depth, k, slot, last % 2, nw, nc, j, got[j],
                                             w[j], crc32c(0, chunk.data(), chunk.size()));
                            }
                        }
                    std::printf(", \"launches\": %llu, \"unaligned_share\": 0.5, \"blocks_wrong\": %d, "
                                "\"wrong_unaligned\": %d, \"pass\": %d}\n",
                                (unsigned long long)launches, bad, bad_unaligned, w);
                }
            }
        for (crc32c_plan *u : uplans) crc32c_plan_destroy(u);
        crc32c_plan_destroy(plan);
        for (auto &s : streams) (void)hipStreamDestroy(s);
        return 0;
    }
    for (int w = 0; w < (sweep_only ? 0 : 2); ++w) {
        run("single", [&](int k) {
            for (int i = 0; i < iters; ++i) {
                CHECK(crc32c_plan_exec(plan, bufs[k], outs[k], streams[k]) == 0);
                CHECK(hipStreamSynchronize(streams[k]) == hipSuccess);
            }
        });
        std::printf(", \"pass\": %d}\n", w);
    }

    // queue (depth 1), queue2, queue4, ...: `depth` blocks in flight per
    // thread (submit the next, then wait for the oldest)
    for (int depth = 1; depth <= maxdepth; depth *= 2)
        for (int w = 0; w < 2; ++w) {
            crc32c_blocks *q = nullptr;
            CHECK(crc32c_blocks_create(plan, max_blocks, window_us, &q) == 0);
            char name[32];
            std::snprintf(name, sizeof name, depth == 1 ? "queue" : "queue%d", depth);
            uint64_t wc0 = 0, wc1 = 0;
            CHECK(crc32c_debug_blocks_worker_cpu_ns(q, &wc0) == 0);
            const Clock::time_point q0 = Clock::now();
            run(name, [&](int k) {
                if (depth == 1) {
                    for (int i = 0; i < iters; ++i) CHECK(crc32c_block_checksums(q, bufs[k], outs[k]) == 0);
                    return;
                }
                std::vector<uint64_t> ring(depth);
                for (int i = 0; i < iters; ++i) {
                    const int slot = i % depth;
                    if (i >= depth) CHECK(crc32c_block_wait(q, ring[slot]) == 0);
                    const int b = depth * k + slot;
                    CHECK(crc32c_block_submit(q, bufs[b], outs[b], &ring[slot]) == 0);
                }
                for (int i = std::max(0, iters - depth); i < iters; ++i) CHECK(crc32c_block_wait(q, ring[i % depth]) == 0);
            });
            CHECK(crc32c_debug_blocks_worker_cpu_ns(q, &wc1) == 0);
            const double qs = seconds(q0, Clock::now());
            uint64_t flushes = 0, blocks = 0;
            CHECK(crc32c_blocks_stats(q, &flushes, &blocks) == 0);
            std::printf(", \"max_blocks\": %u, \"window_us\": %u, \"launches\": %llu, \"blocks_per_launch\": %.2f, "
                        "\"worker_cpu_us_per_block\": %.3f, \"worker_busy\": %.2f, \"pass\": %d}\n",
                        max_blocks, window_us, (unsigned long long)flushes, double(blocks) / double(flushes ? flushes : 1),
                        double(wc1 - wc0) * 1e-3 / (double(nthreads) * iters), double(wc1 - wc0) * 1e-9 / qs, w);
            CHECK(crc32c_blocks_destroy(q) == 0);
        }
    // resident kernel: the product queue's resident mode
    // (crc32c_blocks_create_resident: rqueue, rqueue2) and the debug
    // library's A/B shapes (resident, resident2), depth 1 and 2; the outputs
    // are compared with the queue's (the last queue run wrote every buffer's)
    {
        std::vector<std::vector<uint32_t>> want(nbuf, std::vector<uint32_t>(nout));
        CHECK(hipDeviceSynchronize() == hipSuccess);
        for (int i = 0; i < nbuf; ++i) CHECK(hipMemcpy(want[i].data(), outs[i], nout * 4, hipMemcpyDeviceToHost) == hipSuccess);
        auto check_outs = [&](int depth) {
            int bad = 0;
            std::vector<uint32_t> got(nout);
            for (int k = 0; k < nthreads; ++k)
                for (int slot = 0; slot < depth; ++slot) {
                    const int b = depth * k + slot;
                    CHECK(hipMemcpy(got.data(), outs[b], nout * 4, hipMemcpyDeviceToHost) == hipSuccess);
                    bad += got != want[b];
                }
            return bad;
        };
        for (int depth = 1; depth <= std::min(maxdepth, 2); ++depth)
            for (int w = 0; w < 2; ++w) {
                for (int i = 0; i < nbuf; ++i) CHECK(hipMemset(outs[i], 0, nout * 4) == hipSuccess);
                CHECK(hipDeviceSynchronize() == hipSuccess);
                crc32c_blocks *q = nullptr;
                CHECK(crc32c_blocks_create_resident(plan, 2000, &q) == 0);
                run(depth == 1 ? "rqueue" : "rqueue2", [&](int k) {
                    if (depth == 1) {
                        for (int i = 0; i < iters; ++i) CHECK(crc32c_block_checksums(q, bufs[k], outs[k]) == 0);
                        return;
                    }
                    std::vector<uint64_t> ring(depth);
                    for (int i = 0; i < iters; ++i) {
                        const int slot = i % depth;
                        if (i >= depth) CHECK(crc32c_block_wait(q, ring[slot]) == 0);
                        const int b = depth * k + slot;
                        CHECK(crc32c_block_submit(q, bufs[b], outs[b], &ring[slot]) == 0);
                    }
                    for (int i = std::max(0, iters - depth); i < iters; ++i) CHECK(crc32c_block_wait(q, ring[i % depth]) == 0);
                });
                uint64_t launches = 0, blocks = 0;
                CHECK(crc32c_blocks_stats(q, &launches, &blocks) == 0);
                CHECK(crc32c_blocks_destroy(q) == 0);
                std::printf(", \"launches\": %llu, \"blocks_wrong\": %d, \"pass\": %d}\n", (unsigned long long)launches,
                            check_outs(depth), w);
            }
        for (int depth = 1; depth <= std::min(maxdepth, 2); ++depth)
            for (int w = 0; w < 2; ++w) {
                for (int i = 0; i < nbuf; ++i) CHECK(hipMemset(outs[i], 0, nout * 4) == hipSuccess);
                CHECK(hipDeviceSynchronize() == hipSuccess);
                crc32c_resident *r = nullptr;
                CHECK(crc32c_debug_resident_create(plan, 2000, &r) == 0);
                run(depth == 1 ? "resident" : "resident2", [&](int k) {
                    std::vector<uint64_t> ring(depth);
                    for (int i = 0; i < iters; ++i) {
                        const int slot = i % depth;
                        if (i >= depth) CHECK(crc32c_debug_resident_wait(r, ring[slot]) == 0);
                        const int b = depth * k + slot;
                        CHECK(crc32c_debug_resident_submit(r, bufs[b], outs[b], &ring[slot]) == 0);
                        if (depth == 1) CHECK(crc32c_debug_resident_wait(r, ring[slot]) == 0);
                    }
                    if (depth > 1)
                        for (int i = std::max(0, iters - depth); i < iters; ++i)
                            CHECK(crc32c_debug_resident_wait(r, ring[i % depth]) == 0);
                });
                uint64_t launches = 0;
                CHECK(crc32c_debug_resident_stats(r, &launches) == 0);
                std::string trace;
                if (const char *st = std::getenv("HDFS_CRC32C_RESIDENT_STAMPS"); st && st[0] == '1') {
                    // medians over the run's last tickets (ring of 4096), us (stamps: 100 MHz)
                    std::vector<uint64_t> stm(4 * 4096);
                    uint64_t rtt = 0, polls = 0;
                    CHECK(crc32c_debug_resident_trace(r, stm.data(), &rtt, &polls) == 0);
                    const uint64_t nt = uint64_t(nthreads) * iters, n = std::min<uint64_t>(nt, 4096);
                    std::vector<double> d[4];
                    for (uint64_t t = nt - n; t < nt; ++t) {
                        const uint64_t *x = &stm[4 * (t % 4096)];
                        if (!x[0] || !x[1] || !x[2] || !x[3]) continue;
                        d[0].push_back((double(x[1]) - double(x[0])) / 100.0);  // forwarded -> seen by a worker
                        d[1].push_back((double(x[2]) - double(x[1])) / 100.0);  // seen -> its tiles stored
                        d[2].push_back((double(x[3]) - double(x[2])) / 100.0);  // stored -> collected
                        d[3].push_back((double(x[3]) - double(x[0])) / 100.0);  // forwarded -> collected
                    }
                    auto med = [](std::vector<double> &v) {
                        if (v.empty()) return -1.0;
                        std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
                        return v[v.size() / 2];
                    };
                    char buf[512];
                    std::snprintf(buf, sizeof buf,
                                  ", \"trace_us\": {\"fwd_to_seen\": %.2f, \"seen_to_stored\": %.2f, "
                                  "\"stored_to_collected\": %.2f, \"fwd_to_collected\": %.2f, \"host_poll_rtt\": %.2f, "
                                  "\"tickets\": %zu}",
                                  med(d[0]), med(d[1]), med(d[2]), med(d[3]), polls ? double(rtt) / double(polls) / 100.0 : -1.0,
                                  d[3].size());
                    trace = buf;
                }
                CHECK(crc32c_debug_resident_destroy(r) == 0);
                int bad = 0;
                std::vector<uint32_t> got(nout);
                for (int k = 0; k < nthreads; ++k)
                    for (int slot = 0; slot < depth; ++slot) {
                        const int b = depth * k + slot;
                        CHECK(hipMemcpy(got.data(), outs[b], nout * 4, hipMemcpyDeviceToHost) == hipSuccess);
                        bad += got != want[b];
                    }
                std::printf(", \"launches\": %llu, \"blocks_wrong\": %d%s, \"pass\": %d}\n", (unsigned long long)launches,
                            bad, trace.c_str(), w);
            }
    }
    if (sweep_only) {
        crc32c_plan_destroy(plan);
        for (auto &s : streams) (void)hipStreamDestroy(s);
        return 0;
    }

    // one thread: submit max_blocks blocks, wait for the last (a flush cycle
    // with no thread hand-off), and the host's issue cost of one
    // crc32c_plan_exec_blocks call of max_blocks blocks
    {
        crc32c_blocks *q = nullptr;
        CHECK(crc32c_blocks_create(plan, max_blocks, window_us, &q) == 0);
        const uint32_t nb = std::min<uint32_t>(max_blocks, uint32_t(nbuf));
        const int cycles = 500;
        Clock::time_point t0 = Clock::now();
        for (int c = 0; c < cycles + 50; ++c) {
            if (c == 50) t0 = Clock::now();
            uint64_t t = 0;
            for (uint32_t b = 0; b < nb; ++b) CHECK(crc32c_block_submit(q, bufs[b], outs[b], &t) == 0);
            CHECK(crc32c_block_wait(q, t) == 0);
        }
        const double s = seconds(t0, Clock::now());
        std::printf("{\"mode\": \"queue_one_thread\", \"blocks_per_flush\": %u, \"us_per_cycle\": %.3f, "
                    "\"us_per_block\": %.3f}\n", nb, s / cycles * 1e6, s / cycles / nb * 1e6);
        CHECK(crc32c_blocks_destroy(q) == 0);
        const void *pays[32];
        uint32_t *os[32];
        for (uint32_t i = 0; i < nb && i < 32; ++i) pays[i] = bufs[i], os[i] = outs[i];
        hipStream_t s0 = streams[0];
        for (int i = 0; i < 50; ++i) CHECK(crc32c_plan_exec_blocks(plan, pays, os, nb, s0) == 0);
        CHECK(hipStreamSynchronize(s0) == hipSuccess);
        const int n = 200;
        t0 = Clock::now();
        for (int i = 0; i < n; ++i) CHECK(crc32c_plan_exec_blocks(plan, pays, os, nb, s0) == 0);
        const double issue = seconds(t0, Clock::now());
        CHECK(hipStreamSynchronize(s0) == hipSuccess);
        std::printf("{\"mode\": \"exec_blocks_issue\", \"blocks_per_launch\": %u, \"host_us_per_call\": %.3f}\n", nb,
                    issue / n * 1e6);
        // where a call's host time goes: the same loop over single calls
        // (in bursts of 4 calls on an idle stream, so a full queue's
        // back-pressure is not counted as issue cost)
        auto issue_cost = [&](const char *what, auto fn) {
            for (int i = 0; i < 50; ++i) fn();
            CHECK(hipStreamSynchronize(s0) == hipSuccess);
            double tot = 0;
            for (int r = 0; r < n / 4; ++r) {
                const auto a = Clock::now();
                for (int i = 0; i < 4; ++i) fn();
                tot += seconds(a, Clock::now());
                CHECK(hipStreamSynchronize(s0) == hipSuccess);
            }
            std::printf("{\"mode\": \"issue_cost\", \"call\": \"%s\", \"host_us\": %.3f}\n", what, tot / n * 1e6);
        };
        issue_cost("crc32c_plan_exec 1 block", [&] { CHECK(crc32c_plan_exec(plan, bufs[0], outs[0], s0) == 0); });
        issue_cost("crc32c_plan_exec_blocks 1", [&] { CHECK(crc32c_plan_exec_blocks(plan, pays, os, 1, s0) == 0); });
        issue_cost("crc32c_plan_exec_blocks 16", [&] { CHECK(crc32c_plan_exec_blocks(plan, pays, os, nb, s0) == 0); });
        hipEvent_t ev;
        CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess);
        issue_cost("hipEventRecord", [&] { CHECK(hipEventRecord(ev, s0) == hipSuccess); });
        issue_cost("hipStreamIsCapturing", [&] {
            hipStreamCaptureStatus cs;
            CHECK(hipStreamIsCapturing(s0, &cs) == hipSuccess);
        });
        issue_cost("hipThreadExchangeStreamCaptureMode x2", [&] {
            hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
            CHECK(hipThreadExchangeStreamCaptureMode(&m) == hipSuccess);
            CHECK(hipThreadExchangeStreamCaptureMode(&m) == hipSuccess);
        });
        issue_cost("hipEventQuery", [&] { (void)hipEventQuery(ev); });
        (void)hipEventDestroy(ev);
    }

    // pipelined: one thread keeps `depth` multi-block launches in flight on
    // one stream, each followed by an event it polls (hipEventQuery), and
    // launches the next batch when the oldest completes -- the queue
    // worker's loop without any other thread: the rate a single issuing
    // thread can sustain against the GPU's.
    for (int depth : {1, 2, 3}) {
        const uint32_t nb = std::min<uint32_t>(max_blocks, 32u);
        const uint32_t groups = std::max<uint32_t>(1u, uint32_t(nbuf) / nb);
        hipStream_t s = streams[0];
        std::vector<hipEvent_t> evs(depth);
        for (auto &e : evs) CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess);
        const void *pays[32];
        uint32_t *os[32];
        int issued = 0, done = 0;
        auto launch = [&] {
            const uint32_t g0 = (uint32_t(issued) % groups) * nb;
            for (uint32_t k = 0; k < nb; ++k) pays[k] = bufs[g0 + k], os[k] = outs[g0 + k];
            CHECK(crc32c_plan_exec_blocks(plan, pays, os, nb, s) == 0);
            CHECK(hipEventRecord(evs[issued % depth], s) == hipSuccess);
            issued++;
        };
        const int total = 1500, skip = 200;
        Clock::time_point t0 = Clock::now();
        while (done < total) {
            while (issued < total && issued - done < depth) launch();
            while (hipEventQuery(evs[done % depth]) == hipErrorNotReady) __builtin_ia32_pause();
            if (++done == skip) t0 = Clock::now();
        }
        const double sec = seconds(t0, Clock::now());
        std::printf("{\"mode\": \"pipelined\", \"depth\": %d, \"blocks_per_launch\": %u, \"us_per_launch\": %.3f, "
                    "\"us_per_block\": %.3f}\n",
                    depth, nb, sec / (total - skip) * 1e6, sec / (total - skip) / nb * 1e6);
        for (auto &e : evs) (void)hipEventDestroy(e);
    }

    // kernel: the GPU's time per block in back-to-back multi-block launches
    // (kernel: the same nb buffers every launch -- nb x 4 MiB may stay in
    // the 256 MiB last-level cache; kernel_rotating: consecutive launches
    // take the next nb of all nbuf buffers, as the queue modes do)
    for (int rot = 0; rot < 2; ++rot)
    for (uint32_t nb : {1u, 4u, 8u, 16u, 32u}) {
        if (nb > uint32_t(nbuf)) break;
        hipStream_t s = streams[0];
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess);
        const void *pays[32];
        uint32_t *os[32];
        const uint32_t groups = rot ? std::max<uint32_t>(1u, uint32_t(nbuf) / nb) : 1u;
        auto launch = [&](int i) {
            const uint32_t g0 = (uint32_t(i) % groups) * nb;
            for (uint32_t k = 0; k < nb; ++k) pays[k] = bufs[g0 + k], os[k] = outs[g0 + k];
            CHECK(crc32c_plan_exec_blocks(plan, pays, os, nb, s) == 0);
        };
        for (int i = 0; i < 200; ++i) launch(i);
        const int n = 1000;
        CHECK(hipEventRecord(e0, s) == hipSuccess);
        for (int i = 0; i < n; ++i) launch(i);
        CHECK(hipEventRecord(e1, s) == hipSuccess);
        CHECK(hipStreamSynchronize(s) == hipSuccess);
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1) == hipSuccess);
        std::printf("{\"mode\": \"%s\", \"blocks_per_launch\": %u, \"bytes_rotated\": %llu, \"us_per_launch\": %.3f, "
                    "\"us_per_block\": %.3f}\n",
                    rot ? "kernel_rotating" : "kernel", nb, (unsigned long long)groups * nb * kBlock, ms * 1e3 / n,
                    ms * 1e3 / n / nb);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
    crc32c_plan_destroy(plan);  // (before the streams it was launched on)
    for (auto &s : streams) (void)hipStreamDestroy(s);
    for (int i = 0; i < nbuf; ++i) {
        (void)hipFree(bufs[i]);
        (void)hipFree(outs[i]);
    }
    crc32c_ctx_destroy(ctx);
    return 0;
}
