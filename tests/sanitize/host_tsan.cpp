// ThreadSanitizer run of the host runtime's threaded code (TEST
// INFRASTRUCTURE): the staging copies' worker threads and their piece
// hand-off to the H2D queue (host_copy.h, used by crc32c_batch_host on
// pageable payloads), the lazily initialised CPU dispatcher and tables
// (crc32c(), crc32c_chunks_cpu -- libfuse calls them from many worker
// threads, fuse.c:1771), and concurrent plan building / framing / frame
// parsing.  Built with -fsanitize=thread and run by
// tests/test_host_sanitize.py; any data race aborts the run.  The GPU-side
// objects (contexts, plans) serialise on their own mutexes and are covered by
// the GPU suite's threaded test.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "crc_math.h"
#include "hdfs_crc32c.h"
#include "host_copy.h"
#include "plan.h"

extern "C" {
uint32_t oracle_crc32c_bytewise(uint32_t crc, const void *buf, size_t len);
// frames.cpp verifies through the GPU runtime, not part of this host build.
int64_t crc32c_verify_host(crc32c_ctx *, const void *, const crc32c_packet *, size_t, const uint32_t *, uint32_t,
                           uint64_t *) {
    return -19;
}
}

namespace {

std::mutex g_mu;
int g_fail = 0;
void failf(const char *what) {
    std::lock_guard<std::mutex> l(g_mu);
    std::fprintf(stderr, "FAIL: %s\n", what);
    ++g_fail;
}

void staging_copies() {
    const size_t n = (48u << 20) + 12345;  // above the 8 MiB threading threshold, ragged end
    std::vector<uint8_t> src(n), dst(n, 0);
    for (size_t i = 0; i < n; ++i) src[i] = uint8_t(i * 2654435761u >> 13);
    for (int rep = 0; rep < 3; ++rep) {
        std::fill(dst.begin(), dst.end(), 0);
        size_t seen = 0;
        // ready() runs on the calling thread once every copier's share of a
        // piece is in: it reads the whole piece, as the H2D copy would.
        hdfs_crc::copy_range_pipelined(dst.data(), src.data(), n, 8u << 20, [&](size_t off, size_t len) {
            if (off != seen || std::memcmp(dst.data() + off, src.data() + off, len) != 0) failf("pipelined piece");
            seen += len;
        });
        if (seen != n) failf("pipelined total");
        std::fill(dst.begin(), dst.end(), 0);
        hdfs_crc::copy_range(dst.data(), src.data(), n);
        if (std::memcmp(dst.data(), src.data(), n) != 0) failf("copy_range");
    }
    // gather of scattered packets (the batch_host gather path)
    std::vector<size_t> offs;
    for (size_t o = 0; o + 70000 < n; o += 70000 + 333) offs.push_back(o);
    std::vector<uint8_t> g(offs.size() * 70000);
    hdfs_crc::parallel_copy(offs.size(), g.size(), [&](size_t b, size_t e) {
        for (size_t k = b; k < e; ++k) std::memcpy(g.data() + k * 70000, src.data() + offs[k], 70000);
    });
    for (size_t k = 0; k < offs.size(); ++k)
        if (std::memcmp(g.data() + k * 70000, src.data() + offs[k], 70000) != 0) failf("gather");
}

// Many threads hit the lazily initialised paths at once.
void concurrent_host_calls() {
    std::vector<uint8_t> buf(200000);
    for (size_t i = 0; i < buf.size(); ++i) buf[i] = uint8_t(i * 31 + 7);
    const uint32_t want = oracle_crc32c_bytewise(0, buf.data(), buf.size());
    std::vector<std::thread> th;
    for (int t = 0; t < 12; ++t)
        th.emplace_back([&, t] {
            if (crc32c(0, buf.data(), buf.size()) != want) failf("crc32c");
            std::vector<uint32_t> out(400);
            if (crc32c_chunks_cpu(buf.data(), buf.size(), 512, out.data(), t & 1 ? CRC32C_BIG_ENDIAN : 0) != 0)
                failf("chunks_cpu");
            (void)hdfs_crc32(0, buf.data(), 1000);
            hdfs_crc::HostPlan hp;
            std::vector<crc32c_packet> pk(64);
            for (size_t i = 0; i < pk.size(); ++i) pk[i] = crc32c_packet{i * 65536 + t, i * 100, 65536, 512u + 500u * (i % 3)};
            if (hdfs_crc::build_plan(pk.data(), pk.size(), &hp) != 0) failf("build_plan");
            const crc32c_buffer bufs[3] = {{buf.data(), 1000}, {nullptr, 5000 + uint64_t(t)}, {buf.data() + 7, 90000}};
            hdfs_crc::HostPlan wp;
            if (hdfs_crc::build_write_plan(bufs, 3, 3, 90000, 100, 65536, 512, t & 1 ? hdfs_crc::kPoly : hdfs_crc::kPolyIeee,
                                           &wp) != 0)
                failf("build_write_plan");
            std::vector<uint32_t> sums(6400, 0x01020304u);
            std::vector<uint8_t> fr(crc32c_frame_packets(pk.data(), pk.size(), sums.data(), 0, 0, 0, 4, nullptr, 0, nullptr));
            crc32c_frame_packets(pk.data(), pk.size(), sums.data(), 0, 0, 0, 4, fr.data(), fr.size(), nullptr);
            uint64_t used = 0;
            (void)crc32c_parse_frames(fr.data(), fr.size(), nullptr, 0, &used);
            uint8_t md5[16];
            crc32c_block_md5(sums.data(), sums.size(), 0, md5);
        });
    for (auto &x : th) x.join();
}

}  // namespace

int main() {
    setenv("HDFS_CRC32C_COPY_THREADS", "8", 1);
    staging_copies();
    concurrent_host_calls();
    if (g_fail) {
        std::fprintf(stderr, "%d failures\n", g_fail);
        return 1;
    }
    std::printf("host tsan run clean\n");
    return 0;
}
