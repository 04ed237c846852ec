// launch_rate.cpp -- diagnostic: how fast a C caller issues plan launches.
//
// The FUSE write path (src/fuse.c:580-647) checksums one 4 MiB block per
// write_block call; a C caller of this library does that as one
// crc32c_plan_exec per block.  This program times N back-to-back
// crc32c_plan_exec calls on one plan of P packets of 64 KiB from C++ (no
// Python): the host's issue time per call and the GPU's time per launch
// (hipEvents around the N launches), device-resident payload.
//
//   tools/launch_rate [packets=64] [launches=4000]
// prints one JSON line.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "hdfs_crc32c.h"

#define CHECK(x)                                                           \
    do {                                                                   \
        if (!(x)) {                                                        \
            std::fprintf(stderr, "launch_rate: %s failed (line %d)\n", #x, __LINE__); \
            return 1;                                                      \
        }                                                                  \
    } while (0)

int main(int argc, char **argv) {
    const size_t npk = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 64;
    const int n = argc > 2 ? std::atoi(argv[2]) : 4000;
    const uint32_t len = 65536, bpc = 512;
    std::vector<crc32c_packet> pk(npk);
    for (size_t i = 0; i < npk; ++i) {
        pk[i].payload_off = uint64_t(i) * len;
        pk[i].out_idx = uint64_t(i) * (len / bpc);
        pk[i].len = len;
        pk[i].bpc = bpc;
    }
    crc32c_ctx *ctx = nullptr;
    CHECK(crc32c_ctx_create(0, &ctx) == 0);
    crc32c_plan *plan = nullptr;
    CHECK(crc32c_plan_create(ctx, pk.data(), npk, 0, &plan) == 0);
    const size_t bytes = npk * len, nsums = npk * (len / bpc);
    const int nbuf = 4;
    std::vector<void *> src(nbuf), dst(nbuf);
    for (int b = 0; b < nbuf; ++b) {
        CHECK(hipMalloc(&src[b], bytes) == hipSuccess);
        CHECK(hipMemset(src[b], 0x5a + b, bytes) == hipSuccess);
        CHECK(hipMalloc(&dst[b], nsums * 4) == hipSuccess);
    }
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess);
    for (int i = 0; i < 500; ++i)
        CHECK(crc32c_plan_exec(plan, src[i % nbuf], static_cast<uint32_t *>(dst[i % nbuf]), s) == 0);
    CHECK(hipStreamSynchronize(s) == hipSuccess);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess);
    CHECK(hipEventRecord(e0, s) == hipSuccess);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i)
        CHECK(crc32c_plan_exec(plan, src[i % nbuf], static_cast<uint32_t *>(dst[i % nbuf]), s) == 0);
    const auto t1 = std::chrono::steady_clock::now();
    CHECK(hipEventRecord(e1, s) == hipSuccess);
    CHECK(hipStreamSynchronize(s) == hipSuccess);
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1) == hipSuccess);
    const double issue_us = std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
    std::printf("{\"packets\": %zu, \"launches\": %d, \"host_issue_us\": %.3f, \"gpu_us_per_launch\": %.3f, "
                "\"gib_s\": %.1f}\n",
                npk, n, issue_us, ms * 1e3 / n, double(bytes) * n / (ms * 1e-3) / (1u << 30));
    for (int b = 0; b < nbuf; ++b) {
        (void)hipFree(src[b]);
        (void)hipFree(dst[b]);
    }
    crc32c_plan_destroy(plan);
    crc32c_ctx_destroy(ctx);
    return 0;
}
