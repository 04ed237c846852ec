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
//   tools/launch_rate write [iterations=2000]
//   tools/launch_rate raw [launches=4000]   (an empty kernel: HIP's own launch cost)
// prints one JSON line.  `write`: one FUSE-shaped 4 MiB block write per
// iteration (TRUNCATE / NULLPADDING / THEDATA / TRAILINGDATA buffers,
// src/fuse.c:1348-1354) through crc32c_plan_create_buffers -> exec ->
// stream sync -> destroy: the per-write host cost of the buffer-list path.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "hdfs_crc32c.h"

#define CHECK(x)                                                           \
    do {                                                                   \
        if (!(x)) {                                                        \
            std::fprintf(stderr, "launch_rate: %s failed (line %d)\n", #x, __LINE__); \
            return 1;                                                      \
        }                                                                  \
    } while (0)

// An empty kernel with a KParams-sized argument, on the production grid
// shape: HIP's own launch cost, for comparison with crc32c_plan_exec's.
struct BigArg {
    uint64_t w[24];
};
__global__ void empty_kernel(BigArg a) {
    if (a.w[0] == 12345u && threadIdx.x == 1000) a.w[1] = 0;  // (never true; keeps the argument live)
}

static int raw_mode(int n) {
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess);
    BigArg a{};
    for (int i = 0; i < 500; ++i) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(768), 0, s, a);
    CHECK(hipStreamSynchronize(s) == hipSuccess);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess);
    CHECK(hipEventRecord(e0, s) == hipSuccess);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(768), 0, s, a);
    const auto t1 = std::chrono::steady_clock::now();
    CHECK(hipEventRecord(e1, s) == hipSuccess);
    CHECK(hipStreamSynchronize(s) == hipSuccess);
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1) == hipSuccess);
    std::printf("{\"mode\": \"raw_empty_kernel\", \"launches\": %d, \"host_issue_us\": %.3f, "
                "\"gpu_us_per_launch\": %.3f}\n",
                n, std::chrono::duration<double, std::micro>(t1 - t0).count() / n, ms * 1e3 / n);
    return 0;
}

static int write_mode(int iters) {
    const uint64_t mb4 = 4u << 20;
    crc32c_ctx *ctx = nullptr;
    CHECK(crc32c_ctx_create(0, &ctx) == 0);
    uint8_t *d = nullptr;
    uint32_t *out = nullptr;
    CHECK(hipMalloc(reinterpret_cast<void **>(&d), mb4 + 64) == hipSuccess);
    CHECK(hipMemset(d, 0x3c, mb4 + 64) == hipSuccess);
    CHECK(hipMalloc(reinterpret_cast<void **>(&out), 8192 * 4) == hipSuccess);
    const crc32c_buffer bufs[4] = {{d, 100000}, {nullptr, 300000}, {d + 400000, 3000000},
                                   {d + 3400017, mb4 - 3400000}};
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess);
    double t_create = 0, t_exec = 0, t_sync = 0, t_destroy = 0;
    for (int it = -50; it < iters; ++it) {
        const auto a = std::chrono::steady_clock::now();
        crc32c_plan *plan = nullptr;
        CHECK(crc32c_plan_create_buffers(ctx, bufs, 4, 0, mb4, 0, 65536, 512, 0, &plan) == 0);
        const auto b = std::chrono::steady_clock::now();
        CHECK(crc32c_plan_exec(plan, nullptr, out, s) == 0);
        const auto c = std::chrono::steady_clock::now();
        CHECK(hipStreamSynchronize(s) == hipSuccess);
        const auto e = std::chrono::steady_clock::now();
        CHECK(crc32c_plan_destroy(plan) == 0);
        const auto f = std::chrono::steady_clock::now();
        if (it < 0) continue;
        t_create += std::chrono::duration<double, std::micro>(b - a).count();
        t_exec += std::chrono::duration<double, std::micro>(c - b).count();
        t_sync += std::chrono::duration<double, std::micro>(e - c).count();
        t_destroy += std::chrono::duration<double, std::micro>(f - e).count();
    }
    // the HIP calls a plan's life is made of, alone (16 KiB of descriptors)
    double t_malloc = 0, t_free = 0, t_copy = 0, t_copy_async = 0;
    std::vector<uint8_t> host(16384, 1);
    uint8_t *pinned = nullptr;
    CHECK(hipHostMalloc(reinterpret_cast<void **>(&pinned), 16384, 0) == hipSuccess);
    for (int it = 0; it < 200; ++it) {
        const auto a = std::chrono::steady_clock::now();
        void *x = nullptr;
        CHECK(hipMalloc(&x, 16384) == hipSuccess);
        const auto b = std::chrono::steady_clock::now();
        CHECK(hipMemcpy(x, host.data(), 16384, hipMemcpyHostToDevice) == hipSuccess);
        const auto c = std::chrono::steady_clock::now();
        CHECK(hipMemcpyAsync(x, pinned, 16384, hipMemcpyHostToDevice, s) == hipSuccess);
        const auto e = std::chrono::steady_clock::now();
        CHECK(hipStreamSynchronize(s) == hipSuccess);
        const auto f = std::chrono::steady_clock::now();
        CHECK(hipFree(x) == hipSuccess);
        const auto g = std::chrono::steady_clock::now();
        t_malloc += std::chrono::duration<double, std::micro>(b - a).count();
        t_copy += std::chrono::duration<double, std::micro>(c - b).count();
        t_copy_async += std::chrono::duration<double, std::micro>(e - c).count();
        t_free += std::chrono::duration<double, std::micro>(g - f).count();
    }
    (void)hipHostFree(pinned);
    std::printf("{\"mode\": \"write\", \"iterations\": %d, \"create_us\": %.2f, \"exec_issue_us\": %.2f, "
                "\"sync_us\": %.2f, \"destroy_us\": %.2f, \"total_us\": %.2f, \"hipMalloc_16KiB_us\": %.2f, "
                "\"hipMemcpy_pageable_16KiB_us\": %.2f, \"hipMemcpyAsync_pinned_issue_us\": %.2f, "
                "\"hipFree_us\": %.2f}\n",
                iters, t_create / iters, t_exec / iters, t_sync / iters, t_destroy / iters,
                (t_create + t_exec + t_sync + t_destroy) / iters, t_malloc / 200, t_copy / 200, t_copy_async / 200,
                t_free / 200);
    (void)hipFree(d);
    (void)hipFree(out);
    crc32c_ctx_destroy(ctx);
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 1 && std::string(argv[1]) == "write") return write_mode(argc > 2 ? std::atoi(argv[2]) : 2000);
    if (argc > 1 && std::string(argv[1]) == "raw") return raw_mode(argc > 2 ? std::atoi(argv[2]) : 4000);
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
