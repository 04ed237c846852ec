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
//   tools/launch_rate calls [packets=64] [launches=4000]
// prints one JSON line.  `calls`: per call kind on the same plan, host issue
// time and GPU time per launch -- exec, verify (crc32c_plan_verify), verify
// with a mismatch bitmap (crc32c_plan_verify_bitmap), exec followed by a
// hipEventRecord of a timing-disabled event (the price of a completion record
// per launch), exec + hipStreamIsCapturing.
//   tools/launch_rate rtt [launches=2000]
// one launch then a wait for it, back to back (submit -> complete latency of
// a single writer): an empty kernel with hipStreamSynchronize, the plan of
// one 4 MiB block with hipStreamSynchronize, and the same with a spin on
// hipEventQuery of a stop event instead of the blocking synchronise.
//   tools/launch_rate multi [packets=256] [steps=2000]
// config 4's per-rank step at N = 8 on one GPU (a 16 MiB shard = 4 blocks of
// 64 packets): crc32c_plan_exec of the shard, crc32c_multi_plan_exec in place
// (no RCCL call) and with CRC32C_MULTI_SELF_SEND (the shard's checksums
// through one RCCL send/recv group, as a peer's gather), each host-issued and
// replayed from a HIP graph of 100 steps (kernels + RCCL group captured).  `write`: one FUSE-shaped 4 MiB block write per
// iteration (TRUNCATE / NULLPADDING / THEDATA / TRAILINGDATA buffers,
// src/fuse.c:1348-1354) through crc32c_plan_create_buffers -> exec ->
// stream sync -> destroy: the per-write host cost of the buffer-list path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "hdfs_crc32c.h"

// (internal, exported by the library: a multi-block launch whose last kernel
// completes `stop` -- hipExtLaunchKernel's stop event; diagnostic use only)
struct ihipStream_t;
struct ihipEvent_t;
namespace hdfs_crc {
int exec_blocks(crc32c_plan *plan, const void *const *dev_payloads, uint32_t *const *dev_outs, size_t nblocks,
                hipStream_t stream, hipEvent_t stop);
}

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

// One call kind timed like main's exec loop: warm-up, then n calls between
// two events; host issue time and GPU time per call.
template <class F>
static int time_calls(const char *name, hipStream_t s, int n, F call, bool first) {
    for (int i = 0; i < 300; ++i)
        if (call(i)) return 1;
    if (hipStreamSynchronize(s) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess);
    CHECK(hipEventRecord(e0, s) == hipSuccess);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i)
        if (call(i)) return 1;
    const auto t1 = std::chrono::steady_clock::now();
    CHECK(hipEventRecord(e1, s) == hipSuccess);
    CHECK(hipStreamSynchronize(s) == hipSuccess);
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1) == hipSuccess);
    std::printf("%s\"%s\": {\"host_issue_us\": %.3f, \"gpu_us_per_launch\": %.3f}", first ? "" : ", ", name,
                std::chrono::duration<double, std::micro>(t1 - t0).count() / n, ms * 1e3 / n);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return 0;
}

// Does a stop event per launch cost more the longer it runs?  exec (the
// plan's mark as the stop event), verify, exec again, then multi-block
// launches of one block with no stop event the library sees... (every
// plan launch now completes the plan's mark), with one reused stop event,
// and with a ring of 8 stop events.
static int stopev_mode(size_t npk, int n) {
    const uint32_t len = 65536, bpc = 512;
    std::vector<crc32c_packet> pk(npk);
    for (size_t i = 0; i < npk; ++i) pk[i] = crc32c_packet{uint64_t(i) * len, uint64_t(i) * (len / bpc), len, bpc};
    crc32c_ctx *ctx = nullptr;
    CHECK(crc32c_ctx_create(0, &ctx) == 0);
    crc32c_plan *plan = nullptr;
    CHECK(crc32c_plan_create(ctx, pk.data(), npk, 0, &plan) == 0);
    const size_t bytes = npk * len, nsums = npk * (len / bpc);
    void *src = nullptr;
    uint32_t *dst = nullptr, *res = nullptr;
    CHECK(hipMalloc(&src, bytes) == hipSuccess);
    CHECK(hipMemset(src, 0x5a, bytes) == hipSuccess);
    CHECK(hipMalloc(reinterpret_cast<void **>(&dst), nsums * 4) == hipSuccess);
    CHECK(hipMalloc(reinterpret_cast<void **>(&res), 64) == hipSuccess);
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess);
    CHECK(crc32c_plan_exec(plan, src, dst, s) == 0);
    hipEvent_t ring[8];
    for (auto &e : ring) CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess);
    const void *pays[1] = {src};
    uint32_t *os[1] = {dst};
    std::printf("{\"mode\": \"stopev\", \"packets\": %zu, \"launches\": %d, ", npk, n);
    int rc = time_calls("exec_1", s, n, [&](int) { return crc32c_plan_exec(plan, src, dst, s); }, true);
    rc = rc || time_calls("verify", s, n, [&](int) { return crc32c_plan_verify(plan, src, dst, res, s); }, false);
    rc = rc || time_calls("exec_2", s, n, [&](int) { return crc32c_plan_exec(plan, src, dst, s); }, false);
    rc = rc || time_calls("blocks_stop_one", s, n, [&](int) { return hdfs_crc::exec_blocks(plan, pays, os, 1, s, ring[0]); },
                          false);
    rc = rc || time_calls("blocks_stop_ring8", s, n,
                          [&](int i) { return hdfs_crc::exec_blocks(plan, pays, os, 1, s, ring[i & 7]); }, false);
    rc = rc || time_calls("exec_3", s, n, [&](int) { return crc32c_plan_exec(plan, src, dst, s); }, false);
    std::printf("}\n");
    for (auto &e : ring) (void)hipEventDestroy(e);
    (void)hipFree(src);
    (void)hipFree(dst);
    (void)hipFree(res);
    crc32c_plan_destroy(plan);
    crc32c_ctx_destroy(ctx);
    (void)hipStreamDestroy(s);
    return rc;
}

static int calls_mode(size_t npk, int n) {
    const uint32_t len = 65536, bpc = 512;
    std::vector<crc32c_packet> pk(npk);
    for (size_t i = 0; i < npk; ++i) pk[i] = crc32c_packet{uint64_t(i) * len, uint64_t(i) * (len / bpc), len, bpc};
    crc32c_ctx *ctx = nullptr;
    CHECK(crc32c_ctx_create(0, &ctx) == 0);
    crc32c_plan *plan = nullptr;
    CHECK(crc32c_plan_create(ctx, pk.data(), npk, 0, &plan) == 0);
    const size_t bytes = npk * len, nsums = npk * (len / bpc);
    void *src = nullptr;
    uint32_t *dst = nullptr, *res = nullptr, *bits = nullptr;
    CHECK(hipMalloc(&src, bytes) == hipSuccess);
    CHECK(hipMemset(src, 0x5a, bytes) == hipSuccess);
    CHECK(hipMalloc(reinterpret_cast<void **>(&dst), nsums * 4) == hipSuccess);
    CHECK(hipMalloc(reinterpret_cast<void **>(&res), 64) == hipSuccess);
    CHECK(hipMalloc(reinterpret_cast<void **>(&bits), (nsums + 31) / 32 * 4) == hipSuccess);
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess);
    CHECK(crc32c_plan_exec(plan, src, dst, s) == 0);  // expected values for the verifies
    hipEvent_t ev;
    CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess);
    std::printf("{\"mode\": \"calls\", \"packets\": %zu, \"launches\": %d, ", npk, n);
    int rc = time_calls("exec", s, n, [&](int) { return crc32c_plan_exec(plan, src, dst + 0, s); }, true);
    rc = rc || time_calls("verify", s, n, [&](int) { return crc32c_plan_verify(plan, src, dst, res, s); }, false);
    rc = rc || time_calls("verify_bitmap", s, n,
                          [&](int) { return crc32c_plan_verify_bitmap(plan, src, dst, res, bits, s); }, false);
    rc = rc || time_calls("exec_event_record", s, n, [&](int) {
             return crc32c_plan_exec(plan, src, dst, s) || hipEventRecord(ev, s) != hipSuccess;
         }, false);
    const void *pays[1] = {src};
    uint32_t *os[1] = {dst};
    rc = rc || time_calls("exec_blocks1", s, n, [&](int) { return hdfs_crc::exec_blocks(plan, pays, os, 1, s, nullptr); },
                          false);
    rc = rc || time_calls("exec_blocks1_stop_event", s, n,
                          [&](int) { return hdfs_crc::exec_blocks(plan, pays, os, 1, s, ev); }, false);
    rc = rc || time_calls("exec_is_capturing", s, n, [&](int) {
             hipStreamCaptureStatus cs;
             return crc32c_plan_exec(plan, src, dst, s) || hipStreamIsCapturing(s, &cs) != hipSuccess;
         }, false);
    uint32_t host_res[2] = {1, 1};
    CHECK(hipMemcpy(host_res, res, 8, hipMemcpyDeviceToHost) == hipSuccess);
    std::printf(", \"verify_clean\": %s}\n", (host_res[0] == 0 && host_res[1] == 0xFFFFFFFFu) ? "true" : "false");
    (void)hipEventDestroy(ev);
    (void)hipFree(src);
    (void)hipFree(dst);
    (void)hipFree(res);
    (void)hipFree(bits);
    crc32c_plan_destroy(plan);
    crc32c_ctx_destroy(ctx);
    return rc;
}

// Host-issued and graph-replayed time per step of `step` on stream s.
template <class F>
static int time_step(const char *name, hipStream_t s, int n, F step) {
    for (int i = 0; i < 200; ++i)
        if (step()) return 1;
    CHECK(hipStreamSynchronize(s) == hipSuccess);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess);
    CHECK(hipEventRecord(e0, s) == hipSuccess);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i)
        if (step()) return 1;
    const auto t1 = std::chrono::steady_clock::now();
    CHECK(hipEventRecord(e1, s) == hipSuccess);
    CHECK(hipStreamSynchronize(s) == hipSuccess);
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1) == hipSuccess);
    const double issue = std::chrono::duration<double, std::micro>(t1 - t0).count() / n, eager = ms * 1e3 / n;
    // the same steps captured into one graph (100 steps) and replayed
    const int per = 100, reps = std::max(1, n / per);
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) == hipSuccess);
    int rc = 0;
    for (int i = 0; i < per && !rc; ++i) rc = step();
    const hipError_t ce = hipStreamEndCapture(s, &g);
    if (rc || ce != hipSuccess || hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) {
        std::printf("\"%s\": {\"host_issue_us\": %.3f, \"eager_us\": %.3f, \"graph\": \"capture failed (rc %d, %d)\"}, ",
                    name, issue, eager, rc, int(ce));
        (void)hipGetLastError();
        return 0;
    }
    CHECK(hipGraphLaunch(ge, s) == hipSuccess);
    CHECK(hipStreamSynchronize(s) == hipSuccess);
    CHECK(hipEventRecord(e0, s) == hipSuccess);
    for (int r = 0; r < reps; ++r) CHECK(hipGraphLaunch(ge, s) == hipSuccess);
    CHECK(hipEventRecord(e1, s) == hipSuccess);
    CHECK(hipStreamSynchronize(s) == hipSuccess);
    CHECK(hipEventElapsedTime(&ms, e0, e1) == hipSuccess);
    std::printf("\"%s\": {\"host_issue_us\": %.3f, \"eager_us\": %.3f, \"graph_us\": %.3f}, ", name, issue, eager,
                ms * 1e3 / (reps * per));
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return 0;
}

static int multi_mode(size_t npk, int n) {
    const uint32_t len = 65536, bpc = 512;
    std::vector<crc32c_packet> pk(npk);
    for (size_t i = 0; i < npk; ++i) pk[i] = crc32c_packet{uint64_t(i) * len, uint64_t(i) * (len / bpc), len, bpc};
    const size_t bytes = npk * len, nsums = npk * (len / bpc);
    void *src = nullptr;
    uint32_t *out = nullptr;
    CHECK(hipMalloc(&src, bytes + 64) == hipSuccess);
    CHECK(hipMemset(src, 0x3c, bytes + 64) == hipSuccess);
    CHECK(hipMalloc(reinterpret_cast<void **>(&out), nsums * 4) == hipSuccess);
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess);
    std::printf("{\"mode\": \"multi\", \"packets\": %zu, \"steps\": %d, ", npk, n);
    crc32c_ctx *ctx = nullptr;
    CHECK(crc32c_ctx_create(0, &ctx) == 0);
    crc32c_plan *plan = nullptr;
    CHECK(crc32c_plan_create(ctx, pk.data(), npk, 0, &plan) == 0);
    CHECK(crc32c_plan_exec(plan, src, out, s) == 0);
    if (time_step("shard_plan_exec", s, n, [&] { return crc32c_plan_exec(plan, src, out, s); })) return 1;
    std::vector<uint32_t> want(nsums), got(nsums);
    CHECK(hipStreamSynchronize(s) == hipSuccess);
    CHECK(hipMemcpy(want.data(), out, nsums * 4, hipMemcpyDeviceToHost) == hipSuccess);
    crc32c_plan_destroy(plan);
    crc32c_ctx_destroy(ctx);
    bool exact = true;
    for (uint32_t flags : {0u, CRC32C_MULTI_SELF_SEND}) {
        crc32c_multi *m = nullptr;
        const int dev = 0;
        CHECK(crc32c_multi_create(&dev, 1, &m) == 0);
        crc32c_multi_plan *mp = nullptr;
        CHECK(crc32c_multi_plan_create(m, pk.data(), npk, 64, flags, &mp) == 0);
        const void *shards[1] = {src};
        void *streams[1] = {s};
        CHECK(hipMemset(out, 0, nsums * 4) == hipSuccess);
        CHECK(crc32c_multi_plan_exec(mp, shards, out, streams) == 0);  // (creates the communicator)
        CHECK(hipStreamSynchronize(s) == hipSuccess);
        CHECK(hipMemcpy(got.data(), out, nsums * 4, hipMemcpyDeviceToHost) == hipSuccess);
        exact = exact && got == want;
        if (time_step(flags ? "multi_self_send" : "multi_in_place", s, n,
                      [&] { return crc32c_multi_plan_exec(mp, shards, out, streams); }))
            return 1;
        CHECK(hipStreamSynchronize(s) == hipSuccess);
        CHECK(hipMemcpy(got.data(), out, nsums * 4, hipMemcpyDeviceToHost) == hipSuccess);
        exact = exact && got == want;
        crc32c_multi_plan_destroy(mp);
        crc32c_multi_destroy(m);
    }
    std::printf("\"exact\": %s}\n", exact ? "true" : "false");
    (void)hipFree(src);
    (void)hipFree(out);
    return exact ? 0 : 1;
}

static int rtt_mode(int n) {
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess);
    BigArg a{};
    auto per = [&](auto fn) {
        for (int i = 0; i < 100; ++i)
            if (fn()) return -1.0;
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < n; ++i)
            if (fn()) return -1.0;
        return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
    };
    const double empty = per([&] {
        hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(768), 0, s, a);
        return hipStreamSynchronize(s) != hipSuccess;
    });
    const uint32_t len = 65536, bpc = 512;
    std::vector<crc32c_packet> pk(64);
    for (size_t i = 0; i < 64; ++i) pk[i] = crc32c_packet{uint64_t(i) * len, uint64_t(i) * (len / bpc), len, bpc};
    crc32c_ctx *ctx = nullptr;
    CHECK(crc32c_ctx_create(0, &ctx) == 0);
    crc32c_plan *plan = nullptr;
    CHECK(crc32c_plan_create(ctx, pk.data(), 64, 0, &plan) == 0);
    void *src = nullptr;
    uint32_t *dst = nullptr;
    CHECK(hipMalloc(&src, 64 * len) == hipSuccess);
    CHECK(hipMemset(src, 0x11, 64 * len) == hipSuccess);
    CHECK(hipMalloc(reinterpret_cast<void **>(&dst), 64 * 128 * 4) == hipSuccess);
    const double block_sync = per([&] {
        return crc32c_plan_exec(plan, src, dst, s) || hipStreamSynchronize(s) != hipSuccess;
    });
    hipEvent_t ev;
    CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess);
    const void *pays[1] = {src};
    uint32_t *os[1] = {dst};
    const double block_spin = per([&] {
        if (hdfs_crc::exec_blocks(plan, pays, os, 1, s, ev)) return true;
        hipError_t q;
        while ((q = hipEventQuery(ev)) == hipErrorNotReady) __builtin_ia32_pause();
        return q != hipSuccess;
    });
    std::printf("{\"mode\": \"rtt\", \"launches\": %d, \"empty_kernel_sync_us\": %.3f, \"block_exec_sync_us\": %.3f, "
                "\"block_exec_event_spin_us\": %.3f}\n",
                n, empty, block_sync, block_spin);
    (void)hipEventDestroy(ev);
    (void)hipFree(src);
    (void)hipFree(dst);
    crc32c_plan_destroy(plan);
    crc32c_ctx_destroy(ctx);
    (void)hipStreamDestroy(s);
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 1 && std::string(argv[1]) == "write") return write_mode(argc > 2 ? std::atoi(argv[2]) : 2000);
    if (argc > 1 && std::string(argv[1]) == "raw") return raw_mode(argc > 2 ? std::atoi(argv[2]) : 4000);
    if (argc > 1 && std::string(argv[1]) == "stopev")
        return stopev_mode(argc > 2 ? std::strtoul(argv[2], nullptr, 10) : 64, argc > 3 ? std::atoi(argv[3]) : 4000);
    if (argc > 1 && std::string(argv[1]) == "rtt") return rtt_mode(argc > 2 ? std::atoi(argv[2]) : 2000);
    if (argc > 1 && std::string(argv[1]) == "multi")
        return multi_mode(argc > 2 ? std::strtoul(argv[2], nullptr, 10) : 256, argc > 3 ? std::atoi(argv[3]) : 2000);
    if (argc > 1 && std::string(argv[1]) == "calls")
        return calls_mode(argc > 2 ? std::strtoul(argv[2], nullptr, 10) : 64, argc > 3 ? std::atoi(argv[3]) : 4000);
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
