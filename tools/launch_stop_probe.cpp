// launch_stop_probe.cpp -- diagnostic: what a completion event costs a launch.
// One small kernel (a 256-workgroup store of one word each), launched back to
// back on one stream in three ways:
//   plain      -- hipLaunchKernelGGL
//   stop       -- hipExtLaunchKernelGGL with a stop event (the dispatch
//                 completes the event; no separate command)
//   record     -- hipLaunchKernelGGL, then hipEventRecord of an event
// For each: host issue time per call (bursts of 4 on an idle stream) and the
// GPU's time per launch over 2000 back-to-back launches (timing events
// around them).  Prints one JSON line per way.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
    do {                                                                              \
        if ((x) != hipSuccess) {                                                      \
            std::fprintf(stderr, "launch_stop_probe: %s failed (line %d)\n", #x, __LINE__); \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

__global__ void touch(uint32_t *p) {
    if (threadIdx.x == 0) p[blockIdx.x] = blockIdx.x;
}

int main() {
    std::setvbuf(stdout, nullptr, _IOLBF, 0);
    uint32_t *d = nullptr;
    CHECK(hipMalloc(&d, 4096));
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev_nt, ev_t, e0, e1;
    CHECK(hipEventCreateWithFlags(&ev_nt, hipEventDisableTiming));
    CHECK(hipEventCreate(&ev_t));
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const dim3 g(256), b(64);
    struct Way {
        const char *name;
        int kind;
        hipEvent_t ev;
    } ways[] = {{"plain", 0, nullptr},      {"stop_timing", 1, ev_t}, {"stop_disable_timing", 1, ev_nt},
                {"record_disable_timing", 2, ev_nt}, {"plain_again", 0, nullptr}};
    for (const Way &w : ways) {
        auto one = [&] {
            if (w.kind == 1) {
                hipExtLaunchKernelGGL(touch, g, b, 0, s, nullptr, w.ev, 0u, d);
            } else {
                hipLaunchKernelGGL(touch, g, b, 0, s, d);
                if (w.kind == 2) CHECK(hipEventRecord(w.ev, s));
            }
        };
        for (int i = 0; i < 200; ++i) one();
        CHECK(hipStreamSynchronize(s));
        double host = 0;
        const int bursts = 250;
        for (int r = 0; r < bursts; ++r) {
            const auto a = std::chrono::steady_clock::now();
            for (int i = 0; i < 4; ++i) one();
            host += std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
            CHECK(hipStreamSynchronize(s));
        }
        const int n = 2000;
        CHECK(hipEventRecord(e0, s));
        for (int i = 0; i < n; ++i) one();
        CHECK(hipEventRecord(e1, s));
        CHECK(hipStreamSynchronize(s));
        CHECK(hipGetLastError());
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"way\": \"%s\", \"host_us_per_call\": %.3f, \"gpu_us_per_launch\": %.3f}\n", w.name,
                    host / (bursts * 4) * 1e6, ms * 1e3 / n);
    }
    CHECK(hipStreamDestroy(s));
    CHECK(hipFree(d));
    return 0;
}
