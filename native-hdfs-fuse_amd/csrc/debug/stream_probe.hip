// stream_probe.hip -- DIAGNOSTIC: achievable HBM read bandwidth on this
// device for a few plain streaming-read shapes, to price the CRC kernel's
// roofline against what the chip actually delivers.  Not on the product path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hdfs_crc32c_debug.h"

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u32x4 *p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}

// Grid-stride read of 16 B per lane, UNROLL loads in flight per lane,
// XOR-folded so nothing is dead; one dword per thread written at the end.
template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void probe_read(const u32x4 *__restrict__ src, uint64_t n16, uint32_t *out) {
    const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    uint32_t acc = 0;
    uint64_t i = tid;
    for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = ld16<NT>(src + i + u * stride);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) {
        const u32x4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[tid] = acc;
}

// Tile-shaped reads like the CRC kernel's: a wave reads one tile of UNROLL
// consecutive KiB (one 1 KiB wave instruction each).  RANGE: every workgroup
// owns an equal contiguous range of tiles and its waves take them round-
// robin; otherwise the chip's waves take tiles grid-stride.
template <int THREADS, int UNROLL, bool RANGE>
__global__ __launch_bounds__(THREADS) void probe_tiles(const u32x4 *__restrict__ src, uint64_t bytes, uint32_t *out) {
    constexpr uint32_t kWaves = THREADS / 64;
    constexpr uint64_t kTile = 1024ull * UNROLL;
    const uint64_t ntiles = bytes / kTile;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint64_t t, tend, step;
    if (RANGE) {
        t = ntiles * blockIdx.x / gridDim.x + wv;
        tend = ntiles * (blockIdx.x + 1) / gridDim.x;
        step = kWaves;
    } else {
        t = uint64_t(blockIdx.x) * kWaves + wv;
        tend = ntiles;
        step = uint64_t(gridDim.x) * kWaves;
    }
    uint32_t acc = 0;
    for (; t < tend; t += step) {
        const u32x4 *p = src + t * (kTile / 16) + lane;
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = __builtin_nontemporal_load(p + 64 * u);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    out[blockIdx.x * THREADS + threadIdx.x] = acc;
}

// Tile reads handed out dynamically: each wave takes GRAB consecutive 8 KiB
// tiles per atomicAdd on one device counter (DYN) or the same tiles in the
// same per-wave order statically (grid-stride over groups of GRAB tiles), so
// the two differ only in who decides the order.
template <int GRAB, bool DYN>
__global__ __launch_bounds__(1024) void probe_dyn(const u32x4 *__restrict__ src, uint64_t bytes, uint32_t *out,
                                                  uint32_t *ctr) {
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t ngroups = bytes / (8192ull * GRAB);
    const uint64_t nw = uint64_t(gridDim.x) * 16;
    uint64_t g = uint64_t(blockIdx.x) * 16 + wv;
    uint32_t acc = 0;
    for (;;) {
        if (DYN) {
            uint32_t t = 0;
            if (lane == 0) t = atomicAdd(ctr, 1u);
            g = __builtin_amdgcn_readfirstlane(t);
        }
        if (g >= ngroups) break;
        for (int k = 0; k < GRAB; ++k) {
            const u32x4 *p = src + (g * GRAB + k) * 512 + lane;
            u32x4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(p + 64 * u);
#pragma unroll
            for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        }
        if (!DYN) g += nw;
    }
    out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

}  // namespace

// shape: 0-3 grid-stride (256 threads; unroll 4 / 8 / 4 nt / 16);
// 4-7 grid-stride nt, unroll 2 / 8 / 16 / 1;
// 8-15 tile probes, 1024 threads: 8 KiB tiles range / stride, 4 KiB range /
// stride, then 512 threads: 8 KiB range / stride, 4 KiB range / stride.
extern "C" int crc32c_debug_stream_probe(const void *dev_src, uint64_t bytes, uint32_t *dev_out, uint32_t grid,
                                         int shape, void *stream) {
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t n16 = bytes / 16;
    const u32x4 *src = (const u32x4 *)dev_src;
    switch (shape) {
    case 0: hipLaunchKernelGGL((probe_read<4, false>), dim3(grid), dim3(256), 0, s, src, n16, dev_out); break;
    case 1: hipLaunchKernelGGL((probe_read<8, false>), dim3(grid), dim3(256), 0, s, src, n16, dev_out); break;
    case 2: hipLaunchKernelGGL((probe_read<4, true>), dim3(grid), dim3(256), 0, s, src, n16, dev_out); break;
    case 3: hipLaunchKernelGGL((probe_read<16, false>), dim3(grid), dim3(256), 0, s, src, n16, dev_out); break;
    case 4: hipLaunchKernelGGL((probe_read<2, true>), dim3(grid), dim3(256), 0, s, src, n16, dev_out); break;
    case 5: hipLaunchKernelGGL((probe_read<8, true>), dim3(grid), dim3(256), 0, s, src, n16, dev_out); break;
    case 6: hipLaunchKernelGGL((probe_read<16, true>), dim3(grid), dim3(256), 0, s, src, n16, dev_out); break;
    case 7: hipLaunchKernelGGL((probe_read<1, true>), dim3(grid), dim3(256), 0, s, src, n16, dev_out); break;
    case 8: hipLaunchKernelGGL((probe_tiles<1024, 8, true>), dim3(grid), dim3(1024), 0, s, src, bytes, dev_out); break;
    case 9: hipLaunchKernelGGL((probe_tiles<1024, 8, false>), dim3(grid), dim3(1024), 0, s, src, bytes, dev_out); break;
    case 10: hipLaunchKernelGGL((probe_tiles<1024, 4, true>), dim3(grid), dim3(1024), 0, s, src, bytes, dev_out); break;
    case 11: hipLaunchKernelGGL((probe_tiles<1024, 4, false>), dim3(grid), dim3(1024), 0, s, src, bytes, dev_out); break;
    case 12: hipLaunchKernelGGL((probe_tiles<512, 8, true>), dim3(grid), dim3(512), 0, s, src, bytes, dev_out); break;
    case 13: hipLaunchKernelGGL((probe_tiles<512, 8, false>), dim3(grid), dim3(512), 0, s, src, bytes, dev_out); break;
    case 14: hipLaunchKernelGGL((probe_tiles<512, 4, true>), dim3(grid), dim3(512), 0, s, src, bytes, dev_out); break;
    case 15: hipLaunchKernelGGL((probe_tiles<512, 4, false>), dim3(grid), dim3(512), 0, s, src, bytes, dev_out); break;
    case 16:
    case 17:
    case 18:
    case 19: {
        // the counter lives past the per-thread outputs (grid <= 256 here)
        uint32_t *ctr = dev_out + (1u << 20) - 64;
        if (grid > 256) return -22;
        if (hipMemsetAsync(ctr, 0, 4, s) != hipSuccess) return -5;
        if (shape == 16) hipLaunchKernelGGL((probe_dyn<1, true>), dim3(grid), dim3(1024), 0, s, src, bytes, dev_out, ctr);
        if (shape == 17) hipLaunchKernelGGL((probe_dyn<1, false>), dim3(grid), dim3(1024), 0, s, src, bytes, dev_out, ctr);
        if (shape == 18) hipLaunchKernelGGL((probe_dyn<4, true>), dim3(grid), dim3(1024), 0, s, src, bytes, dev_out, ctr);
        if (shape == 19) hipLaunchKernelGGL((probe_dyn<4, false>), dim3(grid), dim3(1024), 0, s, src, bytes, dev_out, ctr);
        break;
    }
    default: return -22;
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
