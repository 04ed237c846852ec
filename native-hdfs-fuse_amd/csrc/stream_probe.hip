// stream_probe.hip -- DIAGNOSTIC: achievable HBM read bandwidth on this
// device for a few plain streaming-read shapes, to price the CRC kernel's
// roofline against what the chip actually delivers.  Not on the product path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hdfs_crc32c_debug.h"

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

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
        for (int u = 0; u < UNROLL; ++u) v[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) {
        const u32x4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[tid] = acc;
}

}  // namespace

extern "C" int crc32c_debug_stream_probe(const void *dev_src, uint64_t bytes, uint32_t *dev_out, uint32_t grid,
                                         int shape, void *stream) {
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t n16 = bytes / 16;
    switch (shape) {
    case 0: hipLaunchKernelGGL((probe_read<4, false>), dim3(grid), dim3(256), 0, s, (const u32x4 *)dev_src, n16, dev_out); break;
    case 1: hipLaunchKernelGGL((probe_read<8, false>), dim3(grid), dim3(256), 0, s, (const u32x4 *)dev_src, n16, dev_out); break;
    case 2: hipLaunchKernelGGL((probe_read<4, true>), dim3(grid), dim3(256), 0, s, (const u32x4 *)dev_src, n16, dev_out); break;
    default: hipLaunchKernelGGL((probe_read<16, false>), dim3(grid), dim3(256), 0, s, (const u32x4 *)dev_src, n16, dev_out); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
