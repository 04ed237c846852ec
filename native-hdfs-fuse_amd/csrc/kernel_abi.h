// kernel_abi.h -- what the host runtime hands the CRC32C kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc_math.h"
#include "plan.h"

namespace hdfs_crc {

constexpr uint32_t kKernelLdsBytes = uint32_t(kLdsBytes);
constexpr uint32_t kKernelShiftOff = uint32_t(kLdsShiftOff);
// Device copy of the LDS image, zero-padded so every staging load of a
// 1024-thread workgroup (16 B per thread per round) is in bounds.
constexpr uint32_t kTableAlloc = ((kKernelLdsBytes + 16384 - 1) / 16384) * 16384;
// S4 device image: the LDS image (staged by LDS-DMA, rounded up to 1 KiB),
// then the byte tables T0..T3 once more in compact form (4 x 256 dwords) for
// the fast-staging variant, which replicates them over the lane columns with
// LDS writes instead of copying all 32 replicas from L2.
constexpr uint32_t kS4CompactOff = ((uint32_t(kS4Bytes) + 1023u) / 1024u) * 1024u;
constexpr uint32_t kTableAllocS4 = ((kS4CompactOff + 4096u + 16384u - 1u) / 16384u) * 16384u;

struct KParams {
    const FastTile *tiles;
    const GenItem *gen;
    const uint8_t *payload;
    uint32_t *out;
    const uint8_t *table;  // kLdsBytes, staged into LDS by every workgroup
    const uint8_t *table_s4;  // kS4Bytes: the slicing-by-4 variants' image
    uint32_t ntiles;
    uint32_t ngen;
    uint32_t flags;
    uint32_t c_lg[5];
    uint32_t c_small[4];
    uint64_t *stamps;  // diagnostic variant only: 4 x u64 per wave
};

// Kernel variants; 0 is the production kernel, the others stay built for
// A/B measurement and diagnostics (tools/kbench.py, tools/stamps.py).
struct KernelVariant {
    const char *name;
    uint32_t threads;
    uint32_t wg_per_cu;
};
constexpr int kNumVariants = 25;
extern const KernelVariant kVariants[kNumVariants];

// Persistent grid: min(work items / waves per workgroup, wg_per_cu * CUs) of the variant.
hipError_t launch_plan_kernel(const KParams &p, int variant, uint32_t num_cu, hipStream_t stream);

}  // namespace hdfs_crc
