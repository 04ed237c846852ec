// kernel_abi.h -- what the host runtime hands the CRC32C kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc_math.h"
#include "plan.h"

namespace hdfs_crc {

constexpr uint32_t kKernelLdsBytes = uint32_t(kLdsBytes);
constexpr uint32_t kKernelShiftOff = uint32_t(kLdsShiftOff);
constexpr uint32_t kKernelWgPerCu = 2;  // 2 x 73 KiB of LDS per CU
// Device copy of the LDS image, zero-padded so every staging load of a
// 1024-thread workgroup (16 B per thread per round) is in bounds.
constexpr uint32_t kTableAlloc = ((kKernelLdsBytes + 16384 - 1) / 16384) * 16384;
constexpr uint32_t kTableAllocS4 = ((uint32_t(kS4Bytes) + 16384 - 1) / 16384) * 16384;

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
    uint32_t *queue;       // tail-queue variants: this launch's LaunchSlot (zero on entry)
    uint32_t *queue_next;  // the slot the launch kQueueSlots / 2 later gets: zeroed by this launch
    uint32_t static_tiles; // tail-queue variants: tiles [0, static_tiles) are dealt statically
    uint32_t chunk_shift;  // tail-queue variants: tail chunk = 1 << chunk_shift tiles
    uint32_t tail_steal;   // tail-queue variants: 1 = steal from other XCDs' heads once the own one is drained
};

// Tail queue (see crc32c_kernel.hip): per-launch counters, one per XCD, each
// on its own 128-byte line (word x at queue[32 x]).  A launch finds its slot
// zeroed (hipMemset at context creation, then the launch kQueueSlots / 2
// earlier on the context, which clears it as a side job).
constexpr uint32_t kSlotWords = 8;
struct LaunchSlot {
    uint32_t w[kSlotWords * 32];
};
constexpr uint32_t kQueueSlots = 64;

// Kernel variants; 0 is the production kernel, the others stay built for
// A/B measurement and diagnostics (tools/kbench.py, tools/stamps.py).
struct KernelVariant {
    const char *name;
    uint32_t threads;
    uint32_t wg_per_cu;
};
constexpr int kNumVariants = 29;
extern const KernelVariant kVariants[kNumVariants];

// Persistent grid: min(work items / waves per workgroup, kKernelWgPerCu * CUs).
hipError_t launch_plan_kernel(const KParams &p, int variant, uint32_t num_cu, hipStream_t stream);

}  // namespace hdfs_crc
