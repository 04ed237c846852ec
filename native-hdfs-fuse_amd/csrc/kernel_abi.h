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
    // Verification (crc32c_plan_verify): compare with expect[] instead of
    // storing to out[]; the last workgroup writes result[0] = mismatches,
    // result[1] = min bad index.
    const uint32_t *expect;
    uint32_t *result;
    // Scheduler slot of this launch (kSlotWords u32s, see below) and the
    // other slot of the pair, which this launch resets for the next one.
    uint32_t *sched;
    uint32_t *sched_next;
    uint32_t nheads;  // dynamic scheduler heads in use (<= kMaxHeads)
    uint32_t static_tiles;  // scheduler-wave variants: tiles [0, static_tiles) are split statically
    uint32_t ring_target;   // scheduler-wave variants: tiles queued ahead before the next grab
    uint32_t grab_unit;     // scheduler-wave variants: tiles per lane per grab
};

// Device scratch of one launch ("slot"), u32 words.  Launches of one plan
// (or one host-pipeline stage) alternate between two slots and are
// serialised on the GPU, so a launch may reset the slot its predecessor used.
//   heads: up to kMaxHeads tile counters of the dynamic scheduler, 8 KiB
//          apart so they do not share a memory channel's atomic unit; 0 at
//          launch start;
//   ticket / vcount / vfirst: verification's grid-wide merge; 0 / 0 / ~0 at
//          launch start, restored by the launch's last workgroup.
constexpr uint32_t kMaxHeads = 32;
constexpr uint32_t kHeadStride = 17408;  // 68 KiB: heads spread over memory channels
constexpr uint32_t kTicketWord = kMaxHeads * kHeadStride;
constexpr uint32_t kVCountWord = kTicketWord + 32;
constexpr uint32_t kVFirstWord = kTicketWord + 64;
constexpr uint32_t kSlotWords = kTicketWord + 96;

// Fills two slots' initial state (2 * kSlotWords words).
inline void init_sched_slots(uint32_t *w) {
    for (uint32_t i = 0; i < 2 * kSlotWords; ++i) w[i] = 0;
    w[kVFirstWord] = 0xffffffffu;
    w[kSlotWords + kVFirstWord] = 0xffffffffu;
}

// Kernel variants; 0 is the production kernel, the others stay built for
// A/B measurement and diagnostics (tools/kbench.py, tools/stamps.py).
struct KernelVariant {
    const char *name;
    uint32_t threads;
    uint32_t wg_per_cu;
    uint32_t heads = 0;  // dynamic scheduler heads (0: static tile ranges, no scheduler slots)
    uint32_t static_pct = 0;  // scheduler-wave variants: share of the tiles split statically
    uint32_t ring_target = 20;
    uint32_t grab_unit = 2;
};
constexpr int kNumVariants = 50;
// Variants whose verification mode is built (crc32c_plan_verify).
inline bool variant_verifies(int v) { return v == 0 || v == 1 || v == 21 || v == 22; }
extern const KernelVariant kVariants[kNumVariants];

// Persistent grid: min(work items / waves per workgroup, wg_per_cu * CUs) of the variant.
hipError_t launch_plan_kernel(const KParams &p, int variant, uint32_t num_cu, hipStream_t stream);

}  // namespace hdfs_crc
