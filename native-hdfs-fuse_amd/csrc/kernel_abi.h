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
// After the S4 image (at kTableAllocS4): the compact S4 image (crc_math.h
// kS4C*), padded to whole 1 KiB staging pieces.
constexpr uint32_t kS4COff = kTableAllocS4;
constexpr uint32_t kTableAllocS4C = ((uint32_t(kS4CBytes) + 16384 - 1) / 16384) * 16384;
// After it (at kZeroCrcOff): crc(0, zeros(n)) for n = 0 .. kZeroCrcMax
// (crc_math.h zero_crc_table), read by general items with scalar loads.
constexpr uint32_t kZeroCrcOff = kS4COff + kTableAllocS4C;
constexpr uint32_t kTableAllocS4Full = kZeroCrcOff + ((4 * (kZeroCrcMax + 1) + 16384 - 1) / 16384) * 16384;

// One block of a multi-block launch (crc32c_plan_exec_blocks): the plan's
// work items describe one block's shape; block b's copy of item i reads at
// payload + src_i + payload_delta and writes out[out_i + out_delta].
struct BlockRef {
    uint64_t payload_delta;
    uint32_t out_delta;
    uint32_t reserved;
};
// Blocks one launch carries (in the kernel arguments: 16 B each).
constexpr uint32_t kMaxLaunchBlocks = 32;

constexpr uint32_t kGeneralItems = 1u, kGeneralShift = 2u, kGeneralHalf = 4u, kGeneralPadded = 8u;  // KParams::general

struct KParams {
    const FastTile *tiles;  // power-of-two and general tiles
    const GenItem *gen;
    const SegItem *seg;
    const GenPiece *pieces;  // SegItem pieces
    const ConstRun *consts;
    const uint8_t *payload;
    uint32_t *out;
    const uint8_t *table;     // kLdsBytes: the nibble image (A/B variant 1)
    const uint8_t *table_s4;  // kS4Bytes: the slicing-by-4 image (production)
    uint32_t ntiles;
    uint32_t ngen;
    uint32_t nseg;
    uint32_t nconst;
    uint32_t general;  // kGeneralItems: tiles[] holds general tiles; kGeneralShift: some tile is off 16-byte
                       // alignment; kGeneralHalf: half tiles; kGeneralPadded: padded power-of-two tiles (each
                       // selects a build that has that code)
    uint32_t skip_z;   // 1: no item shifts by Z^(512 s): the S4 images are staged without their Z section
    uint32_t flags;
    uint32_t c_lg[5];
    uint32_t c_small[4];
    uint64_t *stamps;  // diagnostic variants only: 4 x u64 per wave
    // Verification (crc32c_plan_verify): compare with expect[] instead of
    // storing to out[]; the last workgroup writes result[0] = mismatches,
    // result[1] = min bad index.
    const uint32_t *expect;
    uint32_t *result;
    // Optional (crc32c_plan_verify_bitmap): bit i set for every mismatching
    // checksum i; its bad_words u32s are zeroed by workgroup 0 of the launch
    // itself before it publishes the launch key (crc32c_device.h verify_init).
    uint32_t *bad_bits;
    uint32_t bad_words;
    // Verification slot of this launch (kSlotWords u32s): the key of the
    // launch that initialised p.result.
    uint32_t *sched;
    // The plan's completion counters (kDoneCtrs u64s, kDoneCtrStride bytes
    // apart), or null (launches that are not a plan's): the last wave of
    // every workgroup adds 1 to counter blockIdx % kDoneCtrs.
    unsigned long long *done_ctr;
    // Multi-block launch: nblocks > 0 runs the plan's block_tiles tiles once
    // per block (tile j = block j / block_tiles, tile j % block_tiles); the
    // plan has tiles only.  0: an ordinary launch.
    uint32_t nblocks;
    uint32_t block_tiles;
    BlockRef blocks[kMaxLaunchBlocks];
};

// Device state of verification launches ("slot", kSlotWords u32s, one
// 128-B line): the 64-bit key of the launch that last initialised its
// result (kernel: launch_key, from the dispatch packet's address and the
// queue's dispatch id -- unique per launch, graph replays included).
// Workgroup 0 of a verification launch writes {0, ~0} to p.result and then
// its key; a workgroup with mismatches waits for the key before it adds to
// the result, and a clean workgroup touches neither (no grid-wide ticket).
// Launches sharing a slot run in GPU order (a plan's verify launches).
constexpr uint32_t kEpochWord = 0;  // u64
constexpr uint32_t kSlotWords = 32;

// A plan's completion counters (crc32c_plan_destroy without touching the
// launch streams): in the plan's device block after its verify slot,
// kDoneCtrs u64 counters kDoneCtrStride bytes apart (one per XCD's
// workgroups: workgroup b runs on XCD b % 8), zero at upload.  The last wave
// of every workgroup of a plan launch adds 1 (a non-returning device-scope
// atomic, after every read of the plan's memory); the host counts the
// workgroups it launched, so a destroyed plan's block is reusable once the
// counters sum to that (read back on the context's upload stream).
constexpr uint32_t kDoneCtrOff = 256;
constexpr uint32_t kDoneCtrs = 8;
constexpr uint32_t kDoneCtrStride = 128;
constexpr uint32_t kPlanHeadBytes = kDoneCtrOff + kDoneCtrs * kDoneCtrStride;  // the work items follow

// A plan's block shape as the resident kernel reads it (resident_engine.h):
// at kResShapeOff of the plan's device block, between the verify slot and
// the completion counters, written with the items at upload.  A block
// submitted to a resident queue names its plan's record in its ring slot.
struct ResShape {
    const FastTile *tiles;  // power-of-two tiles (offsets from the block's payload)
    const GenItem *gen;     // general chunks (a trimmed first packet, packet tails)
    uint32_t ntiles, ngen;
    uint32_t simple;  // 1: every tile 16-byte aligned from the block start, no GenItem
    uint32_t pad;
};
constexpr uint32_t kResShapeOff = 128;
static_assert(kSlotWords * sizeof(uint32_t) <= kResShapeOff && kResShapeOff + sizeof(ResShape) <= kDoneCtrOff,
              "the shape record sits between the verify slot and the counters");

// Fills a slot's initial state (kSlotWords words): no launch's key.
inline void init_sched_slots(uint32_t *w) {
    for (uint32_t i = 0; i < kSlotWords; ++i) w[i] = 0;
    w[kEpochWord] = w[kEpochWord + 1] = 0xffffffffu;
}

// The production kernel (crc32c_kernel.hip): one 12-wave workgroup per CU,
// min(work items, CUs) of them; p.expect selects the verification mode.
// `stop` (optional): an event the launch itself completes (hipExtLaunchKernel's
// stop event -- no extra command on the stream, unlike an hipEventRecord).
// `grid` (optional): the workgroups launched.
hipError_t launch_plan_kernel(const KParams &p, uint32_t num_cu, hipStream_t stream, hipEvent_t stop = nullptr,
                              uint32_t *grid = nullptr);
// Loads the production kernels' code object onto the current device.
hipError_t preload_plan_kernels();

}  // namespace hdfs_crc
