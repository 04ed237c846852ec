// crc32c_device.h -- device code of the CDNA4 (gfx950) CRC32C chunk kernel.
//
// Included by crc32c_kernel.hip (the production instantiations, in
// libhdfs_crc32c.so) and by debug/crc32c_variants.hip (A/B and diagnostic
// instantiations, only in libhdfs_crc32c_debug.so).
//
// Computes hadoop_rpc_send_packet's checksum vector (hadooprpc.c:733-742:
// crc32c(0, chunk) per bytesPerChecksum chunk, crc32c.c semantics) for a
// whole batch of device-resident packets in one launch.  Integer/bitwise
// work, HBM-bound; no MFMA.  Design (DESIGN.md has the derivation and the
// measurements behind each choice):
//
//  * CRC32C is affine over GF(2): for a chunk M of n bytes,
//      crc32c(0, M) = lin(M) ^ crc32c(0, zeros(n)),
//    and lin(M) is the XOR of one 32-bit contribution per (byte position,
//    byte value).  So there is no serial dependency inside a chunk.
//  * Coalesced HBM loads: one wave instruction reads 1 KiB contiguous
//    (16 B per lane) = two 512-byte blocks; lane q of each half owns bytes
//    16q .. 16q+15 of its block in EVERY instruction.  Loads are
//    non-temporal buffer loads bounded by the tile (partial tiles read zeros).
//  * Lookups, production (kModeS4): each lane chains its 16-byte piece
//    d0..d3 through the slicing-by-4 step S (crc32c.c's crc32c_table[0..3],
//    one 4-byte column per lane so the 32 lanes of a half-wave always hit 32
//    different banks): u = S(S(S(d0) ^ d1) ^ d2) ^ d3, then one column-
//    specific operator N_q = Z_{16(31-q)} o S (8 nibble lookups) moves the
//    piece's contribution to the block end.  20 LDS lookups + 37 VALU per
//    16 bytes; 152 KiB of LDS, one workgroup per CU, 12 waves (768 threads).
//  * Wave-level reduction: each lane's per-piece value is XOR-reduced over
//    the 32 lanes of its block with a DPP reduce-scatter, which also packs
//    the 16 block results of a tile into 16 lanes for one coalesced store.
//  * bpc = 1024..8192 (power of two): per-block results are shifted by
//    Z^(512*s) (nibble tables in LDS) and XORed across the blocks of a chunk
//    with DPP / swizzle steps.
//  * Any other bpc in [4, 8192], and packet tails (general items,
//    crc32c_general.h): each chunk is right-aligned into k = ceil(bpc / 512)
//    virtual blocks (leading zeros do not change lin; the bytes before a
//    chunk in its first block are masked off), crc = lin ^ crc(0, zeros(n))
//    from a table; one wave runs an item's blocks as 16-block subtiles
//    (chunks may span two), shifting blocks by Z^(512*s) and gathering a
//    chunk's blocks with a prefix XOR.
//  * Tiles off 16-byte alignment (general builds): aligned loads, each
//    lane's bytes reassembled with a DPP wave shift and v_alignbyte.
//  * Work distribution: each workgroup owns an equal range of 8 KiB tiles;
//    its waves pull tiles from an LDS counter (the SIMD arbiter's age
//    priority makes static per-wave assignment finish 2x apart).  The
//    smallest batches split each tile over 4 waves (quarter units).
//  * Chunks fitting no tile (crc32c_items.h): half a wave per chunk
//    (GenItem), the chunk right-aligned into zero-prefixed virtual 512-byte
//    blocks, Horner-combined with Z^512.  Chunks assembled from several
//    buffers (SegItem) are read piece by piece into the same windows; chunks
//    of zero fill only (ConstRun) are written from plan-time constants.
//  * Verification (crc32c_plan_verify): the same kernel compares instead of
//    storing; the expected values are fetched with the tile and the last
//    workgroup 0 initialises the result; only mismatching workgroups add to it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernel_abi.h"

namespace hdfs_crc_dev {

using hdfs_crc::ConstRun;
using hdfs_crc::FastTile;
using hdfs_crc::GenItem;
using hdfs_crc::GenPiece;
using hdfs_crc::KParams;
using hdfs_crc::SegItem;
using hdfs_crc::kGeneralTile;
using hdfs_crc::kEpochWord;

constexpr uint32_t kLdsBytes = hdfs_crc::kKernelLdsBytes;
constexpr uint32_t kShiftOff = hdfs_crc::kKernelShiftOff;
// Table bytes copied into LDS, rounded up to whole 1 KiB LDS-DMA pieces (the
// device copy is zero-padded to kTableAlloc >= this).
constexpr uint32_t kStageBytes = (kLdsBytes + 1023u) / 1024u * 1024u;
static_assert(kStageBytes <= hdfs_crc::kTableAlloc, "staging reads past the device table");
// The slicing-by-4 kernel's image (crc_math.h): byte tables, N_q, shifts.
constexpr uint32_t kS4Bytes = uint32_t(hdfs_crc::kS4Bytes);
constexpr uint32_t kS4NibOff = uint32_t(hdfs_crc::kS4NibOff);
constexpr uint32_t kS4ShiftOff = uint32_t(hdfs_crc::kS4ShiftOff);
constexpr uint32_t kS4StageBytes = (kS4Bytes + 1023u) / 1024u * 1024u;
static_assert(kS4StageBytes <= hdfs_crc::kTableAllocS4, "staging reads past the device table");

// Kernel modes (template bits).  Production = kModeS4 | kModeNt (+ kModeVerify).
constexpr int kModeNt = 1;          // payload loads non-temporal (streamed once)
constexpr int kModeS4 = 2;          // slicing-by-4 chains + per-column finishing operator (S4 image)
constexpr int kModeStamps = 4;      // DIAGNOSTIC: per-wave timestamps
constexpr int kModeMemDiag = 8;     // DIAGNOSTIC, wrong results: no lookups (memory ceiling)
constexpr int kModeCompDiag = 16;   // DIAGNOSTIC, wrong results: no payload loads (compute ceiling)
constexpr int kModeNoStage = 32;    // DIAGNOSTIC (memory-only): no table staging
constexpr int kModeVerify = 64;     // read side: compare with p.expect[] instead of storing (crc32c_plan_verify)
constexpr int kModeS4C = 512;      // small batches: compact S4 image (T0..T3 once, 28 KiB staged)
constexpr int kModeEarly = 1024;    // the first tile's loads are issued before the table staging
constexpr int kModeHalves = 16384;  // with kModeQuarter, 2 units of 8 blocks per tile instead of 4 (3-6 tiles per CU)
constexpr int kModeQuarter = 4096;  // small batches: power-of-two tiles of chunks <= 2 KiB run as 4 work
                                    // units of 4 blocks each (4x the waves, 1/4 of each wave's latency chain)
constexpr int kModeXcdMap = 2048;   // A/B: workgroup ranges remapped so that each XCD's workgroups hold one
                                    // contiguous 1/8 of the batch (instead of every eighth range)
constexpr int kModeGDiagNoGather = 128;  // DIAGNOSTIC, wrong results: general items skip the per-subtile gather
constexpr int kModeGDiagNoMask = 8192;   // DIAGNOSTIC, wrong results: general items skip the chunk-start masks
constexpr int kModeGeneral = 256;   // the batch has general tiles (a plan without them runs the kernel without
                                    // their code: the power-of-two tile loop stays as compact as round 1's)
// (with kModeGeneral) the batch has no shifted tiles / no general tiles: the
// build leaves that code out, so the other path gets the registers and the
// schedule to itself
constexpr int kModeNoShift = 32768;
constexpr int kModeNoGItems = 65536;
constexpr int kModeGHoist = 131072;  // a general item's next subtile facts computed before this subtile's lookups
                                     // (the both-paths general build: padded chunks 0.5-2 % faster, round 5)
constexpr int kModeGGroup2 = 262144;  // A/B: (with kModeNoShift) general items gathered 2 subtiles at a time, not 4
constexpr int kModeHalfT = 1048576;   // (with kModeGeneral) the build also runs half tiles (their own builds: the
                                      // code costs the other general builds 3-8 %, round 5)
constexpr int kModeNoPadT = 2097152;  // (general builds) no padded power-of-two tiles: the production small-batch
                                      // builds (their code there cost config 3 ~4 %, round 5)
constexpr int kModeOvl = 524288;      // A/B: the first tile's loads issued right after the table staging's, before
                                      // the barrier that waits for the staging (their latencies overlap)
// GEN bits of the tile helpers below: general tiles, shifted (unaligned)
// tiles, general items gathered 4 subtiles at a time (finish_gtile GROUP)
constexpr int kGenItems = 1, kGenShift = 2, kGenGroup4 = 4, kGenGroup2 = 8, kGenHoist = 16, kGenHalf = 32,
              kGenPadded = 64;  // (padded power-of-two tiles: not in builds with kModeNoPadT)

// Work descriptors are read-only for the whole launch: reading them through
// the constant address space lets every (wave-uniform) descriptor fetch be a
// scalar s_load instead of a vector load that would join the payload loads
// on the vector-memory counter.
typedef const __attribute__((address_space(4))) FastTile *ConstTiles;
typedef const __attribute__((address_space(4))) ConstRun *ConstRuns;

__device__ __forceinline__ FastTile tile_at(const KParams &p, uint32_t i) {
    uint32_t b = 0;
    if (p.nblocks) {  // multi-block launch (wave-uniform): tile i of the plan's block shape, block b's copy
        b = i / p.block_tiles;
        i -= b * p.block_tiles;
    }
    const ConstTiles t = (ConstTiles)(p.tiles) + i;
    FastTile r;
    r.src = t->src;
    r.out = t->out;
    r.meta = t->meta;
    if (p.nblocks) {
        r.src += p.blocks[b].payload_delta;
        r.out += p.blocks[b].out_delta;
    }
    return r;
}

// gfx950 has no v_xor3_b32 but has v_bitop3_b32 (any 3-input bitwise
// function by truth table); 0x96 is a ^ b ^ c.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Opaque to the optimiser: stops InstCombine from re-associating the XOR
// trees of different pieces into one tree over every LDS read of the tile
// (which keeps all 256 reads live and spills).
__device__ __forceinline__ void opaque(uint32_t &x) { asm volatile("" : "+v"(x)); }

__device__ __forceinline__ uint32_t lds_u32(const uint8_t *lds, uint32_t off) {
    return *reinterpret_cast<const uint32_t *>(lds + off);
}

// lin() contribution of one lane's 16-byte piece at column col (= lane & 31),
// positional nibble tables (A/B variant 1).  Byte k of the piece: low nibble
// row at k*4096 + n*256, high nibble row at 128 + k*256 + n*4096; the lane's
// column is col*4.  DIAG 1 (diagnostic builds only, wrong results): the
// lookups are skipped.
template <int DIAG>
__device__ __forceinline__ uint32_t piece_lin(const uint8_t *lds, uint4 d, uint32_t col4) {
    uint32_t acc = 0;
    const uint32_t dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t x = dw[w];
        if (DIAG == 1) {
            acc ^= x;
            continue;
        }
        const uint32_t xs[4] = {x << 8, x, x >> 8, x >> 16};
        uint32_t r[8];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const uint32_t k = 4 * w + t;
            r[2 * t] = lds_u32(lds, ((xs[t] & 0x0F00u) | col4) + k * 4096u);
            r[2 * t + 1] = lds_u32(lds, ((xs[t] & 0xF000u) | col4) + 128u + k * 256u);
        }
        acc = xor3(xor3(r[0], r[1], r[2]), xor3(r[3], r[4], r[5]), xor3(r[6], r[7], acc));
    }
    return acc;
}

// (a & mask) | c as ONE v_and_or_b32: left to itself the compiler proves the
// operands disjoint, turns the OR into an add and splits it in two.
__device__ __forceinline__ uint32_t and_or(uint32_t a, uint32_t mask, uint32_t c) {
    uint32_t r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(mask), "v"(c));
    return r;
}

// Per-lane LDS address constants: the lane's column offset, and the same
// with the base of the S4 image's upper byte-table pair / N_q section.
struct LaneCols {
    uint32_t col4;  // (lane & 31) * 4
    uint32_t hi;    // col4 | 65536
    uint32_t nib;   // col4 | kS4NibOff
    uint32_t toff;  // T1 - T0 (= T3 - T2) in bytes: 128, or 1024 in the compact image
};

// S4 image layouts (template parameter IMG): the full image (32 replica
// columns of T0..T3) and the compact image (T0..T3 once each, for small
// batches: crc_math.h kS4C*).  (A half-column image -- 16 replica columns,
// 88 KiB staged -- measured +-0 and was removed)
constexpr int kImgFull = 0, kImgCompact = 2;
constexpr uint32_t kS4CNibOff = uint32_t(hdfs_crc::kS4CNibOff);
constexpr uint32_t kS4CShiftOff = uint32_t(hdfs_crc::kS4CShiftOff);
constexpr uint32_t kS4CStageBytes = (uint32_t(hdfs_crc::kS4CBytes) + 1023u) / 1024u * 1024u;

template <int IMG>
__device__ __forceinline__ LaneCols lane_cols(uint32_t q) {
    if (IMG == kImgCompact)  // T_m[b] at m * 1024 + 4 b: col4 = T0 base, hi = T2 base
        return LaneCols{0u, 2048u, (q << 2) | kS4CNibOff, 1024u};
    return LaneCols{q << 2, (q << 2) | 65536u, (q << 2) | kS4NibOff, 128u};
}

// Byte j of v into address bits 8..15 and the column base's bytes 0 and 2
// into bits 0..7 and 16..23 (v_perm_b32: selectors 0-3 = bytes of the
// second operand, 4-7 = bytes of the first, 0x0C = zero).
template <int J>
__device__ __forceinline__ uint32_t byte_addr(uint32_t v, uint32_t base) {
    return __builtin_amdgcn_perm(v, base, 0x0C020000u | uint32_t(4 + J) << 8);
}

// One slicing-by-4 step: S(v) ^ next, S(v) = T3[v.b0] ^ T2[v.b1] ^ T1[v.b2]
// ^ T0[v.b3] (each table replicated over the lane columns of the image, so
// the 32 lanes of a half-wave always hit 32 different banks).
template <int IMG>
__device__ __forceinline__ uint32_t s4(const uint8_t *lds, const LaneCols &c, uint32_t v, uint32_t next) {
    if (IMG == kImgCompact) {  // byte j of v -> bits 2..9 (v_bfe + v_lshl_add), one copy of each table
        const uint32_t a3 = lds_u32(lds, (__builtin_amdgcn_ubfe(v, 0, 8) << 2) + c.hi + c.toff);
        const uint32_t a2 = lds_u32(lds, (__builtin_amdgcn_ubfe(v, 8, 8) << 2) + c.hi);
        const uint32_t a1 = lds_u32(lds, (__builtin_amdgcn_ubfe(v, 16, 8) << 2) + c.toff);
        const uint32_t a0 = lds_u32(lds, (v >> 24) << 2);
        return xor3(xor3(a3, a2, a1), a0, next);
    }
    const uint32_t a3 = lds_u32(lds, byte_addr<0>(v, c.hi) + c.toff);    // T3: upper pair, odd
    const uint32_t a2 = lds_u32(lds, byte_addr<1>(v, c.hi));             // T2: upper pair, even
    const uint32_t a1 = lds_u32(lds, byte_addr<2>(v, c.col4) + c.toff);  // T1
    const uint32_t a0 = lds_u32(lds, byte_addr<3>(v, c.col4));           // T0
    return xor3(xor3(a3, a2, a1), a0, next);
}

// lin() of the lane's 16-byte piece with the S4 image: u = S(S(S(d0) ^ d1)
// ^ d2) ^ d3 is the register after the piece; N_q(u) = Z_{16(31-q)}(S(u))
// moves it to the block end (8 nibble lookups in the lane's column).
template <int DIAG, int IMG>
__device__ __forceinline__ uint32_t piece_lin_s4(const uint8_t *lds, uint4 d, const LaneCols &c) {
    if (DIAG == 1) return d.x ^ d.y ^ d.z ^ d.w;
    const uint32_t u = s4<IMG>(lds, c, s4<IMG>(lds, c, s4<IMG>(lds, c, d.x, d.y), d.z), d.w);
    const uint32_t xs[8] = {u << 8, u << 4, u, u >> 4, u >> 8, u >> 12, u >> 16, u >> 20};
    uint32_t r[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) r[t] = lds_u32(lds, and_or(xs[t], 0x0F00u, c.nib) + (t >> 1) * 4096u + (t & 1) * 128u);
    return xor3(xor3(r[0], r[1], r[2]), xor3(r[3], r[4], r[5]), r[6] ^ r[7]);
}

template <bool S4, int DIAG, int IMG>
__device__ __forceinline__ uint32_t piece(const uint8_t *lds, uint4 d, const LaneCols &c) {
    if (S4) return piece_lin_s4<DIAG, IMG>(lds, d, c);
    return piece_lin<DIAG>(lds, d, c.col4);
}

// Z^(512*s)(x), s in 1..15, from 8 nibble tables (16 entries each).
template <bool S4, int IMG>
__device__ __forceinline__ uint32_t zshift(const uint8_t *lds, uint32_t s, uint32_t x) {
    const uint32_t base = (!S4 ? kShiftOff : IMG == kImgCompact ? kS4CShiftOff : kS4ShiftOff) + (s - 1u) * 512u;
    uint32_t r = 0;
#pragma unroll
    for (int t = 0; t < 8; ++t) r ^= lds_u32(lds, base + t * 64u + ((x >> (4 * t)) & 15u) * 4u);
    return r;
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, 0xF, 0xF, false));
}
constexpr int kDppXor1 = 0xB1;   // quad_perm(1,0,3,2): lane ^ 1
constexpr int kDppXor2 = 0x4E;   // quad_perm(2,3,0,1): lane ^ 2
constexpr int kDppXor8 = 0x128;  // row_ror:8 inside a 16-lane row: lane ^ 8

template <int XORMASK>
__device__ __forceinline__ uint32_t swz_xor(uint32_t v) {
    // ds_swizzle bit mode inside 32-lane groups: and 0x1F, or 0, xor XORMASK.
    return static_cast<uint32_t>(__builtin_amdgcn_ds_swizzle(static_cast<int>(v), 0x1F | (XORMASK << 10)));
}

__device__ __forceinline__ uint32_t allreduce32(uint32_t x) {
    x ^= dpp<kDppXor1>(x);
    x ^= dpp<kDppXor2>(x);
    x ^= swz_xor<4>(x);
    x ^= dpp<kDppXor8>(x);
    x ^= swz_xor<16>(x);
    return x;
}

__device__ __forceinline__ uint32_t out_order(uint32_t crc, uint32_t flags) {
    return (flags & 1u) ? __builtin_bswap32(crc) : crc;  // htonl on the wire, hadooprpc.c:71-75
}

// The workgroup's verification state in LDS (after the tables and the tile
// counter): vacc[0] mismatches, vacc[1] lowest bad index, vacc[2] entries of
// the bad-index list (vacc + kVaccList, kBadList of them), vacc[3] flags.
constexpr uint32_t kBadList = 256;
constexpr uint32_t kVaccList = 7;
constexpr uint32_t kVaccTimedOut = 1u;        // vacc[3]: a key wait of this workgroup gave up
constexpr uint32_t kVaccFinishTimedOut = 2u;  // ... verify_finish's own (thread 0)
constexpr uint32_t kVaccRedo = 4u;            // ... and the key appeared later: bits set again
constexpr uint32_t kVerifyKeyPolls = 1u << 17;
constexpr uint32_t kVerifyOverlapBit = 0x80000000u;

// Waits until every vector-memory operation of the wave has completed; for a
// returning device-scope atomic that means it has been performed.
__device__ __forceinline__ void wait_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// The queue's dispatch id of this launch (the AQL packet index; LLVM has the
// intrinsic, clang no builtin for it).
extern "C" __device__ uint64_t llvm_amdgcn_dispatch_id() __asm("llvm.amdgcn.dispatch.id");

// A key unique to this launch (graph replays included): the address of its
// dispatch packet in the queue's ring and the queue's dispatch id, mixed.
__device__ __forceinline__ uint64_t launch_key() {
    const uint64_t ptr = uint64_t(reinterpret_cast<uintptr_t>(__builtin_amdgcn_dispatch_ptr()));
    return ptr + llvm_amdgcn_dispatch_id() * 0x9E3779B97F4A7C15ull;
}

// Waits (bounded: kVerifyKeyPolls polls, ~0.1-0.3 s) until the slot holds
// this launch's key, i.e. workgroup 0 has initialised the result and cleared
// the bitmap for this launch (polled with a returning atomic, performed where
// the key was written; acquire: the clear is visible after it).  False when
// it gave up.
__device__ __forceinline__ bool wait_launch_key(const KParams &p) {
    const unsigned long long key = launch_key();
    unsigned long long *ep = reinterpret_cast<unsigned long long *>(p.sched + kEpochWord);
    for (uint32_t polls = 0;; ++polls) {
        if (__hip_atomic_fetch_add(ep, 0ull, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == key) return true;
        if (polls == kVerifyKeyPolls) return false;
        __builtin_amdgcn_s_sleep(8);
    }
}

// A mismatch (VERIFY): bump the workgroup's LDS count and lower its LDS
// first-bad index (vacc[0], vacc[1]; merged grid-wide by verify_finish), and,
// when the caller passed a bitmap, note the index for it: the bitmap is
// cleared by workgroup 0 of this same launch, so a bit may only be set after
// this launch's key is published -- the first kBadList indices of the
// workgroup wait in LDS for verify_finish, later ones wait for the key here
// (rare path: a clean launch executes none of this).
__device__ __forceinline__ void mismatch(const KParams &p, uint32_t *vacc, uint32_t idx) {
    atomicAdd(vacc, 1u);
    atomicMin(vacc + 1, idx);
    if (!p.bad_bits) return;
    const uint32_t slot = atomicAdd(vacc + 2, 1u);
    if (slot < kBadList) {
        vacc[kVaccList + slot] = idx;
    } else {
        if (!wait_launch_key(p)) atomicOr(vacc + 3, kVaccTimedOut);
        atomicOr(p.bad_bits + (idx >> 5), 1u << (idx & 31u));
    }
}

// Checksum `idx` of the batch: stored, or (VERIFY) compared with `expect`.
template <bool VERIFY>
__device__ __forceinline__ void emit(const KParams &p, uint32_t *vacc, uint32_t idx, uint32_t crc, uint32_t expect) {
    const uint32_t v = out_order(crc, p.flags);
    if (VERIFY) {
        if (v != expect) mismatch(p, vacc, idx);
    } else {
        p.out[idx] = v;
    }
}

// ---- launch-wide verification result (kernel_abi.h slots) ----------------
// Start of a verification launch, the last wave of workgroup 0 (dispatched
// first, so a workgroup waiting for the key never waits for a workgroup that
// has not been placed): the caller's bitmap, when there is one, is cleared
// with vector stores (1 KiB per store instruction; config 2's 64 KiB is 64 of
// them), the result becomes {0, ~0} (returning device-scope atomics), and
// once both are performed the slot takes this launch's key (a release
// store).  No host-side memset of the bitmap or reset of the result precedes
// a launch (round 4 cleared the bitmap with a hipMemsetD32Async before every
// launch: 8.0 against 4.2 us per config-3 verify).
__device__ __forceinline__ void verify_init(const KParams &p, int lane) {
    if (p.bad_bits) {
        uint32_t *b = p.bad_bits;
        const uint32_t n = p.bad_words;
        const uint32_t head = min(n, uint32_t(((16u - (uintptr_t(b) & 15u)) & 15u) >> 2));
        if (uint32_t(lane) < head) b[lane] = 0;
        uint4 *v = reinterpret_cast<uint4 *>(b + head);
        const uint32_t nv = (n - head) >> 2;
        for (uint32_t i = uint32_t(lane); i < nv; i += 64u) v[i] = make_uint4(0, 0, 0, 0);
        const uint32_t tail = (n - head) & 3u;
        if (uint32_t(lane) < tail) b[head + 4u * nv + uint32_t(lane)] = 0;
    }
    if (lane == 0) {
        uint32_t a = __hip_atomic_exchange(p.result, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t c = __hip_atomic_exchange(p.result + 1, 0xffffffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("" : "+v"(a), "+v"(c));  // (returning forms: the wait covers them)
    }
    wait_vmem();  // (the whole wave's stores and atomics)
    if (lane == 0)
        __hip_atomic_store(reinterpret_cast<unsigned long long *>(p.sched + kEpochWord),
                           static_cast<unsigned long long>(launch_key()), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// The workgroup's listed bad indices into the caller's bitmap (every thread).
template <uint32_t THREADS>
__device__ __forceinline__ void set_listed_bits(const KParams &p, const uint32_t *vacc) {
    if (!p.bad_bits) return;
    const uint32_t n = min(vacc[2], kBadList);
    for (uint32_t i = threadIdx.x; i < n; i += THREADS) {
        const uint32_t idx = vacc[kVaccList + i];
        atomicOr(p.bad_bits + (idx >> 5), 1u << (idx & 31u));
    }
}

// Thread 0: this workgroup's count and lowest bad index into the result,
// with the overlap bit when its key wait gave up.
__device__ __forceinline__ void add_to_result(const KParams &p, const uint32_t *vacc, bool overlap) {
    if (overlap) {
        uint32_t o = __hip_atomic_fetch_or(p.result, kVerifyOverlapBit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("" : "+v"(o));
    }
    uint32_t a = __hip_atomic_fetch_add(p.result, vacc[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t b = __hip_atomic_fetch_min(p.result + 1, vacc[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("" : "+v"(a), "+v"(b));
    wait_vmem();
}

// End of a verification launch, every thread of every workgroup, after a
// workgroup barrier.  A clean workgroup does nothing; one with mismatches
// waits until workgroup 0 has initialised the result and cleared the bitmap
// for this launch (the slot holds this launch's key), then adds its count,
// lowers the first bad index and sets its listed bits.  The clean launch's
// tail is therefore empty: round 2's sharded tickets (every workgroup one
// returning atomic, the last of each shard a second, the last of those the
// publish) cost a small batch ~1.4 us (config 3: 5.05 vs 3.58 us, DESIGN.md
// section 5).
//
// The wait is bounded (kVerifyKeyPolls polls, ~0.1-0.3 s): if another verify
// launch of the same plan overlaps this one (a graph replay beside a direct
// verify on another stream: the library cannot order those) its key may
// replace this launch's before this workgroup sees it.  The workgroup then
// gives up waiting, adds its count and bits anyway and sets bit 31 of
// result[0] (kVerifyOverlapBit): "indeterminate -- overlapping verify
// launches of one plan".  A wait can also give up because workgroup 0 of
// this launch is merely late; its initialisation would then erase what this
// workgroup added, so the workgroup waits a second time, and if the key does
// appear it adds its count, the overlap bit and its bits again.  The kernel
// always finishes.
template <uint32_t THREADS>
__device__ __forceinline__ void verify_finish(const KParams &p, uint32_t *vacc) {
    if (!vacc[0]) return;  // (uniform: read after the barrier)
    if (threadIdx.x == 0) {
        // (kVaccTimedOut may also come from a mismatch past the LDS list
        // that gave up waiting: the result is then marked indeterminate)
        if (!wait_launch_key(p)) vacc[3] |= kVaccTimedOut | kVaccFinishTimedOut;
        add_to_result(p, vacc, (vacc[3] & kVaccTimedOut) != 0);
    }
    __syncthreads();
    set_listed_bits<THREADS>(p, vacc);
    if (!(vacc[3] & kVaccFinishTimedOut)) return;  // (uniform)
    // this workgroup added before workgroup 0's initialisation may have run:
    // once the key appears (the initialisation done), add again
    __syncthreads();
    if (threadIdx.x == 0) {
        const bool late_init = wait_launch_key(p);
        if (late_init) add_to_result(p, vacc, true);
        vacc[3] = late_init ? kVaccRedo : 0u;
    }
    __syncthreads();
    if (vacc[3] == kVaccRedo) set_listed_bits<THREADS>(p, vacc);
}

// ---- tiles: one wave, 16 blocks ------------------------------------------
// Block of the tile whose lin() lane `lane` holds after block_lin's
// reduce-scatter, and whether the lane emits that block's chunk checksum.
__device__ __forceinline__ uint32_t rep_block(int lane) {
    return 2u * (((lane & 8) ? 1u : 0u) + ((lane & 2) ? 2u : 0u) + ((lane & 1) ? 4u : 0u)) + (uint32_t(lane) >> 5);
}
// Inverse: a lane (lane bits 2 and 4 clear) that holds block b's lin().
__device__ __forceinline__ uint32_t block_lane(uint32_t b) {
    const uint32_t i = b >> 1;
    return ((i >> 2) & 1u) | (((i >> 1) & 1u) << 1) | ((i & 1u) << 3) | ((b & 1u) << 5);
}
__device__ __forceinline__ bool rep_lane(int lane, uint32_t blk, uint32_t nb, uint32_t lg) {
    return ((lane & 0x14) == 0) && ((blk & ((1u << lg) - 1u)) == 0) && blk < nb;
}

// A buffer resource for a wave-uniform range, built from SGPRs.  The
// compiler cannot always prove a work item's base and length uniform (in
// the verify instances of the general builds it could not), and a resource
// it believes divergent makes it wrap EVERY load in a readfirstlane
// "waterfall" loop (16 of them per general item in those kernels, round 2).
// readfirstlane of a value that is uniform is exact; on SGPR inputs it
// folds away.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const uint8_t *base, uint32_t bytes) {
    // (readfirstlane returns int: each half goes through uint32_t before it
    // is widened, or a low word >= 2^31 would sign-extend over the high one)
    const uint64_t a = reinterpret_cast<uint64_t>(base);
    const uint32_t hi = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(a >> 32))));
    const uint32_t lo = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(a))));
    const uint64_t ua = uint64_t(hi) << 32 | uint64_t(lo);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(ua), 0,
                                             int(__builtin_amdgcn_readfirstlane(bytes)), 0x00020000);
}

// Loads of one power-of-two tile: instruction i reads 1 KiB contiguous
// (blocks 2i, 2i+1) through a buffer descriptor whose range is the tile's
// nb * 512 valid bytes.  Lanes of blocks a partial tile does not have fall
// outside the range and read zeros without touching memory (lin() of zeros
// is 0, so they need no mask), every lane uses the same one-VGPR offset plus
// an immediate, and the instruction stream has no divergent branch.
// AUX 2 = non-temporal.  VERIFY: the expected checksum the lane compares is
// fetched with the tile.
template <int AUX, bool COMPDIAG, bool VERIFY>
__device__ __forceinline__ void load_tile(const KParams &p, FastTile t, int lane, uint4 v[8], uint32_t &ev) {
    if (COMPDIAG) {  // synthetic data, no memory traffic
        const uint32_t x = uint32_t(t.src) * 2654435761u + uint32_t(lane) * 40503u;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = make_uint4(x ^ i, x + i, x * 3u + i, x ^ (i << 16));
        return;
    }
    const uint32_t nb = t.meta & 0xffu;
    const __amdgpu_buffer_rsrc_t rsrc =
        uniform_rsrc(p.payload + t.src, nb * 512u);
    const uint32_t voff = 16u * uint32_t(lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const auto r = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + 1024u * i, 0, AUX);
        v[i] = make_uint4(r[0], r[1], r[2], r[3]);
    }
    if (VERIFY) {  // default policy: the next tile's lanes read the rest of the line
        const uint32_t lg = (t.meta >> 8) & 0xffu, blk = rep_block(lane);
        if (rep_lane(lane, blk, nb, lg)) ev = p.expect[t.out + (blk >> lg)];
    }
    // Keep the loads ahead of whatever compute follows.
    __builtin_amdgcn_sched_barrier(0);
}

// lin() of a tile's 8 pieces (instruction i's 16 bytes per lane), each
// piece first passed through prep(i, piece) (general tiles: the chunk-start
// masks), so that piece i's lookups start as soon as its own load is back.
template <int DIAG, bool S4, int IMG, typename Prep, int NP = 8>
__device__ __forceinline__ void tile_pieces(const uint8_t *lds, uint4 v[8], uint32_t pc[8], int lane, Prep prep) {
    const LaneCols cols = lane_cols<IMG>(uint32_t(lane & 31));
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        prep(i, v[i]);
        pc[i] = piece<S4, DIAG, IMG>(lds, v[i], cols);
        opaque(pc[i]);
        // One piece at a time (nibble tables: 32 independent reads each), or
        // two (S4: a piece is a chain of 4 dependent steps, so two chains
        // interleave to keep 8 reads in flight): keeps the scheduler from
        // hoisting every piece's LDS reads together (register pressure).
        if (!S4 || (i & 1)) __builtin_amdgcn_sched_barrier(0);
    }
}
struct NoPrep {
    __device__ __forceinline__ void operator()(int, uint4 &) const {}
};

// The tile's 8 piece values -> one lin() per block: reduce-scatter over lane
// bits 0, 1, 3 (8 values -> 1), then all-reduce over lane bits 2 and 4.
// Afterwards lane l holds lin() of block rep_block(l) = 2*i + h with
// i = b3 + 2*b1 + 4*b0 (b = bits of l).
// (whole = false: the last all-reduce step is skipped, so lanes 0..15 and
// 16..31 of the block keep the lin() of their own half; half tiles)
__device__ __forceinline__ uint32_t block_lin(const uint32_t pc[8], int lane, bool whole = true) {
    const bool b0 = lane & 1, b1 = lane & 2, b3 = lane & 8;
    uint32_t u[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t keep = b0 ? pc[k + 4] : pc[k];
        const uint32_t send = b0 ? pc[k] : pc[k + 4];
        u[k] = keep ^ dpp<kDppXor1>(send);
    }
    uint32_t w2[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t keep = b1 ? u[j + 2] : u[j];
        const uint32_t send = b1 ? u[j] : u[j + 2];
        w2[j] = keep ^ dpp<kDppXor2>(send);
    }
    uint32_t x;
    {
        const uint32_t keep = b3 ? w2[1] : w2[0];
        const uint32_t send = b3 ? w2[0] : w2[1];
        x = keep ^ dpp<kDppXor8>(send);
    }
    x ^= swz_xor<4>(x);
    const uint32_t y = swz_xor<16>(x);
    return whole ? x ^ y : x;
}

// Power-of-two tile: blocks combined per chunk, chunk checksums stored (or
// compared); cst = the chunk length's affine constant crc(0, zeros(bpc)).
template <bool S4, bool VERIFY, int IMG>
__device__ __forceinline__ void reduce_emit(const KParams &p, const uint8_t *lds, uint32_t *vacc, FastTile t,
                                            const uint32_t pc[8], uint32_t ev, int lane, uint32_t cst) {
    const uint32_t nb = t.meta & 0xffu;
    const uint32_t lg = (t.meta >> 8) & 0xffu;
    uint32_t x = block_lin(pc, lane);
    const uint32_t blk = rep_block(lane);
    if (lg) {  // chunks of 2^lg blocks: shift each block to the chunk end, XOR them
        const uint32_t nbc = 1u << lg;
        const uint32_t s = nbc - 1u - (blk & (nbc - 1u));
        if (s) x = zshift<S4, IMG>(lds, s, x);
        x ^= static_cast<uint32_t>(__shfl_xor(static_cast<int>(x), 32));  // block bit 0 = lane bit 5
        if (lg >= 2) x ^= dpp<kDppXor8>(x);                               // block bit 1 = lane bit 3
        if (lg >= 3) x ^= dpp<kDppXor2>(x);                               // block bit 2 = lane bit 1
        if (lg >= 4) x ^= dpp<kDppXor1>(x);                               // block bit 3 = lane bit 0
    }
    const uint32_t crc = x ^ cst;
    if (rep_lane(lane, blk, nb, lg)) emit<VERIFY>(p, vacc, t.out + (blk >> lg), crc, ev);
}
template <bool S4, bool VERIFY, int IMG>
__device__ __forceinline__ void reduce_emit(const KParams &p, const uint8_t *lds, uint32_t *vacc, FastTile t,
                                            const uint32_t pc[8], uint32_t ev, int lane) {
    reduce_emit<S4, VERIFY, IMG>(p, lds, vacc, t, pc, ev, lane, p.c_lg[(t.meta >> 8) & 0xffu]);
}

}  // namespace hdfs_crc_dev

#include "crc32c_general.h"  // general items (needs the helpers above)

namespace hdfs_crc_dev {

// ---- power-of-two tiles off 16-byte alignment (GENERAL builds) ----------
// A dwordx4 load that straddles a 16-byte boundary costs the memory pipeline
// about twice an aligned one (config 2 five bytes off: 58 us memory-only
// against 42.6).  Such a tile (r = its address mod 16, uniform) is instead
// loaded from the aligned address below it, 16 bytes per lane as usual,
// plus the 16 bytes after the window (for the last lane); lane q's own 16
// bytes then start r bytes into its load and end r bytes into the next
// lane's, which a wave shift (DPP wave_shl:1) and v_alignbyte reassemble.
__device__ __forceinline__ uint32_t tile_misalign(const KParams &p, FastTile t) {
    return uint32_t(reinterpret_cast<uintptr_t>(p.payload + t.src)) & 15u;
}

// (the loads alone, from a payload base: also the resident kernel's,
// resident_engine.h)
template <int AUX>
__device__ __forceinline__ void load_shifted_raw(const uint8_t *payload, FastTile t, uint32_t r, int lane, uint4 v[9]) {
    const uint32_t nb = t.meta & 0xffu;
    const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(payload + t.src - r, r + nb * 512u);
    const uint32_t voff = 16u * uint32_t(lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + 1024u * i, 0, AUX);
        v[i] = make_uint4(x[0], x[1], x[2], x[3]);
    }
    {  // lane 0 only: the tile's last 16 bytes (a load that straddles the end of
       // the descriptor's range reads zeros, so the last lane cannot take its
       // tail from the next lane's load)
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, lane == 0 ? r + nb * 512u - 16u : 0x80000000u, 0,
                                                             AUX);
        v[8] = make_uint4(x[0], x[1], x[2], x[3]);
    }
}

template <int AUX, bool VERIFY>
__device__ __forceinline__ void load_tile_shifted(const KParams &p, FastTile t, uint32_t r, int lane, uint4 v[9],
                                                  uint32_t &ev) {
    load_shifted_raw<AUX>(p.payload, t, r, lane, v);
    if (VERIFY) {
        const uint32_t nb = t.meta & 0xffu, lg = (t.meta >> 8) & 0xffu, blk = rep_block(lane);
        if (rep_lane(lane, blk, nb, lg)) ev = p.expect[t.out + (blk >> lg)];
    }
    __builtin_amdgcn_sched_barrier(0);
}

// Piece i of a shifted tile: bytes r .. r + 15 of (this lane's load, the
// next lane's load); lane 63 takes lane 0 of load i + 1; the tile's last
// lane (block nb - 1's lane 31) takes the tile's last 16 bytes (v[8]).
// r = 4 M + b, M a template parameter: each piece is straight-line code, so
// piece i waits only for loads i and i + 1 (a branch on M inside every piece
// made the compiler wait for all nine loads before the first lookup).
template <uint32_t M>
struct ShiftPrep {
    const uint4 *v;
    uint32_t b;
    int lane;
    uint32_t last_i;  // load instruction and lane of the tile's last 16 bytes
    int last_lane;
    __device__ __forceinline__ uint32_t shl1(uint32_t own, uint32_t last) const {
        // DPP wave_shl:1 -- lane l reads lane l + 1; lane 63 (no source) keeps `last`'s lane 63
        return uint32_t(__builtin_amdgcn_update_dpp(int(last), int(own), 0x130, 0xF, 0xF, false));
    }
    __device__ __forceinline__ static uint32_t rol1(uint32_t x) {
        // DPP wave_rol:1 -- lane l reads lane (l + 1) mod 64: lane 63 gets lane 0
        return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x134, 0xF, 0xF, false));
    }
    __device__ __forceinline__ uint32_t ab(uint32_t hi, uint32_t lo) const {
        return __builtin_amdgcn_alignbyte(hi, lo, b);
    }
    __device__ __forceinline__ void operator()(int i, uint4 &x) const {
        const uint4 nx = v[i + 1];
        const uint32_t n0 = shl1(x.x, rol1(nx.x));
        if constexpr (M == 0) {
            x = make_uint4(ab(x.y, x.x), ab(x.z, x.y), ab(x.w, x.z), ab(n0, x.w));
        } else if constexpr (M == 1) {
            const uint32_t n1 = shl1(x.y, rol1(nx.y));
            x = make_uint4(ab(x.z, x.y), ab(x.w, x.z), ab(n0, x.w), ab(n1, n0));
        } else if constexpr (M == 2) {
            const uint32_t n1 = shl1(x.y, rol1(nx.y));
            const uint32_t n2 = shl1(x.z, rol1(nx.z));
            x = make_uint4(ab(x.w, x.z), ab(n0, x.w), ab(n1, n0), ab(n2, n1));
        } else {
            const uint32_t n1 = shl1(x.y, rol1(nx.y));
            const uint32_t n2 = shl1(x.z, rol1(nx.z));
            const uint32_t n3 = shl1(x.w, rol1(nx.w));
            x = make_uint4(ab(n0, x.w), ab(n1, n0), ab(n2, n1), ab(n3, n2));
        }
        if (uint32_t(i) == last_i) {
            const uint4 t = v[8];
            const uint4 f = make_uint4(__builtin_amdgcn_readfirstlane(t.x), __builtin_amdgcn_readfirstlane(t.y),
                                       __builtin_amdgcn_readfirstlane(t.z), __builtin_amdgcn_readfirstlane(t.w));
            if (lane == last_lane) x = f;
        }
    }
};

// ---- padded power-of-two tiles (builds with the general-tile code) -------
// bpc = 512 * 2^lg - pad (plan.h): chunk j of the tile is virtual blocks
// j 2^lg .. (j + 1) 2^lg - 1, its data right-aligned behind pad zero bytes
// (leading zeros leave lin() unchanged), so the tile reduces like a
// power-of-two one and only the affine constant differs.  Lane q of block b
// reads bytes 512 (b mod 2^lg) + 16 q - pad of chunk b >> lg through a
// descriptor that starts 16 bytes before the tile (the straddling lane
// reads up to 15 bytes before a chunk); lanes wholly inside a pad read
// zeros without touching memory, and the straddling lane's bytes before the
// chunk are masked (PadPrep).  Round 5: these chunks ran as general items
// before (per-subtile gather, block facts on the scalar unit).
__device__ __forceinline__ uint32_t tile_pad(FastTile t) { return (t.meta >> 18) & 511u; }

template <int AUX, bool VERIFY>
__device__ __forceinline__ void load_tile_padded(const KParams &p, FastTile t, int lane, uint4 v[8], uint32_t &ev) {
    const uint32_t nb = t.meta & 0xffu, lg = (t.meta >> 8) & 0xffu, pad = tile_pad(t);
    const uint32_t bpc = (512u << lg) - pad, km = (1u << lg) - 1u;
    const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(p.payload + t.src - 16u, 16u + (nb >> lg) * bpc);
    // Offset of lane l in instruction i = a wave-uniform part + a lane part:
    //   lg >= 1: blocks 2i, 2i + 1 are blocks w, w + 1 of chunk 2i >> lg
    //            (1 KiB contiguous): (2i >> lg) bpc + 512 w - pad, + 16 l;
    //   lg = 0:  block 2i + h is chunk 2i + h: 2i bpc - pad, + h bpc + 16 q.
    // A lane wholly inside a first block's pad reads nothing (bit 31: past
    // the range).  Blocks past nb read what they read: their lin() is never
    // combined with a block of the tile's chunks nor stored.
    const uint32_t h = uint32_t(lane) >> 5, q16 = 16u * (uint32_t(lane) & 31u);
    const uint32_t lane_all = lg ? 16u * uint32_t(lane) : h * bpc + q16;
    const uint32_t lane_first = (q16 + 16u <= pad && (lg == 0u || h == 0u)) ? 0x80000000u : lane_all;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t b2 = 2u * uint32_t(i), w = b2 & km;  // (uniform)
        const uint32_t ubase = 16u + (b2 >> lg) * bpc + 512u * w - pad;
        const auto r = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (w ? lane_all : lane_first) + ubase, 0, AUX);
        v[i] = make_uint4(r[0], r[1], r[2], r[3]);
    }
    if (VERIFY) {
        const uint32_t blk = rep_block(lane);
        if (rep_lane(lane, blk, nb, lg)) ev = p.expect[t.out + (blk >> lg)];
    }
    __builtin_amdgcn_sched_barrier(0);
}

// The lanes of a chunk's first block keep their bytes at positions >= pad -
// 16 q (kp; all ones in other blocks' lanes), selected per piece without a
// branch (a branch between the two interleaved lookup chains of a piece pair
// would split them).  Only a pad that is not a multiple of 16 leaves a lane
// straddling the chunk start; otherwise the tile runs without this prep.
struct PadPrep {
    uint4 kp;
    uint32_t km;
    __device__ __forceinline__ void operator()(int i, uint4 &x) const {
        apply_keep(x, kp, 0u - uint32_t(((2u * uint32_t(i)) & km) == 0u));
    }
};

// ---- half tiles (builds with the general-tile code) -----------------------
// bpc <= 256 (M = 0), 512 < bpc <= 768 (M = 1) or 1024 < bpc <= 1280 (M = 2):
// a chunk is M full 512-byte
// blocks after a partial part of r = bpc - 512 M <= 256 bytes, right-aligned
// into a 256-byte half block behind padh = 256 - r zeros.  Two partial parts
// share one block: its upper half (lanes 16..31, whose columns are the last
// 256 bytes before a block end) holds chunk 2m's, its lower half (lanes
// 0..15) chunk 2m + 1's, those lanes taking the N_q finishing operators of
// columns q + 16 (the T tables are the same in every column, so their
// lookups keep their own, conflict-free columns).  A pair block's lin() is
// reduced per half (block_lin without its last all-reduce step).
//   M = 0: 16 pair blocks, up to 32 chunks per tile.
//   M = 1: block c < 10 is chunk c's full block, block 10 + m the pair block
//          of chunks 2m, 2m + 1 (up to 10 chunks per tile, 15 blocks); chunk
//          c's lin = Z^512(its partial half's lin) ^ its full block's lin.
//   M = 2: blocks 2c, 2c + 1 are chunk c's (c < 6), 12 + m the pair blocks
//          (6 chunks, 15 blocks); lin = Z^1024(partial) ^ Z^512(block 2c)
//          ^ block 2c + 1.
// The tile holds n chunks; slots past n read what they read (never stored).
// Round 5: bpc 700 took 2 virtual blocks per chunk as a padded tile, 1.5
// here.
__device__ __forceinline__ bool is_half(FastTile t) { return (t.meta & 0xC0000000u) == hdfs_crc::kHalfTile; }

// Tile geometry of half tiles: full-block load instructions first (M = 1:
// chunks 2i, 2i + 1, one block each; M = 2: chunk i's two blocks), then the
// pair instructions; the full chunks' blocks before the pair blocks.
template <uint32_t M>
struct HalfShape {
    static constexpr uint32_t kFullInstr = M == 0 ? 0u : M == 1 ? 5u : 6u;
    static constexpr uint32_t kFullBlocks = 2u * kFullInstr;  // (pair block m: kFullBlocks + m)
};

// In the verify build the lane constants of half tiles are recomputed per
// tile (an opaque copy of the lane index): hoisted out of the tile loop they
// stayed live across it, some were spilled and reloaded between a tile's
// loads, and the scratch wait then waited for the payload loads too (bpc 700
// verify 64 against exec 53 us, round 5).  The exec build holds them without
// spilling, and recomputing them there put ~25 VALU before each tile's
// loads (+5 %).
__device__ __forceinline__ int fresh_lane(int lane) {
    asm volatile("" : "+v"(lane));
    return lane;
}

template <int AUX, bool VERIFY, uint32_t M>
__device__ __forceinline__ void load_tile_half(const KParams &p, FastTile t, int lane, uint4 v[8], uint32_t &ev) {
    using S = HalfShape<M>;
    if (VERIFY) lane = fresh_lane(lane);
    const uint32_t n = t.meta & 0xffu, padh = (t.meta >> 18) & 511u;
    const uint32_t r = 256u - padh, bpc = 512u * M + r;
    const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(p.payload + t.src - 16u, 16u + n * bpc);
    const uint32_t h = uint32_t(lane) >> 5, q = uint32_t(lane) & 31u, u = q >> 4, q16h = 16u * (q & 15u);
    // pair instruction j: half-wave h is pair block 2j + h (chunks 4j + 2h,
    // 4j + 2h + 1), lane (u, q') of it reads 16 q' past chunk 4j + 2h + 1 - u's
    // half-block start c bpc - padh; full instruction i: M = 1, half-wave h
    // is chunk 2i + h's full block, from c bpc + r; M = 2, the wave reads
    // chunk i's two full blocks (1 KiB from i bpc + r)
    const uint32_t lane_pair = q16h + 16u <= padh ? 0x80000000u : (2u * h + 1u - u) * bpc + q16h;
    const uint32_t lane_full = M == 1 ? h * bpc + 16u * q : 16u * uint32_t(lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t voff;
        if (uint32_t(i) >= S::kFullInstr) {
            const uint32_t j = uint32_t(i) - S::kFullInstr;
            voff = lane_pair + (16u + 4u * j * bpc - padh);
        } else {
            voff = lane_full + (16u + (M == 1 ? 2u : 1u) * uint32_t(i) * bpc + r);
        }
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, 0, AUX);
        v[i] = make_uint4(x[0], x[1], x[2], x[3]);
    }
    if (VERIFY) {
        const uint32_t blk = rep_block(lane);
        const uint32_t c = M == 0 ? 2u * blk + 1u - ((uint32_t(lane) >> 4) & 1u) : blk / (M ? M : 1u);
        const bool rep = M == 0 ? (lane & 4) == 0 : (lane & 0x14) == 0 && blk < S::kFullBlocks && blk % (M ? M : 1u) == 0;
        if (rep && c < n) ev = p.expect[t.out + c];
    }
    __builtin_amdgcn_sched_barrier(0);
}

template <int DIAG, bool S4, bool VERIFY, int IMG, uint32_t M>
__device__ __forceinline__ void finish_half(const KParams &p, const uint8_t *lds, uint32_t *vacc, FastTile t,
                                            uint4 v[8], uint32_t ev, int lane) {
    using S = HalfShape<M>;
    if (VERIFY) lane = fresh_lane(lane);
    const uint32_t n = t.meta & 0xffu, padh = (t.meta >> 18) & 511u;
    typedef const __attribute__((address_space(4))) uint32_t *ConstU32;
    const ConstU32 zc = (ConstU32)(p.table_s4 + hdfs_crc::kZeroCrcOff);
    const uint32_t cst = zc[512u * M + 256u - padh];  // (a scalar load, in flight during the lookups)
    const uint32_t q = uint32_t(lane) & 31u;
    // a pair block's lanes keep their bytes at positions >= padh - 16 q' of
    // their half (lanes wholly inside the pad loaded nothing)
    const uint4 kp = keep_masks(int(padh) - int(16u * (q & 15u)));
    const LaneCols cols = lane_cols<IMG>(q);
    LaneCols colp = cols;
    colp.nib = lane_cols<IMG>(q | 16u).nib;
    uint32_t pc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const bool pair = uint32_t(i) >= S::kFullInstr;
        if (pair && !(DIAG & 4)) {
            v[i].x &= kp.x;
            v[i].y &= kp.y;
            v[i].z &= kp.z;
            v[i].w &= kp.w;
        }
        pc[i] = piece<S4, DIAG, IMG>(lds, v[i], pair ? colp : cols);
        opaque(pc[i]);
        if (!S4 || (i & 1)) __builtin_amdgcn_sched_barrier(0);
    }
    const uint32_t blk = rep_block(lane);
    uint32_t x = block_lin(pc, lane, M != 0 && blk < S::kFullBlocks);
    uint32_t c;
    bool rep;
    if (M == 0) {  // lane bit 4: the half, upper = chunk 2 blk
        c = 2u * blk + 1u - ((uint32_t(lane) >> 4) & 1u);
        rep = (lane & 4) == 0;
    } else {
        // chunk c = blk / M: its full blocks (M = 2: block 2c shifted by
        // Z^512 and joined with block 2c + 1, lane bit 5), then its partial
        // half from pair block kFullBlocks + c / 2, shifted by Z^(512 M)
        constexpr uint32_t kM = M ? M : 1u;
        c = blk / kM;
        uint32_t xf = x;  // (x itself stays: the pair blocks' lanes are read below)
        if (M == 2) {
            const uint32_t xs = (blk & 1u) ? x : zshift<S4, IMG>(lds, 1u, x);
            xf = xs ^ static_cast<uint32_t>(__shfl_xor(static_cast<int>(xs), 32));
        }
        const uint32_t src =
            blk < S::kFullBlocks ? block_lane(S::kFullBlocks + (c >> 1)) | ((1u - (c & 1u)) << 4) : uint32_t(lane);
        const uint32_t y = uint32_t(__builtin_amdgcn_ds_bpermute(int(src << 2), int(x)));
        x = xf ^ zshift<S4, IMG>(lds, kM, y);
        rep = (lane & 0x14) == 0 && blk < S::kFullBlocks && blk % kM == 0;
    }
    if (rep && c < n) emit<VERIFY>(p, vacc, t.out + c, x ^ cst, ev);
}

template <int AUX, int DIAG, bool COMPDIAG, bool S4, bool VERIFY, int IMG, int GEN>
__device__ __forceinline__ void finish_tile(const KParams &p, const uint8_t *lds, uint32_t *vacc, FastTile t,
                                            uint4 v[9], uint32_t ev, int lane) {
    uint32_t pc[8];
    if ((GEN & kGenItems) && (t.meta & kGeneralTile)) {
        finish_gtile<AUX, DIAG, COMPDIAG, S4, VERIFY, IMG, (GEN & kGenGroup4) ? 4u : (GEN & kGenGroup2) ? 2u : 1u,
                     (GEN & kGenHoist) != 0>(p, lds, vacc, t, v, ev, lane);
        return;
    }
    if ((GEN & kGenHalf) && is_half(t)) {
        switch ((t.meta >> 8) & 0xffu) {  // (uniform) M
            case 0: finish_half<DIAG, S4, VERIFY, IMG, 0>(p, lds, vacc, t, v, ev, lane); break;
            case 1: finish_half<DIAG, S4, VERIFY, IMG, 1>(p, lds, vacc, t, v, ev, lane); break;
            default: finish_half<DIAG, S4, VERIFY, IMG, 2>(p, lds, vacc, t, v, ev, lane); break;
        }
        return;
    }
    if ((GEN & kGenPadded) && tile_pad(t)) {
        const uint32_t pad = tile_pad(t), lg = (t.meta >> 8) & 0xffu;
        typedef const __attribute__((address_space(4))) uint32_t *ConstU32;
        const ConstU32 zc = (ConstU32)(p.table_s4 + hdfs_crc::kZeroCrcOff);
        const uint32_t cst = zc[(512u << lg) - pad];  // (a scalar load, in flight during the lookups)
        if (pad & 15u) {  // (uniform) a lane straddles each chunk start
            const bool first = lg == 0u || lane < 32;  // (a first block's lanes, where instruction i holds one)
            const uint4 ones = make_uint4(~0u, ~0u, ~0u, ~0u);
            tile_pieces<DIAG, S4, IMG>(
                lds, v, pc, lane,
                PadPrep{first ? keep_masks(int(pad) - int(16u * (uint32_t(lane) & 31u))) : ones, (1u << lg) - 1u});
        } else {
            tile_pieces<DIAG, S4, IMG>(lds, v, pc, lane, NoPrep{});
        }
        reduce_emit<S4, VERIFY, IMG>(p, lds, vacc, t, pc, ev, lane, cst);
        return;
    }
    const uint32_t r = (GEN & kGenShift) && !COMPDIAG ? tile_misalign(p, t) : 0u;
    if (r) {
        const uint32_t b = r & 3u, li = ((t.meta & 0xffu) - 1u) >> 1;
        const int ll = int(((t.meta & 0xffu) - 1u) & 1u) * 32 + 31;
        switch (r >> 2) {
            case 0: tile_pieces<DIAG, S4, IMG>(lds, v, pc, lane, ShiftPrep<0>{v, b, lane, li, ll}); break;
            case 1: tile_pieces<DIAG, S4, IMG>(lds, v, pc, lane, ShiftPrep<1>{v, b, lane, li, ll}); break;
            case 2: tile_pieces<DIAG, S4, IMG>(lds, v, pc, lane, ShiftPrep<2>{v, b, lane, li, ll}); break;
            default: tile_pieces<DIAG, S4, IMG>(lds, v, pc, lane, ShiftPrep<3>{v, b, lane, li, ll}); break;
        }
    } else {
        tile_pieces<DIAG, S4, IMG>(lds, v, pc, lane, NoPrep{});
    }
    reduce_emit<S4, VERIFY, IMG>(p, lds, vacc, t, pc, ev, lane);
}

template <int AUX, bool COMPDIAG, bool VERIFY, int GEN>
__device__ __forceinline__ void load_any(const KParams &p, FastTile t, int lane, uint4 v[9], uint32_t &ev) {
    if ((GEN & kGenItems) && (t.meta & kGeneralTile)) {
        load_gtile<VERIFY>(p, t, lane, ev);
    } else if ((GEN & kGenHalf) && !COMPDIAG && is_half(t)) {
        switch ((t.meta >> 8) & 0xffu) {
            case 0: load_tile_half<AUX, VERIFY, 0>(p, t, lane, v, ev); break;
            case 1: load_tile_half<AUX, VERIFY, 1>(p, t, lane, v, ev); break;
            default: load_tile_half<AUX, VERIFY, 2>(p, t, lane, v, ev); break;
        }
    } else if ((GEN & kGenPadded) && !COMPDIAG && tile_pad(t)) {
        load_tile_padded<AUX, VERIFY>(p, t, lane, v, ev);
    } else if ((GEN & kGenShift) && !COMPDIAG && tile_misalign(p, t)) {
        load_tile_shifted<AUX, VERIFY>(p, t, tile_misalign(p, t), lane, v, ev);
    } else {
        load_tile<AUX, COMPDIAG, VERIFY>(p, t, lane, v, ev);
    }
}

// ---- quarter units (kModeQuarter): blocks 4u .. 4u + 3 of a tile ---------
// A small batch leaves most of the chip's waves idle and each busy wave's
// load -> 8 chained pieces -> reduce latency is the launch.  Unit j of a
// launch is quarter u = j & 3 of tile j >> 2: for power-of-two chunks of at
// most 4 blocks (bpc <= 2048) a quarter holds whole chunks, so it is an
// ordinary tile of <= 4 blocks, loaded by 2 instructions and looked up as 2
// pieces per lane.  General items and tiles of longer chunks run whole as
// unit 0 of their tile (units 1-3 are empty).
// SPLIT 2 (A/B, debug library): halves of 8 blocks instead (chunks <= 4 KiB).
// Returns 0 (empty unit), 1 (a whole tile / item in ft) or 2 (a unit in ft).
template <int AUX, bool COMPDIAG, bool VERIFY, int GEN, int SPLIT = 4>
__device__ __forceinline__ int load_unit(const KParams &p, uint32_t j, int lane, FastTile &ft, uint4 v[9],
                                         uint32_t &ev) {
    constexpr uint32_t kUB = 16 / SPLIT;  // blocks per unit
    constexpr int kNP = 8 / SPLIT;        // load instructions (pieces per lane) per unit
    const FastTile x = tile_at(p, j / SPLIT);
    const uint32_t u = j % SPLIT;
    const uint32_t lg = (x.meta >> 8) & 0xffu;
    if (((GEN & kGenItems) && (x.meta & kGeneralTile)) || ((GEN & kGenPadded) && tile_pad(x)) ||
        ((GEN & kGenHalf) && is_half(x)) ||
        (1u << lg) > kUB) {
        if (u) return 0;
        ft = x;
        load_any<AUX, COMPDIAG, VERIFY, GEN>(p, ft, lane, v, ev);
        return 1;
    }
    const uint32_t nb = x.meta & 0xffu;
    if (kUB * u >= nb) return 0;
    ft.src = x.src + 512u * kUB * u;
    ft.out = x.out + ((kUB * u) >> lg);
    ft.meta = min(nb - kUB * u, kUB) | (lg << 8);
    if (COMPDIAG) {
        load_tile<AUX, true, false>(p, ft, lane, v, ev);
        return 2;
    }
    const uint32_t nbq = ft.meta & 0xffu;
    const __amdgpu_buffer_rsrc_t rsrc =
        uniform_rsrc(p.payload + ft.src, nbq * 512u);
    const uint32_t voff = 16u * uint32_t(lane);
#pragma unroll
    for (int i = 0; i < kNP; ++i) {
        const auto r = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + 1024u * i, 0, AUX);
        v[i] = make_uint4(r[0], r[1], r[2], r[3]);
    }
    if (VERIFY) {
        const uint32_t blk = rep_block(lane);
        if (rep_lane(lane, blk, nbq, lg)) ev = p.expect[ft.out + (blk >> lg)];
    }
    __builtin_amdgcn_sched_barrier(0);
    return 2;
}

template <int DIAG, bool S4, bool VERIFY, int IMG, int SPLIT = 4>
__device__ __forceinline__ void finish_quarter(const KParams &p, const uint8_t *lds, uint32_t *vacc, FastTile t,
                                               uint4 v[8], uint32_t ev, int lane) {
    constexpr int kNP = 8 / SPLIT;
    uint32_t pc[8];
    tile_pieces<DIAG, S4, IMG, NoPrep, kNP>(lds, v, pc, lane, NoPrep{});
#pragma unroll
    for (int i = kNP; i < 8; ++i) pc[i] = 0;  // blocks past the unit: none
    reduce_emit<S4, VERIFY, IMG>(p, lds, vacc, t, pc, ev, lane);
}

// One tile index from the workgroup's LDS counter (one ds_add_rtn per wave).
__device__ __forceinline__ uint32_t pool_grab(uint32_t *pool_ctr, int lane) {
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(pool_ctr, 1u);
    return __builtin_amdgcn_readfirstlane(t);
}

}  // namespace hdfs_crc_dev

#include "crc32c_items.h"  // GenItem / SegItem / ConstRun work items

// THREADS per workgroup, WPS = waves per SIMD the launch bound asks for
// (= workgroups per CU x THREADS / 256; it caps VGPRs at 512 / WPS).
template <int THREADS, int WPS, int MODE>
__global__ __launch_bounds__(THREADS, WPS) void hdfs_crc32c_plan_kernel(hdfs_crc::KParams p) {
    using namespace hdfs_crc_dev;
    constexpr bool NT = (MODE & kModeNt) != 0;
    constexpr bool S4 = (MODE & kModeS4) != 0;
    constexpr bool STAMPS = (MODE & kModeStamps) != 0;
    constexpr bool COMPDIAG = (MODE & kModeCompDiag) != 0;
    // (bit 0: no lookups; bits 1-2: general-item ablations -- diagnostic builds only)
    constexpr int DIAG = ((MODE & kModeMemDiag) ? 1 : 0) | ((MODE & kModeGDiagNoGather) ? 2 : 0) |
                         ((MODE & kModeGDiagNoMask) ? 4 : 0);
    constexpr bool NOSTAGE = (MODE & kModeNoStage) != 0;
    constexpr bool VERIFY = (MODE & kModeVerify) != 0;
    constexpr bool C = S4 && (MODE & kModeS4C) != 0;
    constexpr int IMG = C ? kImgCompact : kImgFull;
    constexpr bool GENERAL = (MODE & kModeGeneral) != 0;
    constexpr int GEN = !GENERAL ? 0
                                 : ((MODE & kModeNoGItems) ? 0 : kGenItems) |
                                       ((MODE & kModeNoShift) ? ((MODE & kModeGGroup2) ? kGenGroup2 : kGenGroup4)
                                                              : (kGenShift | kGenGroup2)) |
                                       ((MODE & kModeGHoist) ? kGenHoist : 0) | ((MODE & kModeHalfT) ? kGenHalf : 0) |
                                       ((!(MODE & (kModeNoGItems | kModeNoPadT))) ? kGenPadded : 0);
    constexpr bool EARLY = (MODE & kModeEarly) != 0;
    constexpr bool OVL = !EARLY && (MODE & kModeOvl) != 0;
    constexpr bool QUARTER = (MODE & kModeQuarter) != 0;
    constexpr bool XCDMAP = (MODE & kModeXcdMap) != 0;
    constexpr int SPLIT = (MODE & kModeHalves) ? 2 : 4;  // units per tile
    constexpr int AUX = NT ? 2 : 0;
    constexpr uint32_t kWaves = THREADS / 64;
    constexpr uint32_t kStage = !S4 ? kStageBytes : C ? kS4CStageBytes : kS4StageBytes;
    // One LDS array: the tables, then the workgroup's tile counter and (VERIFY)
    // its mismatch count, first bad index and bad-index list (vacc).
    __shared__ __attribute__((aligned(16))) uint8_t lds[kStage + 32 + (VERIFY ? 4 * kBadList : 0)];
    uint32_t *pool_ctr = reinterpret_cast<uint32_t *>(lds + kStage);
    uint32_t *vacc = pool_ctr + 1;
    uint32_t *exit_ctr = pool_ctr + 5;  // waves of the workgroup done
    const uint8_t *table = !S4 ? p.table : C ? p.table_s4 + hdfs_crc::kS4COff : p.table_s4;
    const int lane = int(threadIdx.x & 63u);
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave in workgroup

    // Diagnostic build only (STAMPS): per-wave s_memrealtime stamps at start,
    // after table staging and at exit, plus HW_ID / XCC_ID, written to a
    // buffer nothing else reads.  Production variants contain no stamp.
    uint64_t t_start = 0, t_staged = 0;
    if (STAMPS) t_start = __builtin_amdgcn_s_memrealtime();

    // This workgroup's equal, contiguous range of tiles [tbeg, tend).  Wave
    // wv starts on tile tbeg + wv; the LDS counter hands out the rest.
    // (QUARTER: units, 4 per tile)
    const uint64_t nunits = QUARTER ? uint64_t(SPLIT) * p.ntiles : uint64_t(p.ntiles);
    // (XCDMAP: workgroup b runs on XCD b % 8; give XCD x the contiguous ranges
    // x * G/8 .. (x + 1) * G/8 - 1)
    const uint32_t rng = XCDMAP && (gridDim.x % 8u) == 0 ? (blockIdx.x % 8u) * (gridDim.x / 8u) + blockIdx.x / 8u
                                                         : blockIdx.x;
    const uint32_t tbeg = uint32_t((nunits * rng) / gridDim.x);
    const uint32_t tend = uint32_t((nunits * (rng + 1)) / gridDim.x);
    if (threadIdx.x == 0) {
        *pool_ctr = tbeg + kWaves;
        *exit_ctr = 0;
        if (VERIFY) {
            vacc[0] = 0;
            vacc[1] = 0xffffffffu;
            vacc[2] = 0;
            vacc[3] = 0;
        }
    }
    uint32_t t = tbeg + wv;
    FastTile ft{0, 0, 0};
    uint4 v[9];  // (v[8]: the bytes after a shifted tile's window)
    uint32_t ev = 0;  // VERIFY: expected checksum fetched with the tile
    int kind = 1;     // QUARTER: what load_unit found (0 empty, 1 tile / item, 2 quarter)
    auto load_next = [&](uint32_t j) {
        if (QUARTER) {
            kind = load_unit<AUX, COMPDIAG, VERIFY, GEN, SPLIT>(p, j, lane, ft, v, ev);
        } else {
            ft = tile_at(p, j);
            load_any<AUX, COMPDIAG, VERIFY, GEN>(p, ft, lane, v, ev);
        }
    };
    // EARLY: the first tile's loads go out before the staging (their latency
    // overlaps it).  Measured slower for large batches -- 3072 waves x 8 KiB
    // in flight queue the 152 KiB staging DMA behind them -- so only the
    // small-batch kernel (compact image, 28 KiB) does it.
    if (EARLY && t < tend) load_next(t);
    // Stage the tables by LDS-DMA (1 KiB per wave instruction, no VGPRs); a
    // launch of constant runs only needs none.
    const bool tables = (p.ntiles | p.ngen | p.nseg) != 0;
    constexpr uint32_t kStageChunks = kStage / 1024u;
    // (a batch with no Z^(512 s) shift -- bpc-512 tiles only -- leaves the
    // image's Z section out: 144 of 152 chunks, compact 20 of 28)
    constexpr uint32_t kNoZChunks = !S4 ? kStageChunks : C ? uint32_t(hdfs_crc::kS4CShiftOff / 1024u)
                                                           : uint32_t(hdfs_crc::kS4ShiftOff / 1024u);
    static_assert(!S4 || kNoZChunks * 1024u == (C ? hdfs_crc::kS4CShiftOff : hdfs_crc::kS4ShiftOff),
                  "the Z section starts on a staging chunk");
    const uint32_t nstage = p.skip_z ? kNoZChunks : kStageChunks;
    if (!NOSTAGE && tables) {
        // Every workgroup copies the same chunks: start each one at a
        // different chunk (the 32 CUs of an XCD would otherwise walk the same
        // L2 lines, hence the same L2 channel, in lock step).
        const uint32_t rot = (blockIdx.x * 37u) % nstage;
        for (uint32_t i = wv; i < nstage; i += kWaves) {
            const uint32_t c = i + rot < nstage ? i + rot : i + rot - nstage;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(table + c * 1024u + 16u * uint32_t(lane)),
                (__attribute__((address_space(3))) void *)(lds + c * 1024u), 16, 0, 0);
        }
    }
    if (OVL && t < tend) load_next(t);
    __syncthreads();
    if (STAMPS) t_staged = __builtin_amdgcn_s_memrealtime();
    // (the last wave: idle in small batches; in large ones the workgroup's
    // tile pool absorbs its late start)
    if (VERIFY && blockIdx.x == 0 && wv == kWaves - 1) verify_init(p, lane);

    // Gen pairs, seg pairs and constant runs, dealt over every wave of the
    // grid after the tiles.  (Before the tiles, so that their latency-bound
    // loads would overlap the other waves' tile streaming, measured -2.8 ..
    // +1 %: not kept)
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + wv);
    const uint32_t nwaves = gridDim.x * kWaves;
    auto items = [&]() {
        const uint32_t ngp = (p.ngen + 1u) >> 1, nsp = (p.nseg + 1u) >> 1;
        const uint32_t nitems = ngp + nsp + p.nconst;
        for (uint32_t g = wave; g < nitems; g += nwaves) {
            if (g < ngp)
                gen_pair<S4, VERIFY, IMG>(p, lds, vacc, g, lane);
            else if (g < ngp + nsp)
                seg_pair<S4, VERIFY, IMG>(p, lds, vacc, g - ngp, lane);
            else
                const_run<VERIFY>(p, vacc, g - ngp - nsp, lane);
        }
    };

    if (!EARLY && !OVL && t < tend) load_next(t);
    while (t < tend) {
        if (!QUARTER || kind == 1)
            finish_tile<AUX, DIAG, COMPDIAG, S4, VERIFY, IMG, GEN>(p, lds, vacc, ft, v, ev, lane);
        else if (kind == 2)
            finish_quarter<DIAG, S4, VERIFY, IMG, SPLIT>(p, lds, vacc, ft, v, ev, lane);
        t = pool_grab(pool_ctr, lane);
        if (t >= tend) break;
        load_next(t);
    }
    items();
    if (VERIFY) {
        __syncthreads();
        verify_finish<THREADS>(p, vacc);
    }
    // The plan's completion count: the workgroup's last wave adds 1 (every
    // wave of it has finished reading the plan's memory by then).
    if (p.done_ctr) {
        uint32_t n = 0;
        if (lane == 0) n = atomicAdd(exit_ctr, 1u);
        n = __builtin_amdgcn_readfirstlane(n);
        if (n == kWaves - 1u && lane == 0)
            __hip_atomic_fetch_add(p.done_ctr + (blockIdx.x % hdfs_crc::kDoneCtrs) * (hdfs_crc::kDoneCtrStride / 8u),
                                   1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (STAMPS && lane == 0 && p.stamps) {  // (no buffer: a plan exec of a stamped variant)
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        const uint32_t hw_id = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        const uint32_t xcc_id = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID
        p.stamps[4 * wave + 0] = t_start;
        p.stamps[4 * wave + 1] = t_staged;
        p.stamps[4 * wave + 2] = t_end;
        p.stamps[4 * wave + 3] = (uint64_t(xcc_id) << 32) | hw_id;
    }
}

namespace hdfs_crc {
// Grid of a launch: one workgroup per CU, or one per work item when there
// are fewer items than CUs (a small batch leaves most waves without a tile;
// they still share the table staging, which is what bounds a small launch).
inline uint32_t production_grid(const KParams &p, uint32_t num_cu, uint32_t units_per_tile = 1) {
    const uint64_t items = uint64_t(p.ntiles) * units_per_tile + (uint64_t(p.ngen) + 1) / 2 +
                           (uint64_t(p.nseg) + 1) / 2 + p.nconst;
    return uint32_t(items < num_cu ? (items ? items : 1) : num_cu);
}
}  // namespace hdfs_crc
