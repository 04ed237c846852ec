// crc32c_kernel.hip -- the CDNA4 (gfx950) CRC32C chunk kernel.
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
//    16 bytes; 152 KiB of LDS, one workgroup per CU, 12 waves (768 threads):
//    16 waves keep 33 % more bytes in flight per CU and stream 2-3 % slower.
//    (The half-column image, kModeS4H, stages 64 KiB less and wins short
//    bursts, but its 2-way bank conflicts lose 1.7 % sustained.)
//  * Lookups, A/B variant 1: positional NIBBLE tables, one 128-byte row per
//    (byte position, nibble value), 2 lookups per byte: 32 lookups + 60 VALU
//    per 16 bytes, 72 KiB, two workgroups per CU.  The kernel is power-capped
//    (1.4 kW) when both HBM and LDS/VALU run flat out, so the 38 % fewer
//    instructions of S4 turn into clock: 44 us vs 49-51 us sustained.
//  * Wave-level reduction: each lane's per-piece value is XOR-reduced over
//    the 32 lanes of its block with a DPP reduce-scatter, which also packs
//    the 16 block results of a tile into 16 lanes for one coalesced store.
//  * bpc = 1024..8192 (config 5): per-block results are shifted by
//    Z^(512*s) (nibble tables in LDS) and XORed across the blocks of a chunk.
//  * Work distribution: each workgroup owns an equal range of 8 KiB tiles;
//    its waves pull tiles from an LDS counter (the SIMD arbiter's age
//    priority makes static per-wave assignment finish 2x apart).  A batch with
//    fewer tiles than CUs x 12 still runs one 12-wave workgroup per CU (or
//    per tile): the idle waves share the table staging.
//  * Tails / odd bpc / unaligned chunks: half a wave per chunk, the chunk is
//    right-aligned into zero-prefixed virtual 512-byte blocks (leading zeros
//    do not change lin), Horner-combined with Z^512.
//  * Verification (crc32c_plan_verify): the same kernel compares instead of
//    storing; the expected values are fetched with the tile and the last
//    workgroup publishes the launch's result (sharded ticket reduction).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernel_abi.h"

namespace {

using hdfs_crc::FastTile;
using hdfs_crc::GenItem;
using hdfs_crc::KParams;
using hdfs_crc::kShardWord;
using hdfs_crc::kTicketShards;
using hdfs_crc::kTicketWord;
using hdfs_crc::kVCountWord;
using hdfs_crc::kVFirstWord;

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

// Kernel modes (template bits).  Production = kModeS4 | kModeNt.
constexpr int kModeNt = 1;          // payload loads non-temporal (streamed once)
constexpr int kModeS4 = 2;          // slicing-by-4 chains + per-column finishing operator (S4 image)
constexpr int kModeStamps = 4;      // DIAGNOSTIC: per-wave timestamps
constexpr int kModeMemDiag = 8;     // DIAGNOSTIC, wrong results: no lookups (memory ceiling)
constexpr int kModeCompDiag = 16;   // DIAGNOSTIC, wrong results: no payload loads (compute ceiling)
constexpr int kModeNoStage = 32;    // DIAGNOSTIC (memory-only): no table staging
constexpr int kModeVerify = 64;     // read side: compare with p.expect[] instead of storing (crc32c_plan_verify)
constexpr int kModeDescPf = 128;    // A/B: next tile grabbed at load time, its descriptor prefetched (vector path)
constexpr int kModeIlp4 = 256;      // A/B: 4 pieces' lookup chains free to interleave
constexpr int kModeIlp8 = 512;      // A/B: all 8 pieces' lookup chains free to interleave
constexpr int kModePrio = 1024;     // A/B: raised wave priority from the end of the lookups to the next tile's loads
constexpr int kModeEarly = 2048;    // A/B: next tile's loads issued between the lookups and the reduce
constexpr int kModeSc0 = 4096;      // A/B: payload loads with the sc0 cache-policy bit as well
constexpr int kModeSc1 = 8192;      // A/B: payload loads with the sc1 cache-policy bit as well
constexpr int kModeXcdShift = 14;   // A/B: bits 14-15 = k: odd-XCD workgroups get k/64 less of the tiles
constexpr int kModeStageShift = 16; // DIAGNOSTIC, wrong results: bits 16-17 = s: stage only 1/2^s of the image
constexpr int kModeCompactDma = 1 << 18;  // A/B: T replica rows staged from the compacted rows (kernel_abi.h)
constexpr int kModeLdsRep = 1 << 19;      // A/B: T replica rows written by ds_write_b128 from a 4 KiB copy in LDS
constexpr int kModeTCols16 = 1 << 20;     // A/B: byte-table lookups from 16 of the 32 replica columns
constexpr int kModeTCols8 = 1 << 21;      // A/B: ... from 8
constexpr int kModeS4H = 1 << 22;         // A/B: half-column S4 image (64 KiB of T tables, 88 KiB staged)

// Work descriptors are read-only for the whole launch: reading them through
// the constant address space lets every (wave-uniform) descriptor fetch be a
// scalar s_load instead of a vector load that would join the payload loads
// on the vector-memory counter.
typedef const __attribute__((address_space(4))) FastTile *ConstTiles;

__device__ __forceinline__ FastTile tile_at(const KParams &p, uint32_t i) {
    const ConstTiles t = (ConstTiles)(p.tiles) + i;
    FastTile r;
    r.src = t->src;
    r.out = t->out;
    r.meta = t->meta;
    return r;
}

// A/B (kModeDescPf): the descriptor through the VECTOR memory path, issued
// behind a tile's payload loads so the lookups never wait for it (a scalar
// load would: lgkmcnt also counts the LDS lookups, and scalar loads return
// out of order).  Every lane loads the same 16 bytes.
__device__ __forceinline__ uint4 tile_prefetch(const KParams &p, uint32_t i) {
    return *reinterpret_cast<const uint4 *>(p.tiles + i);
}
__device__ __forceinline__ FastTile tile_from(uint4 d) {
    FastTile r;
    r.src = (uint64_t(__builtin_amdgcn_readfirstlane(d.y)) << 32) | __builtin_amdgcn_readfirstlane(d.x);
    r.out = __builtin_amdgcn_readfirstlane(d.z);
    r.meta = __builtin_amdgcn_readfirstlane(d.w);
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

// lin() contribution of one lane's 16-byte piece at column col (= lane & 31).
// Byte k of the piece: low nibble row at k*4096 + n*256, high nibble row at
// 128 + k*256 + n*4096; the lane's column is col*4.  Shifting the dword so
// the byte sits in bits 8..15 makes both row offsets a single v_and_or.
// DIAG 1 (diagnostic builds only, wrong results): the lookups are skipped.
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
    uint32_t toff;  // T1 - T0 (= T3 - T2) in bytes: 128, or 64 in the half-column image
};

__device__ __forceinline__ LaneCols lane_cols(uint32_t q) {
    return LaneCols{q << 2, (q << 2) | 65536u, (q << 2) | kS4NibOff, 128u};
}

// Half-column S4 image (A/B, kModeS4H): T0..T3 share one 256-byte row per
// byte value, 16 lane columns each (b*256 + m*64 + 4*(q & 15)), 64 KiB in
// all; the N_q and Z tables stay where the full image has them.
__device__ __forceinline__ LaneCols lane_cols_h(uint32_t q) {
    const uint32_t c4 = (q & 15u) << 2;
    return LaneCols{c4, c4 | 128u, (q << 2) | kS4NibOff, 64u};
}

// Byte j of v into address bits 8..15 and the column base's bytes 0 and 2
// into bits 0..7 and 16..23 (v_perm_b32: selectors 0-3 = bytes of the
// second operand, 4-7 = bytes of the first, 0x0C = zero).
template <int J>
__device__ __forceinline__ uint32_t byte_addr(uint32_t v, uint32_t base) {
    return __builtin_amdgcn_perm(v, base, 0x0C020000u | uint32_t(4 + J) << 8);
}

// One slicing-by-4 step: S(v) ^ next, S(v) = T3[v.b0] ^ T2[v.b1] ^ T1[v.b2]
// ^ T0[v.b3] (each table replicated over the lane columns of the image: 32,
// or 16 in the production half-column image; so the 32
// lanes of a half-wave always hit 32 different banks).
__device__ __forceinline__ uint32_t s4(const uint8_t *lds, const LaneCols &c, uint32_t v, uint32_t next) {
    const uint32_t a3 = lds_u32(lds, byte_addr<0>(v, c.hi) + c.toff);  // T3: upper pair, odd
    const uint32_t a2 = lds_u32(lds, byte_addr<1>(v, c.hi));           // T2: upper pair, even
    const uint32_t a1 = lds_u32(lds, byte_addr<2>(v, c.col4) + c.toff);  // T1
    const uint32_t a0 = lds_u32(lds, byte_addr<3>(v, c.col4));         // T0
    return xor3(xor3(a3, a2, a1), a0, next);
}

// lin() of the lane's 16-byte piece with the S4 image: u = S(S(S(d0) ^ d1)
// ^ d2) ^ d3 is the register after the piece; N_q(u) = Z_{16(31-q)}(S(u))
// moves it to the block end (8 nibble lookups in the lane's column).
template <int DIAG>
__device__ __forceinline__ uint32_t piece_lin_s4(const uint8_t *lds, uint4 d, const LaneCols &c) {
    if (DIAG == 1) return d.x ^ d.y ^ d.z ^ d.w;
    const uint32_t u = s4(lds, c, s4(lds, c, s4(lds, c, d.x, d.y), d.z), d.w);
    const uint32_t xs[8] = {u << 8, u << 4, u, u >> 4, u >> 8, u >> 12, u >> 16, u >> 20};
    uint32_t r[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) r[t] = lds_u32(lds, and_or(xs[t], 0x0F00u, c.nib) + (t >> 1) * 4096u + (t & 1) * 128u);
    return xor3(xor3(r[0], r[1], r[2]), xor3(r[3], r[4], r[5]), r[6] ^ r[7]);
}

template <bool S4, int DIAG>
__device__ __forceinline__ uint32_t piece(const uint8_t *lds, uint4 d, const LaneCols &c) {
    if (S4) return piece_lin_s4<DIAG>(lds, d, c);
    return piece_lin<DIAG>(lds, d, c.col4);
}

// Z^(512*s)(x), s in 1..15, from 8 nibble tables (16 entries each).
template <bool S4 = false>
__device__ __forceinline__ uint32_t zshift(const uint8_t *lds, uint32_t s, uint32_t x) {
    const uint32_t base = (S4 ? kS4ShiftOff : kShiftOff) + (s - 1u) * 512u;
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

// A mismatch (VERIFY): bump the workgroup's LDS count and lower its LDS
// first-bad index (vacc[0], vacc[1]; merged grid-wide by verify_finish).
__device__ __forceinline__ void mismatch(uint32_t *vacc, uint32_t idx) {
    atomicAdd(vacc, 1u);
    atomicMin(vacc + 1, idx);
}

// Checksum `idx` of the batch: stored, or (VERIFY) compared with `expect`.
template <bool VERIFY>
__device__ __forceinline__ void emit(const KParams &p, uint32_t *vacc, uint32_t idx, uint32_t crc, uint32_t expect) {
    const uint32_t v = out_order(crc, p.flags);
    if (VERIFY) {
        if (v != expect) mismatch(vacc, idx);
    } else {
        p.out[idx] = v;
    }
}

// ---- launch-wide verification state (kernel_abi.h slots) -----------------
// Start of a verification launch, one thread of workgroup 0: restore the
// OTHER slot of the pair (used by the previous launch, which has completed)
// for the next launch.
__device__ __forceinline__ void reset_next_slot(const KParams &p) {
    uint32_t *s = p.sched_next;
    atomicExch(s + kTicketWord, 0u);
    atomicExch(s + kVCountWord, 0u);
    atomicExch(s + kVFirstWord, 0xffffffffu);
#pragma unroll
    for (uint32_t i = 0; i < kTicketShards; ++i) atomicExch(s + kShardWord + 32 * i, 0u);
}

// Waits until every vector-memory operation of the wave has completed; for a
// returning device-scope atomic that means it has been performed.
__device__ __forceinline__ void wait_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// End of a verification launch, thread 0 of every workgroup: fold the
// workgroup's count / first-bad index into the slot, take a ticket, and let
// the last workgroup publish the totals to p.result[0..1] (no host-side reset
// of the result is needed).  Every word of the slot is only ever touched by
// device-scope atomics, which are performed in one place, so ordering needs
// only completion waits, no cache fences (a __threadfence() is an L2
// writeback + invalidate, ~3.5 us each on the launch's critical tail).
__device__ __forceinline__ void verify_finish(const KParams &p, const uint32_t *vacc) {
    uint32_t *s = p.sched;
    const uint32_t cnt = vacc[0], first = vacc[1];
    if (cnt) {
        uint32_t a = atomicAdd(s + kVCountWord, cnt);
        uint32_t b = atomicMin(s + kVFirstWord, first);
        asm volatile("" : "+v"(a), "+v"(b));  // returning forms: the wait below covers them
        wait_vmem();
    }
    // shard ticket, then (last of the shard) the global ticket
    const uint32_t shard = blockIdx.x % kTicketShards;
    const uint32_t shards = min(gridDim.x, kTicketShards);
    const uint32_t in_shard = (gridDim.x - shard + kTicketShards - 1u) / kTicketShards;
    if (atomicAdd(s + kShardWord + 32u * shard, 1u) != in_shard - 1u) return;
    if (atomicAdd(s + kTicketWord, 1u) == shards - 1u) {
        // every other workgroup's adds completed before its tickets
        p.result[0] = atomicAdd(s + kVCountWord, 0u);
        p.result[1] = atomicAdd(s + kVFirstWord, 0u);
    }
}

// ---- fast path: one wave, 16 blocks of full chunks -----------------------
// Block of the tile whose lin() lane `lane` holds after finish_tile's
// reduce-scatter, and whether the lane emits that block's chunk checksum.
__device__ __forceinline__ uint32_t rep_block(int lane) {
    return 2u * (((lane & 8) ? 1u : 0u) + ((lane & 2) ? 2u : 0u) + ((lane & 1) ? 4u : 0u)) + (uint32_t(lane) >> 5);
}
__device__ __forceinline__ bool rep_lane(int lane, uint32_t blk, uint32_t nb, uint32_t lg) {
    return ((lane & 0x14) == 0) && ((blk & ((1u << lg) - 1u)) == 0) && blk < nb;
}

// Loads of one tile: instruction i reads 1 KiB contiguous (blocks 2i, 2i+1)
// through a buffer descriptor whose range is the tile's nb * 512 valid
// bytes.  Lanes of blocks a partial tile does not have fall outside the range
// and read zeros without touching memory (lin() of zeros is 0, so they need
// no mask), every lane uses the same one-VGPR offset plus an immediate, and
// the instruction stream has no divergent branch.  AUX 2 = non-temporal.
// VERIFY: the expected checksum the lane compares is fetched with the tile.
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
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(p.payload + t.src), 0, int(nb * 512u), 0x00020000);
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

// lin() per piece, then reduce to one lin() per block, combine the blocks of
// each chunk, store (or compare) the chunk checksums.
// lin() of pieces I0 .. I1-1 of a tile (instruction i's 16 bytes per lane).
// GROUP > 2 (A/B): GROUP pieces' chains are left free to interleave (no
// per-piece pin, a scheduling barrier only every GROUP pieces).
template <int DIAG, bool S4, int I0, int I1, int GROUP = 2, uint32_t TCOLS = 31, bool H = false>
__device__ __forceinline__ void tile_pieces(const uint8_t *lds, const uint4 v[8], uint32_t pc[8], int lane) {
    LaneCols cols = H ? lane_cols_h(uint32_t(lane & 31)) : lane_cols(uint32_t(lane & 31));
    if (TCOLS != 31) {  // A/B: byte-table lookups from fewer replica columns (N_q keeps all 32)
        cols.col4 = (uint32_t(lane) & TCOLS) << 2;
        cols.hi = cols.col4 | 65536u;
    }
#pragma unroll
    for (int i = I0; i < I1; ++i) {
        pc[i] = piece<S4, DIAG>(lds, v[i], cols);
        if (GROUP <= 2) opaque(pc[i]);
        if (GROUP > 2) {
            if ((i + 1) % GROUP == 0) __builtin_amdgcn_sched_barrier(0);
            continue;
        }
        // One piece at a time (nibble tables: 32 independent reads each), or
        // two (S4: a piece is a chain of 4 dependent steps, so two chains
        // interleave to keep 8 reads in flight): keeps the scheduler from
        // hoisting every piece's LDS reads together (register pressure).
        if (!S4 || (i & 1)) __builtin_amdgcn_sched_barrier(0);
    }
}

template <int DIAG, bool S4, bool VERIFY>
__device__ __forceinline__ void reduce_emit(const KParams &p, const uint8_t *lds, uint32_t *vacc, FastTile t,
                                            const uint32_t pc[8], uint32_t ev, int lane);

template <int DIAG, bool S4, bool VERIFY, int GROUP = 2, uint32_t TCOLS = 31, bool H = false>
__device__ __forceinline__ void finish_tile(const KParams &p, const uint8_t *lds, uint32_t *vacc, FastTile t,
                                            const uint4 v[8], uint32_t ev, int lane) {
    uint32_t pc[8];
    tile_pieces<DIAG, S4, 0, 8, GROUP, TCOLS, H>(lds, v, pc, lane);
    reduce_emit<DIAG, S4, VERIFY>(p, lds, vacc, t, pc, ev, lane);
}

// The tile's 8 piece values -> one lin() per block, blocks combined per chunk,
// chunk checksums stored (or compared).
template <int DIAG, bool S4, bool VERIFY>
__device__ __forceinline__ void reduce_emit(const KParams &p, const uint8_t *lds, uint32_t *vacc, FastTile t,
                                            const uint32_t pc[8], uint32_t ev, int lane) {
    const uint32_t nb = t.meta & 0xffu;
    const uint32_t lg = (t.meta >> 8) & 0xffu;

    // Reduce-scatter over lane bits 0, 1, 3 (8 values -> 1), then all-reduce
    // over lane bits 2 and 4.  Afterwards lane l holds lin() of block
    // rep_block(l) = 2*i + h with i = b3 + 2*b1 + 4*b0 (b = bits of l).
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
    x ^= swz_xor<16>(x);
    const uint32_t blk = rep_block(lane);

    if (lg) {  // chunks of 2^lg blocks: shift each block to the chunk end, XOR them
        const uint32_t nbc = 1u << lg;
        const uint32_t s = nbc - 1u - (blk & (nbc - 1u));
        if (s) x = zshift<S4>(lds, s, x);
        x ^= static_cast<uint32_t>(__shfl_xor(static_cast<int>(x), 32));  // block bit 0 = lane bit 5
        if (lg >= 2) x ^= dpp<kDppXor8>(x);                               // block bit 1 = lane bit 3
        if (lg >= 3) x ^= dpp<kDppXor2>(x);                               // block bit 2 = lane bit 1
        if (lg >= 4) x ^= dpp<kDppXor1>(x);                               // block bit 3 = lane bit 0
    }
    const uint32_t crc = x ^ p.c_lg[lg];
    if (rep_lane(lane, blk, nb, lg)) emit<VERIFY>(p, vacc, t.out + (blk >> lg), crc, ev);
}

// One tile index from the workgroup's LDS counter (one ds_add_rtn per wave).
__device__ __forceinline__ uint32_t pool_grab(uint32_t *pool_ctr, int lane) {
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(pool_ctr, 1u);
    return __builtin_amdgcn_readfirstlane(t);
}

// ---- general path: half a wave per chunk of any length / alignment -------
__device__ __forceinline__ uint32_t bytes_mask(int64_t n) {
    return n >= 4 ? 0xffffffffu : (n <= 0 ? 0u : ((1u << (8 * uint32_t(n))) - 1u));
}

// Loads the aligned 16 bytes at a0 when they touch [cbeg, cend), zeroes the
// bytes outside it and XORs 0xff into the bytes inside [cbeg, ffend)
// (the register pre-inversion of crc32c.c:237 moved into the data).
__device__ __forceinline__ void load_piece(uintptr_t a0, uintptr_t cbeg, uintptr_t cend, uintptr_t ffend,
                                           uint32_t w[4]) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (a0 < cend && a0 + 16 > cbeg) v = *reinterpret_cast<const uint4 *>(a0);
    const uint32_t dv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uintptr_t d = a0 + 4u * j;
        const uint32_t lo = bytes_mask(int64_t(cbeg - d));
        const uint32_t keep = bytes_mask(int64_t(cend - d)) & ~lo;
        const uint32_t ff = bytes_mask(int64_t(ffend - d)) & ~lo;
        w[j] = (dv[j] & keep) ^ ff;
    }
}

// Bytes sh .. sh+15 of the 32 bytes w[0..7]: a two-stage dword select (by 2,
// then by 1) and v_alignbyte.  Written out as values so the compiler cannot
// turn it into an indexed scratch access.
__device__ __forceinline__ uint4 funnel(const uint32_t w[8], uint32_t sh) {
    const bool by2 = (sh & 8u) != 0, by1 = (sh & 4u) != 0;
    const uint32_t bi = sh & 3u;
    const uint32_t t0 = by2 ? w[2] : w[0], t1 = by2 ? w[3] : w[1], t2 = by2 ? w[4] : w[2];
    const uint32_t t3 = by2 ? w[5] : w[3], t4 = by2 ? w[6] : w[4], t5 = by2 ? w[7] : w[5];
    const uint32_t s0 = by1 ? t1 : t0, s1 = by1 ? t2 : t1, s2 = by1 ? t3 : t2;
    const uint32_t s3 = by1 ? t4 : t3, s4 = by1 ? t5 : t4;
    return make_uint4(__builtin_amdgcn_alignbyte(s1, s0, bi), __builtin_amdgcn_alignbyte(s2, s1, bi),
                      __builtin_amdgcn_alignbyte(s3, s2, bi), __builtin_amdgcn_alignbyte(s4, s3, bi));
}

template <bool S4, bool VERIFY, bool H = false>
__device__ __forceinline__ void gen_pair(const KParams &p, const uint8_t *lds, uint32_t *vacc, uint32_t pair,
                                         int lane) {
    const uint32_t h = uint32_t(lane) >> 5, q = uint32_t(lane) & 31u;
    const uint32_t idx = 2u * pair + h;
    const bool valid = idx < p.ngen;
    GenItem g{0, 0, 0};
    if (valid) g = p.gen[idx];
    const uint32_t r = g.len;
    const uint32_t nbv = (r + 511u) >> 9;  // virtual 512-byte blocks
    const uint32_t nmax = max(__builtin_amdgcn_readlane(nbv, 0), __builtin_amdgcn_readlane(nbv, 32));
    const int64_t pad = int64_t(nbv) * 512 - int64_t(r);
    const uintptr_t cbeg = reinterpret_cast<uintptr_t>(p.payload) + g.src;
    const uintptr_t cend = cbeg + r;
    const uintptr_t ffend = r >= 4 ? cbeg + 4 : cbeg;
    uint32_t acc = 0;
    for (uint32_t m = 0; m < nmax; ++m) {
        uint32_t lin = 0;
        if (m < nbv) {
            const int64_t o = int64_t(m) * 512 + int64_t(16 * q) - pad;  // may be negative (zero prefix)
            const uintptr_t a = cbeg + uintptr_t(o);
            const uintptr_t a0 = a & ~uintptr_t(15);
            uint32_t w[8];
            load_piece(a0, cbeg, cend, ffend, w);
            load_piece(a0 + 16, cbeg, cend, ffend, w + 4);
            lin = piece<S4, 0>(lds, funnel(w, uint32_t(a & 15u)), H ? lane_cols_h(q) : lane_cols(q));
        }
        lin = allreduce32(lin);
        if (m < nbv) acc = zshift<S4>(lds, 1, acc) ^ lin;
    }
    if (valid && q == 0) {
        const uint32_t crc = acc ^ (r >= 4 ? 0xffffffffu : p.c_small[r]);
        emit<VERIFY>(p, vacc, g.out, crc, VERIFY ? p.expect[g.out] : 0u);
    }
}

}  // namespace

// THREADS per workgroup, WPS = waves per SIMD the launch bound asks for
// (= workgroups per CU x THREADS / 256; it caps VGPRs at 512 / WPS).
template <int THREADS, int WPS, int MODE>
__global__ __launch_bounds__(THREADS, WPS) void hdfs_crc32c_plan_kernel(KParams p) {
    constexpr bool NT = (MODE & kModeNt) != 0;
    constexpr bool S4 = (MODE & kModeS4) != 0;
    constexpr bool STAMPS = (MODE & kModeStamps) != 0;
    constexpr bool COMPDIAG = (MODE & kModeCompDiag) != 0;
    constexpr int DIAG = (MODE & kModeMemDiag) ? 1 : 0;
    constexpr bool NOSTAGE = (MODE & kModeNoStage) != 0;
    constexpr bool VERIFY = (MODE & kModeVerify) != 0;
    constexpr bool DESCPF = (MODE & kModeDescPf) != 0;
    constexpr int GROUP = (MODE & kModeIlp8) ? 8 : (MODE & kModeIlp4) ? 4 : 2;
    constexpr bool PRIO = (MODE & kModePrio) != 0;
    constexpr bool EARLY = (MODE & kModeEarly) != 0;
    constexpr uint32_t TCOLS = (MODE & kModeTCols8) ? 7u : (MODE & kModeTCols16) ? 15u : 31u;
    constexpr bool H = S4 && (MODE & kModeS4H) != 0;
    constexpr int AUX = (NT ? 2 : 0) | ((MODE & kModeSc0) ? 1 : 0) | ((MODE & kModeSc1) ? 16 : 0);
    constexpr uint32_t kWaves = THREADS / 64;
    constexpr uint32_t kStage = S4 ? kS4StageBytes : kStageBytes;
    // One LDS array: the tables, then the workgroup's tile counter and (VERIFY)
    // its mismatch count and first bad index.
    constexpr bool LDSREP = S4 && (MODE & kModeLdsRep) != 0;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kStage + (LDSREP ? 1024 + 4096 : 16)];
    uint32_t *pool_ctr = reinterpret_cast<uint32_t *>(lds + kStage);
    uint32_t *vacc = pool_ctr + 1;
    const uint8_t *table = S4 ? (H ? p.table_s4 + hdfs_crc::kS4HOff : p.table_s4) : p.table;
    const int lane = int(threadIdx.x & 63u);
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave in workgroup

    // Diagnostic build only (STAMPS): per-wave s_memrealtime stamps at start,
    // after table staging and at exit, plus HW_ID / XCC_ID, written to a
    // buffer nothing else reads.  Production variants contain no stamp.
    uint64_t t_start = 0, t_staged = 0;
    if (STAMPS) t_start = __builtin_amdgcn_s_memrealtime();

    // This workgroup's equal, contiguous range of tiles [tbeg, tend).  Wave
    // wv starts on tile tbeg + wv; the LDS counter hands out the rest.
    // (A/B, XCDK > 0 and an even grid: workgroup b's share is 1 + k/64 for
    // even b, 1 - k/64 for odd b, i.e. its range starts at b + (k/64)*(b & 1)
    // shares; blocks go round-robin over the XCDs, so odd b = odd XCD.)
    constexpr uint32_t XCDK = uint32_t(MODE >> kModeXcdShift) & 3u;
    const uint32_t xk = (XCDK && !(gridDim.x & 1u)) ? XCDK : 0u;
    const uint64_t den = 64ull * gridDim.x;
    const uint32_t tbeg = uint32_t((uint64_t(p.ntiles) * (64ull * blockIdx.x + xk * (blockIdx.x & 1u))) / den);
    const uint32_t tend = uint32_t((uint64_t(p.ntiles) * (64ull * (blockIdx.x + 1) + xk * ((blockIdx.x + 1) & 1u))) / den);
    if (VERIFY && blockIdx.x == 0 && threadIdx.x == 0) reset_next_slot(p);
    if (threadIdx.x == 0) {
        *pool_ctr = tbeg + kWaves;
        if (VERIFY) {
            vacc[0] = 0;
            vacc[1] = 0xffffffffu;
        }
    }
    uint32_t t = tbeg + wv;
    FastTile ft{0, 0, 0};
    uint4 v[8];
    uint32_t ev = 0;  // VERIFY: expected checksum fetched with the tile
    // Stage the tables by LDS-DMA (1 KiB per wave instruction, no VGPRs).
    constexpr uint32_t kStageChunks = (kStage / 1024u) >> ((MODE >> kModeStageShift) & 3);
    constexpr bool CDMA = S4 && (MODE & kModeCompactDma) != 0;
    constexpr uint32_t kTChunks = uint32_t(hdfs_crc::kS4NibOff) / 1024u;  // T replica region: 128 chunks
    if (LDSREP) {
        // The T rows' 1024 values (4 KiB) and the N_q / Z tables by LDS-DMA,
        // then every 1 KiB chunk of T replicas written from the LDS copy:
        // lanes 8k..8k+7 fill row 8c + k with one ds_write_b128 each.
        uint8_t *cv = lds + kStage + 1024;
        for (uint32_t c = wv; c < 4u; c += kWaves)
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(table + hdfs_crc::kS4Compact4Off + c * 1024u +
                                                                  16u * uint32_t(lane)),
                (__attribute__((address_space(3))) void *)(cv + c * 1024u), 16, 0, 0);
        for (uint32_t c = kTChunks + wv; c < kStage / 1024u; c += kWaves)
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(table + c * 1024u + 16u * uint32_t(lane)),
                (__attribute__((address_space(3))) void *)(lds + c * 1024u), 16, 0, 0);
        __syncthreads();
        for (uint32_t c = wv; c < kTChunks; c += kWaves) {
            const uint32_t v = reinterpret_cast<const uint32_t *>(cv)[8u * c + (uint32_t(lane) >> 3)];
            *reinterpret_cast<uint4 *>(lds + c * 1024u + 16u * uint32_t(lane)) = make_uint4(v, v, v, v);
        }
    }
    for (uint32_t c = wv; !LDSREP && !NOSTAGE && c < kStageChunks; c += (H && c + kWaves >= 64u && c + kWaves < 128u) ? kWaves + 64u : kWaves) {
        // CDMA: a 1 KiB chunk of the T region is 8 replica rows of 128 B;
        // lanes 8k..8k+7 all read row 8c + k's compacted 16 B.
        const uint8_t *src = (CDMA && c < uint32_t(hdfs_crc::kS4NibOff) / 1024u)
                                 ? table + hdfs_crc::kTableAllocS4 + 16u * (8u * c + (uint32_t(lane) >> 3))
                                 : table + c * 1024u + 16u * uint32_t(lane);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                         (__attribute__((address_space(3))) void *)(lds + c * 1024u), 16, 0, 0);
    }
    __syncthreads();
    if (STAMPS) t_staged = __builtin_amdgcn_s_memrealtime();

    if (t < tend) {
        ft = tile_at(p, t);
        load_tile<AUX, COMPDIAG, VERIFY>(p, ft, lane, v, ev);
    }
    if (DESCPF) {
        // (the first tile's loads are already out)
        uint32_t tn = t < tend ? pool_grab(pool_ctr, lane) : tend;
        uint4 dn = tile_prefetch(p, tn < tend ? tn : 0u);
        while (t < tend) {
            __builtin_amdgcn_sched_barrier(0);
            finish_tile<DIAG, S4, VERIFY>(p, lds, vacc, ft, v, ev, lane);
            t = tn;
            if (t >= tend) break;
            ft = tile_from(dn);
            load_tile<AUX, COMPDIAG, VERIFY>(p, ft, lane, v, ev);
            tn = pool_grab(pool_ctr, lane);
            dn = tile_prefetch(p, tn < tend ? tn : 0u);  // unconditional: keeps vmcnt counts exact
        }
    } else if (EARLY || PRIO) {
        // A/B: the lookups free v[] before the reduce; EARLY issues the next
        // tile's loads there, PRIO lets the wave ahead of its SIMD's others
        // until those loads are out.
        while (t < tend) {
            uint32_t pc[8];
            tile_pieces<DIAG, S4, 0, 8, GROUP>(lds, v, pc, lane);
            if (PRIO) __builtin_amdgcn_s_setprio(2);
            const FastTile cur = ft;
            const uint32_t cev = ev;
            const uint32_t tn = pool_grab(pool_ctr, lane);
            if (EARLY && tn < tend) {
                ft = tile_at(p, tn);
                load_tile<AUX, COMPDIAG, VERIFY>(p, ft, lane, v, ev);
                if (PRIO) __builtin_amdgcn_s_setprio(0);
            }
            reduce_emit<DIAG, S4, VERIFY>(p, lds, vacc, cur, pc, cev, lane);
            t = tn;
            if (!EARLY && t < tend) {
                ft = tile_at(p, t);
                load_tile<AUX, COMPDIAG, VERIFY>(p, ft, lane, v, ev);
            }
            if (PRIO) __builtin_amdgcn_s_setprio(0);
        }
    } else {
        while (t < tend) {
            finish_tile<DIAG, S4, VERIFY, GROUP, TCOLS, H>(p, lds, vacc, ft, v, ev, lane);
            t = pool_grab(pool_ctr, lane);
            if (t >= tend) break;
            ft = tile_at(p, t);
            load_tile<AUX, COMPDIAG, VERIFY>(p, ft, lane, v, ev);
        }
    }

    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + wv);
    const uint32_t nwaves = gridDim.x * kWaves;
    const uint32_t npairs = (p.ngen + 1u) >> 1;
    for (uint32_t g = wave; g < npairs; g += nwaves) gen_pair<S4, VERIFY, H>(p, lds, vacc, g, lane);
    if (VERIFY) {
        __syncthreads();
        if (threadIdx.x == 0) verify_finish(p, vacc);
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
const KernelVariant kVariants[kNumVariants] = {
    {"s4_nt", 768, 1},                          // production: slicing-by-4 chains, 12 waves per CU
    {"nibble_wg1024x2_nt", 1024, 2},            // A/B: positional nibble tables, 32 waves per CU
    {"s4_wg1024x1_nt", 1024, 1},                // A/B: 0 with 16 waves per CU (round-1 production)
    {"s4_wg768x1_nt_memonly", 768, 1},          // DIAGNOSTIC: memory ceiling of 0 (no lookups)
    {"s4_wg768x1_nt_compute_only", 768, 1},     // DIAGNOSTIC: compute ceiling of 0 (no payload loads)
    {"s4_wg768x1_nt_stamps", 768, 1},           // DIAGNOSTIC: 0 with per-wave timestamps
    {"s4_wg768x1_nt_memonly_stamps", 768, 1},   // DIAGNOSTIC: 3 with per-wave timestamps
    {"s4_wg768x1_nt_memonly_nostage", 768, 1},  // DIAGNOSTIC: 3 without the table staging
    {"s4_wg768x1_nt_descpf", 768, 1},           // A/B: 0 with the next descriptor prefetched (vector path)
    {"s4_wg512x1_nt", 512, 1},                  // A/B: 0 with 8 waves per CU
    {"s4_wg768x1_nt_fixed", 768, 1},            // A/B: 0 on ceil(items / 12) workgroups (concentrated)
    {"s4_nt_shapes", 768, 1},                   // A/B: 0 with 8/4/2/1 waves per workgroup for small batches
    {"s4_wg512x1_nt_memonly", 512, 1},          // DIAGNOSTIC: memory ceiling of 9 (8 waves, 64 KiB in flight)
    {"s4_ilp4_wg512x1_nt", 512, 1},             // A/B: 8 waves, 4 chains free to interleave
    {"s4_ilp8_wg512x1_nt", 512, 1},             // A/B: 8 waves, 8 chains free to interleave
    {"s4_ilp4_wg768x1_nt", 768, 1},             // A/B: 12 waves, 4 chains free to interleave
    {"s4_prio_wg768x1_nt", 768, 1},             // A/B: 0 with raised priority from the lookups' end to the next loads
    {"s4_early_wg768x1_nt", 768, 1},            // A/B: 0 with the next tile's loads issued before the reduce
    {"s4_early_prio_wg768x1_nt", 768, 1},       // A/B: 17 + 16
    {"s4_nt_sc0", 768, 1},                      // A/B: 0 with payload loads sc0 | nt
    {"s4_nt_sc1", 768, 1},                      // A/B: 0 with payload loads sc1 | nt
    {"s4_nt_sc0_sc1", 768, 1},                  // A/B: 0 with payload loads sc0 | sc1 | nt
    {"s4_nt_xcd1", 768, 1},                     // A/B: 0 with odd-XCD workgroups given 1/64 fewer tiles
    {"s4_nt_xcd2", 768, 1},                     // A/B: ... 2/64
    {"s4_nt_xcd3", 768, 1},                     // A/B: ... 3/64
    {"s4_nt_stamps_halfstage", 768, 1},         // DIAGNOSTIC: 5 staging half the image (wrong results)
    {"s4_nt_stamps_quarterstage", 768, 1},      // DIAGNOSTIC: 5 staging a quarter of the image (wrong results)
    {"s4_nt_cdma", 768, 1},                     // A/B: 0 with T replica rows staged from compacted rows
    {"s4_nt_cdma_stamps", 768, 1},              // DIAGNOSTIC: 27 with per-wave timestamps
    {"s4_nt_ldsrep", 768, 1},                   // A/B: 0 with T replicas written from a 4 KiB LDS copy
    {"s4_nt_ldsrep_stamps", 768, 1},            // DIAGNOSTIC: 29 with per-wave timestamps
    {"s4_wg704x1_nt", 704, 1},                  // A/B: 0 with 11 waves per CU
    {"s4_wg832x1_nt", 832, 1},                  // A/B: 0 with 13 waves per CU
    {"s4_nt_tcols16", 768, 1},                  // A/B: 0 with byte-table lookups from 16 replica columns
    {"s4_nt_tcols8", 768, 1},                   // A/B: 0 with byte-table lookups from 8 replica columns
    {"s4h_nt", 768, 1},                         // A/B: 0 with the half-column image (88 KiB staged)
    {"s4h_nt_stamps", 768, 1},                  // DIAGNOSTIC: 35 with per-wave timestamps
};

#define HDFS_LAUNCH(T, W, M) hipLaunchKernelGGL((hdfs_crc32c_plan_kernel<T, W, M>), g, b, 0, stream, p)

namespace {
constexpr int kS4Nt = kModeS4 | kModeNt;

// Production grid: one 12-wave workgroup per CU, or one per work item when
// there are fewer items than CUs.  A small batch leaves most waves without a
// tile; they still share the table staging, which is what bounds a small
// launch (one wave alone issues 152 LDS-DMA instructions).
template <int M>
hipError_t launch_production(const KParams &p, uint64_t items, uint32_t num_cu, hipStream_t stream) {
    const uint64_t grid = items < num_cu ? (items ? items : 1) : num_cu;
    const dim3 g{uint32_t(grid), 1, 1}, b{768, 1, 1};
    HDFS_LAUNCH(768, 3, M);
    return hipGetLastError();
}

// A/B (variant 11): waves per workgroup by batch size, 12 or the largest of
// 8 / 4 / 2 / 1 that still gives every CU one item per wave.
uint32_t shape_waves(uint64_t items, uint32_t num_cu) {
    if (items >= uint64_t(12) * num_cu) return 12;
    for (uint32_t w : {8u, 4u, 2u})
        if (items >= uint64_t(w) * num_cu) return w;
    return 1;
}

template <int M>
hipError_t launch_shapes(const KParams &p, uint64_t items, uint32_t num_cu, hipStream_t stream) {
    const uint32_t w = shape_waves(items, num_cu);
    uint64_t grid = (items + w - 1) / w;
    if (grid > num_cu) grid = num_cu;
    if (grid == 0) grid = 1;
    const dim3 g{uint32_t(grid), 1, 1}, b{w * 64u, 1, 1};
    switch (w) {
    case 12: HDFS_LAUNCH(768, 3, M); break;
    case 8: HDFS_LAUNCH(512, 2, M); break;
    case 4: HDFS_LAUNCH(256, 1, M); break;
    case 2: HDFS_LAUNCH(128, 1, M); break;
    default: HDFS_LAUNCH(64, 1, M); break;
    }
    return hipGetLastError();
}
}  // namespace

hipError_t launch_plan_kernel(const KParams &p, int variant, uint32_t num_cu, hipStream_t stream) {
    if (variant < 0 || variant >= kNumVariants) variant = 0;
    const KernelVariant &kv = kVariants[variant];
    const uint64_t items = uint64_t(p.ntiles) + (uint64_t(p.ngen) + 1) / 2;
    if (variant == 0) {
        if (p.expect) {
            if (!p.result || !p.sched || !p.sched_next) return hipErrorInvalidValue;
            return launch_production<kS4Nt | kModeVerify>(p, items, num_cu, stream);
        }
        return launch_production<kS4Nt>(p, items, num_cu, stream);
    }
    if (variant == 11 && !p.expect) return launch_shapes<kS4Nt>(p, items, num_cu, stream);
    const uint64_t waves = uint64_t(kv.threads / 64);
    uint64_t grid = (items + waves - 1) / waves;
    const uint64_t cap = uint64_t(num_cu) * kv.wg_per_cu;
    if (grid > cap) grid = cap;
    if (grid == 0) grid = 1;
    const dim3 g{uint32_t(grid), 1, 1}, b{kv.threads, 1, 1};
    if (p.expect) {  // verification: the A/B kernels 1 and 2 also have a compare mode
        if (!p.result || !p.sched || !p.sched_next) return hipErrorInvalidValue;
        switch (variant) {
        case 1: HDFS_LAUNCH(1024, 8, kModeNt | kModeVerify); break;
        case 2: HDFS_LAUNCH(1024, 4, kS4Nt | kModeVerify); break;
        default: return hipErrorInvalidValue;  // diagnostic variants do not verify
        }
        return hipGetLastError();
    }
    switch (variant) {
    case 1: HDFS_LAUNCH(1024, 8, kModeNt); break;
    case 2: HDFS_LAUNCH(1024, 4, kS4Nt); break;
    case 3: HDFS_LAUNCH(768, 3, kS4Nt | kModeMemDiag); break;
    case 4: HDFS_LAUNCH(768, 3, kS4Nt | kModeCompDiag); break;
    case 5: HDFS_LAUNCH(768, 3, kS4Nt | kModeStamps); break;
    case 6: HDFS_LAUNCH(768, 3, kS4Nt | kModeMemDiag | kModeStamps); break;
    case 7: HDFS_LAUNCH(768, 3, kS4Nt | kModeMemDiag | kModeNoStage); break;
    case 8: HDFS_LAUNCH(768, 3, kS4Nt | kModeDescPf); break;
    case 9: HDFS_LAUNCH(512, 2, kS4Nt); break;
    case 12: HDFS_LAUNCH(512, 2, kS4Nt | kModeMemDiag); break;
    case 13: HDFS_LAUNCH(512, 2, kS4Nt | kModeIlp4); break;
    case 14: HDFS_LAUNCH(512, 2, kS4Nt | kModeIlp8); break;
    case 15: HDFS_LAUNCH(768, 3, kS4Nt | kModeIlp4); break;
    case 16: HDFS_LAUNCH(768, 3, kS4Nt | kModePrio); break;
    case 17: HDFS_LAUNCH(768, 3, kS4Nt | kModeEarly); break;
    case 18: HDFS_LAUNCH(768, 3, kS4Nt | kModeEarly | kModePrio); break;
    case 19: HDFS_LAUNCH(768, 3, kS4Nt | kModeSc0); break;
    case 20: HDFS_LAUNCH(768, 3, kS4Nt | kModeSc1); break;
    case 21: HDFS_LAUNCH(768, 3, kS4Nt | kModeSc0 | kModeSc1); break;
    case 22: HDFS_LAUNCH(768, 3, kS4Nt | (1 << kModeXcdShift)); break;
    case 23: HDFS_LAUNCH(768, 3, kS4Nt | (2 << kModeXcdShift)); break;
    case 24: HDFS_LAUNCH(768, 3, kS4Nt | (3 << kModeXcdShift)); break;
    case 25: HDFS_LAUNCH(768, 3, kS4Nt | kModeStamps | (1 << kModeStageShift)); break;
    case 26: HDFS_LAUNCH(768, 3, kS4Nt | kModeStamps | (2 << kModeStageShift)); break;
    case 27: HDFS_LAUNCH(768, 3, kS4Nt | kModeCompactDma); break;
    case 28: HDFS_LAUNCH(768, 3, kS4Nt | kModeCompactDma | kModeStamps); break;
    case 29: HDFS_LAUNCH(768, 3, kS4Nt | kModeLdsRep); break;
    case 30: HDFS_LAUNCH(768, 3, kS4Nt | kModeLdsRep | kModeStamps); break;
    case 31: HDFS_LAUNCH(704, 3, kS4Nt); break;
    case 32: HDFS_LAUNCH(832, 4, kS4Nt); break;
    case 33: HDFS_LAUNCH(768, 3, kS4Nt | kModeTCols16); break;
    case 34: HDFS_LAUNCH(768, 3, kS4Nt | kModeTCols8); break;
    case 35: HDFS_LAUNCH(768, 3, kS4Nt | kModeS4H); break;
    case 36: HDFS_LAUNCH(768, 3, kS4Nt | kModeS4H | kModeStamps); break;
    default: HDFS_LAUNCH(768, 3, kS4Nt); break;  // 10
    }
    return hipGetLastError();
}
#undef HDFS_LAUNCH
}  // namespace hdfs_crc
