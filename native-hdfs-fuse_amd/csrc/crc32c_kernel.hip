// crc32c_kernel.hip -- the CDNA4 (gfx950) CRC32C chunk kernel.
//
// Computes hadoop_rpc_send_packet's checksum vector (hadooprpc.c:733-742:
// crc32c(0, chunk) per bytesPerChecksum chunk, crc32c.c semantics) for a
// whole batch of device-resident packets in one launch.  Integer/bitwise
// work, HBM-bound; no MFMA.  Design (DESIGN.md has the derivation):
//
//  * CRC32C is affine over GF(2): for a chunk M of n bytes,
//      crc32c(0, M) = lin(M) ^ crc32c(0, zeros(n)),
//    and lin(M) is the XOR of one 32-bit contribution per (byte position,
//    byte value).  So there is no serial dependency inside a chunk.
//  * Coalesced HBM loads: one wave instruction reads 1 KiB contiguous
//    (16 B per lane) = two 512-byte blocks; lane q of each half owns bytes
//    16q .. 16q+15 of its block in EVERY instruction.
//  * The Castagnoli tables live in LDS as positional NIBBLE tables, one
//    128-byte row per nibble value with one 4-byte column per lane: the 32
//    lanes of a ds_read_b32 group always hit 32 different banks (bank =
//    column), so every lookup is conflict-free whatever the data.
//    2 lookups per byte, 64 KiB of LDS (see crc_math.h for the layout).
//  * Wave-level reduction: each lane's per-piece value is XOR-reduced over
//    the 32 lanes of its block with a DPP reduce-scatter, which also packs
//    the 16 block results of a tile into 16 lanes for one coalesced store.
//  * bpc = 1024..8192 (config 5): per-block results are shifted by
//    Z^(512*s) (nibble tables in LDS) and XORed across the blocks of a chunk.
//  * Tails / odd bpc / unaligned chunks: half a wave per chunk, the chunk is
//    right-aligned into zero-prefixed virtual 512-byte blocks (leading zeros
//    do not change lin), Horner-combined with Z^512.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernel_abi.h"

namespace {

using hdfs_crc::FastTile;
using hdfs_crc::GenItem;
using hdfs_crc::KParams;

constexpr uint32_t kLdsBytes = hdfs_crc::kKernelLdsBytes;
constexpr uint32_t kShiftOff = hdfs_crc::kKernelShiftOff;

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

__device__ __forceinline__ uint32_t lds_u32(const uint8_t *lds, uint32_t off) {
    return *reinterpret_cast<const uint32_t *>(lds + off);
}

// lin() contribution of one lane's 16-byte piece at column col (= lane & 31).
// Byte k of the piece: low nibble row at k*4096 + n*256, high nibble row at
// 128 + k*256 + n*4096; the lane's column is col*4.  Shifting the dword so
// the byte sits in bits 8..15 makes both row offsets a single v_and_or.
__device__ __forceinline__ uint32_t piece_lin(const uint8_t *lds, uint4 d, uint32_t col4) {
    uint32_t acc = 0;
    const uint32_t dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t x = dw[w];
        const uint32_t xs[4] = {x << 8, x, x >> 8, x >> 16};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const uint32_t k = 4 * w + t;
            const uint32_t lo = ((xs[t] & 0x0F00u) | col4) + k * 4096u;
            const uint32_t hi = ((xs[t] & 0xF000u) | col4) + 128u + k * 256u;
            acc ^= lds_u32(lds, lo) ^ lds_u32(lds, hi);
        }
    }
    return acc;
}

// Z^(512*s)(x), s in 1..15, from 8 nibble tables (16 entries each).
__device__ __forceinline__ uint32_t zshift(const uint8_t *lds, uint32_t s, uint32_t x) {
    const uint32_t base = kShiftOff + (s - 1u) * 512u;
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

// ---- fast path: one wave, 16 blocks of full chunks -----------------------
// Loads of one tile: instruction i reads 1 KiB contiguous (blocks 2i, 2i+1).
// Lanes of blocks a partial tile does not have re-read block 0 (always
// valid memory) and are masked out in finish_tile, so the instruction
// stream has no divergent branch and the wait counts stay exact.
__device__ __forceinline__ void load_tile(const KParams &p, FastTile t, int lane, uint4 v[8]) {
    const uint32_t nb = t.meta & 0xffu;
    const uint32_t h = uint32_t(lane) >> 5;
    const uint8_t *base = p.payload + t.src;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t off = (2u * i + h < nb) ? 1024u * i + 16u * uint32_t(lane) : 16u * uint32_t(lane & 31);
        v[i] = *reinterpret_cast<const uint4 *>(base + off);
    }
    // Keep the loads ahead of whatever compute follows (the scheduler would
    // otherwise hoist the next tile's first lookups above them and wait).
    __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void finish_tile(const KParams &p, const uint8_t *lds, FastTile t, const uint4 v[8],
                                            int lane) {
    const uint32_t nb = t.meta & 0xffu;
    const uint32_t lg = (t.meta >> 8) & 0xffu;
    const uint32_t col4 = uint32_t(lane & 31) << 2;
    const uint32_t h = uint32_t(lane) >> 5;
    uint32_t pc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        pc[i] = piece_lin(lds, v[i], col4);
        pc[i] = (2u * i + h < nb) ? pc[i] : 0u;
        // One piece at a time: keeps the scheduler from hoisting every
        // piece's 32 LDS reads together (register pressure -> spills).
        __builtin_amdgcn_sched_barrier(0);
    }

    // Reduce-scatter over lane bits 0, 1, 3 (8 values -> 1), then all-reduce
    // over lane bits 2 and 4.  Afterwards lane l holds lin() of block
    // blk = 2*i + h with i = b3 + 2*b1 + 4*b0 (b = bits of l).
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
    const uint32_t blk = 2u * ((b3 ? 1u : 0u) + (b1 ? 2u : 0u) + (b0 ? 4u : 0u)) + h;

    if (lg) {  // chunks of 2^lg blocks: shift each block to the chunk end, XOR them
        const uint32_t nbc = 1u << lg;
        const uint32_t s = nbc - 1u - (blk & (nbc - 1u));
        if (s) x = zshift(lds, s, x);
        x ^= static_cast<uint32_t>(__shfl_xor(static_cast<int>(x), 32));  // block bit 0 = lane bit 5
        if (lg >= 2) x ^= dpp<kDppXor8>(x);                               // block bit 1 = lane bit 3
        if (lg >= 3) x ^= dpp<kDppXor2>(x);                               // block bit 2 = lane bit 1
        if (lg >= 4) x ^= dpp<kDppXor1>(x);                               // block bit 3 = lane bit 0
    }
    const uint32_t crc = x ^ p.c_lg[lg];
    const bool rep = ((lane & 0x14) == 0) && ((blk & ((1u << lg) - 1u)) == 0) && blk < nb;
    if (rep) p.out[t.out + (blk >> lg)] = out_order(crc, p.flags);
}

// Grid-stride over fast tiles.  PIPE: the next tile's 8 KiB is in flight
// (and the descriptor after it requested) while the current one is
// computed, so each wave keeps HBM busy across its own compute.
template <bool PIPE>
__device__ __forceinline__ void fast_loop(const KParams &p, const uint8_t *lds, uint32_t wave, uint32_t nwaves,
                                          int lane) {
    // Tiles of this wave: wave, wave + nwaves, ... (n of them).  All loop
    // control is scalar; tile indices go through readfirstlane so the
    // compiler keeps them (and the descriptor loads) in SGPRs.
    const uint32_t n = wave < p.ntiles ? (p.ntiles - 1u - wave) / nwaves + 1u : 0u;
    auto tile_k = [&](uint32_t k) { return tile_at(p, __builtin_amdgcn_readfirstlane(wave + k * nwaves)); };
    if (!PIPE) {
        FastTile t = tile_k(0);
        for (uint32_t k = 0; k < n; ++k) {
            uint4 v[8];
            load_tile(p, t, lane, v);
            const FastTile tn = tile_k(k + 1 < n ? k + 1 : k);  // prefetch the next descriptor
            finish_tile(p, lds, t, v, lane);
            t = tn;
        }
        return;
    }
    // Two register buffers, unrolled by two so each buffer stays in its own
    // registers: the other buffer's loads are issued before a buffer is
    // computed, so its waits are vmcnt(15..8) and 8 KiB stays in flight.
    // The last one or two tiles are drained outside the loop.
    if (n == 0) return;
    uint4 va[8], vb[8];
    FastTile ta = tile_k(0);
    load_tile(p, ta, lane, va);
    uint32_t k = 0;
    FastTile tb = tile_k(n > 1 ? 1 : 0);
    while (k + 2 < n) {  // tiles k, k+1, k+2 exist
        load_tile(p, tb, lane, vb);
        const FastTile tc = tile_k(k + 2);
        finish_tile(p, lds, ta, va, lane);
        load_tile(p, tc, lane, va);
        const FastTile td = tile_k(k + 3 < n ? k + 3 : k + 2);
        finish_tile(p, lds, tb, vb, lane);
        ta = tc;
        tb = td;
        k += 2;
    }
    if (k + 1 < n) {
        load_tile(p, tb, lane, vb);
        finish_tile(p, lds, ta, va, lane);
        finish_tile(p, lds, tb, vb, lane);
    } else {
        finish_tile(p, lds, ta, va, lane);
    }
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

__device__ __forceinline__ void gen_pair(const KParams &p, const uint8_t *lds, uint32_t pair, int lane) {
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
            lin = piece_lin(lds, funnel(w, uint32_t(a & 15u)), q << 2);
        }
        lin = allreduce32(lin);
        if (m < nbv) acc = zshift(lds, 1, acc) ^ lin;
    }
    if (valid && q == 0) {
        const uint32_t crc = acc ^ (r >= 4 ? 0xffffffffu : p.c_small[r]);
        p.out[g.out] = out_order(crc, p.flags);
    }
}

}  // namespace

template <int THREADS, bool PIPE>
__global__ __launch_bounds__(THREADS, 2 * THREADS / 256) void hdfs_crc32c_plan_kernel(KParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
    {
        // Stage the tables: every load in flight before the first LDS write
        // (the device copy is zero-padded to kTableAlloc bytes, so no load
        // needs a guard).
        constexpr uint32_t kVec = kLdsBytes / 16;
        constexpr uint32_t kPer = (kVec + THREADS - 1) / THREADS;
        const uint4 *g = reinterpret_cast<const uint4 *>(p.table);
        uint4 *sm = reinterpret_cast<uint4 *>(lds);
        uint4 r[kPer];
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) r[k] = g[threadIdx.x + k * THREADS];
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k)
            if (threadIdx.x + k * THREADS < kVec) sm[threadIdx.x + k * THREADS] = r[k];
    }
    __syncthreads();
    const int lane = int(threadIdx.x & 63u);
    constexpr uint32_t kWaves = THREADS / 64;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + (threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * kWaves;
    fast_loop<PIPE>(p, lds, wave, nwaves, lane);
    const uint32_t npairs = (p.ngen + 1u) >> 1;
    for (uint32_t g = wave; g < npairs; g += nwaves) gen_pair(p, lds, g, lane);
}

namespace hdfs_crc {
const KernelVariant kVariants[kNumVariants] = {
    {"wg512_pipe", 512, true},
    {"wg512_plain", 512, false},
    {"wg1024_plain", 1024, false},
};

hipError_t launch_plan_kernel(const KParams &p, int variant, uint32_t num_cu, hipStream_t stream) {
    if (variant < 0 || variant >= kNumVariants) variant = 0;
    const KernelVariant &kv = kVariants[variant];
    const uint64_t items = uint64_t(p.ntiles) + (uint64_t(p.ngen) + 1) / 2;
    const uint64_t waves = uint64_t(kv.threads / 64);
    uint64_t grid = (items + waves - 1) / waves;
    const uint64_t cap = uint64_t(num_cu) * kKernelWgPerCu;
    if (grid > cap) grid = cap;
    if (grid == 0) grid = 1;
    switch (variant) {
    case 1:
        hipLaunchKernelGGL((hdfs_crc32c_plan_kernel<512, false>), dim3(uint32_t(grid)), dim3(512), 0, stream, p);
        break;
    case 2:
        hipLaunchKernelGGL((hdfs_crc32c_plan_kernel<1024, false>), dim3(uint32_t(grid)), dim3(1024), 0, stream, p);
        break;
    default:
        hipLaunchKernelGGL((hdfs_crc32c_plan_kernel<512, true>), dim3(uint32_t(grid)), dim3(512), 0, stream, p);
        break;
    }
    return hipGetLastError();
}
}  // namespace hdfs_crc
