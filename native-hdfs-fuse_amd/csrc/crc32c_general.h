// crc32c_general.h -- general items of the CRC32C kernel (any bpc in
// [4, 8192] outside 512 * 2^k, and packet tails riding behind full chunks):
// geometry, per-subtile block masks, loads, chunk-start masks and the
// subtile loop with its prefix gather.  Internal to crc32c_device.h, which
// includes it after the lookup, reduce and tile helpers it builds on.
#pragma once

namespace hdfs_crc_dev {

// General item geometry (plan.h general_meta): nch <= 16 full chunks of
// bpc bytes (k virtual 512-byte blocks each, the data right-aligned behind
// pad leading zeros), then optionally a tail chunk of tl bytes (kt blocks,
// padt leading zeros) right after them.  Its nb = nch k + kt virtual blocks
// are processed as ceil(nb / 16) subtiles of 16 blocks, one after another
// by one wave, so a chunk may span two subtiles and no block slot is left
// empty between chunks.
struct GShape {
    uint32_t k, nch, pad, bpc, tl, kt, padt, nfb, nb;
    uint64_t src;  // payload offset of the first chunk
};
__device__ __forceinline__ GShape gshape(FastTile t) {
    GShape g;
    g.k = (t.meta >> 8) & 31u;
    g.nch = (t.meta >> 13) & 31u;
    g.pad = (t.meta >> 18) & 511u;
    g.bpc = g.k * 512u - g.pad;
    g.tl = uint32_t(t.src >> 48);
    g.kt = (g.tl + 511u) >> 9;
    g.padt = g.kt * 512u - g.tl;
    g.nfb = g.nch * g.k;
    g.nb = g.nfb + g.kt;
    g.src = t.src & hdfs_crc::kSrcMask;
    return g;
}

// Patterns of whole chunks of k blocks over 16 block slots, the first slot
// being block phi (< k) of a chunk: start bit b = ((b + phi) % k == 0),
// nibble b of dist = k - 1 - (b + phi) % k (the block's distance from its
// chunk's end: the Z^512 power it is shifted by); mod16[k] = 16 % k.
struct GPatterns {
    uint64_t dist[17][16];
    uint32_t start[17][16];
    uint32_t mod16[17];
    constexpr GPatterns() : dist(), start(), mod16() {
        for (int k = 1; k <= 16; ++k) {
            mod16[k] = uint32_t(16 % k);
            for (int phi = 0; phi < k; ++phi)
                for (int b = 0; b < 16; ++b) {
                    dist[k][phi] |= uint64_t(k - 1 - (b + phi) % k) << (4 * b);
                    if ((b + phi) % k == 0) start[k][phi] |= 1u << b;
                }
        }
    }
};
__constant__ const GPatterns kGPat{};

__device__ __forceinline__ uint32_t low_bits(uint32_t n) { return (1u << n) - 1u; }  // n <= 16
__device__ __forceinline__ uint64_t low_nibbles(uint32_t n) { return n >= 16 ? ~0ull : (1ull << (4 * n)) - 1ull; }

// Wave-uniform facts of subtile s (blocks 16 s .. 16 s + 15 of the item),
// one bit or nibble per block, computed on the scalar unit from the
// descriptor and the running state of the subtiles before it; lanes only
// select their block's bit.
struct GSub {
    uint32_t sfull;   // bit b: block starts a full chunk
    uint32_t start;   // ... or the tail chunk
    uint32_t tailm;   // bit b: block of the tail chunk
    uint32_t valid;   // bit b: block < nb
    uint32_t before;  // full chunks started before the subtile
    uint64_t dist;    // nibble b: blocks to the chunk's end
};
struct GState {
    uint32_t before = 0;  // full chunks started in earlier subtiles
    uint32_t phi = 0;     // (16 s) % k
};
__device__ __forceinline__ GSub gsub(const GShape &g, uint32_t s, const GState &st) {
    GSub r;
    const uint32_t base = 16u * s;
    const uint32_t nf = g.nfb > base ? min(g.nfb - base, 16u) : 0u;
    const uint32_t nv = g.nb > base ? min(g.nb - base, 16u) : 0u;
    r.valid = low_bits(nv);
    r.sfull = kGPat.start[g.k][st.phi] & low_bits(nf);
    r.tailm = r.valid & ~low_bits(nf);
    r.start = r.sfull;
    r.dist = kGPat.dist[g.k][st.phi] & low_nibbles(nf);
    if (g.kt) {
        const uint32_t tr = g.nfb - base;  // the tail's first block (wraps when it began in an earlier subtile)
        if (tr < 16u) r.start |= 1u << tr;
        // tail block b: nb - 1 - base - b blocks to its end; kDesc has nibble b = 15 - b
        constexpr uint64_t kDesc = 0x0123456789ABCDEFull;
        const int e = min(max(int(g.nb) - 1 - int(base), 0), 30);  // the tail's last block, local (clamped)
        const uint64_t pat = e <= 15 ? kDesc >> (4 * (15 - e)) : kDesc << (4 * (e - 15));
        r.dist |= pat & low_nibbles(nv) & ~low_nibbles(nf);
    }
    r.before = st.before;
    return r;
}
__device__ __forceinline__ void gstate_next(const GShape &g, const GSub &gs, GState &st) {
    st.before += __builtin_popcount(gs.sfull);
    st.phi += kGPat.mod16[g.k];
    if (st.phi >= g.k) st.phi -= g.k;
}

// Loads of subtile s of a general item: lane q of block b = 2i + h reads
// bytes 512 (16 s + b) + 16 q - D .. +15 of the item, D = pad x (full chunks
// started at or before the block) + (padt in the tail chunk): the virtual
// blocks of chunk c start pad_c bytes before c's data.  The descriptor covers
// [src - 16, src + nch * bpc + tl) (from src when no chunk is padded: then
// the blocks are contiguous and load like a power-of-two tile's).  Lanes
// wholly inside a chunk's zero prefix, or past the last chunk, read zeros
// without touching memory; the straddling lane's bytes before the chunk are
// masked in gsub_pieces.
template <int AUX, bool COMPDIAG>
__device__ __forceinline__ void load_gsub(const uint8_t *payload, const GShape &g, const GSub &gs, uint32_t s,
                                          int lane, uint4 v[8]) {
    if (COMPDIAG) {  // synthetic data, no memory traffic
        const uint32_t x = uint32_t(g.src) * 2654435761u + s * 97u + uint32_t(lane) * 40503u;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = make_uint4(x ^ i, x + i, x * 3u + i, x ^ (i << 16));
        return;
    }
    const uint32_t bytes = g.nch * g.bpc + g.tl;
    if (g.pad == 0 && g.padt == 0) {
        const __amdgpu_buffer_rsrc_t rsrc =
            uniform_rsrc(payload + g.src, bytes);
        const uint32_t voff = 8192u * s + 16u * uint32_t(lane);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const auto r = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + 1024u * i, 0, AUX);
            v[i] = make_uint4(r[0], r[1], r[2], r[3]);
        }
        __builtin_amdgcn_sched_barrier(0);
        return;
    }
    const uint32_t shift = 16u;
    const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(payload + g.src - shift, shift + bytes);
    const uint32_t h = uint32_t(lane) >> 5, q = uint32_t(lane) & 31u;
    const uint32_t upto = 2u << h;  // (upto << 2i) - 1: blocks 0 .. b
    const uint32_t sth = gs.start >> h, vh = gs.valid >> h, th = gs.tailm >> h;
    const uint32_t qs = 16u * q + 16u;
    const uint32_t base = shift + 8192u * s + 16u * uint32_t(lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const bool tail = (th >> (2 * i)) & 1u;
        const uint32_t pc = tail ? g.padt : g.pad;
        // (unpadded full chunks: only the tail is offset)
        const uint32_t d = (g.pad ? g.pad * (gs.before + __builtin_popcount(gs.sfull & ((upto << (2 * i)) - 1u)))
                                  : 0u) +
                           (tail ? g.padt : 0u);
        const bool skip = !((vh >> (2 * i)) & 1u) || (((sth >> (2 * i)) & 1u) && qs <= pc);
        // (bit 31: past any descriptor range -- arithmetic, so no branch around the offset math)
        const uint32_t voff = (base + 1024u * i - d) | (uint32_t(skip) << 31);
        const auto r = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, 0, AUX);
        v[i] = make_uint4(r[0], r[1], r[2], r[3]);
    }
    __builtin_amdgcn_sched_barrier(0);
}

// Where a tile's loads go, a general item only fetches (VERIFY) the expected
// checksums of its chunks: its subtiles are loaded inside finish_gtile's
// loop, so the loaded registers are not carried around that loop (copying
// them would wait for all 8 loads before the first lookup).
template <bool VERIFY>
__device__ __forceinline__ void load_gtile(const KParams &p, FastTile t, int lane, uint32_t &ev) {
    const GShape g = gshape(t);
    if (VERIFY && uint32_t(lane) < g.nch + (g.kt ? 1u : 0u)) ev = p.expect[t.out + uint32_t(lane)];
}

// Bytes of a dword with index < n (n clamped to 0..4).
__device__ __forceinline__ uint32_t bytes_mask(int64_t n) {
    return n >= 4 ? 0xffffffffu : (n <= 0 ? 0u : ((1u << (8 * uint32_t(n))) - 1u));
}

// (GenItems and SegItems, crc32c_items.h) Chunk bytes before position 0 of
// the lane's dwords -> 0, chunk bytes 0..3 ^= 0xff (the register
// pre-inversion of crc32c.c:237 moved into the data).  m = position in the
// lane's 16 bytes where the chunk starts (may be < 0).  Dword j's bytes with
// index < m - 4 j is M_j = 0xffffffff >> (32 - 8 c), c = clamp(m - 4 j, 0,
// 4): one 64-bit shift of 0x00000000ffffffff by clamp(32 - 8 (m - 4 j), 0,
// 32).  Dword k keeps its bytes outside M_k and XORs 0xff into M_{k-1} &
// ~M_k (the bytes m .. m + 3): ~M_k & (w ^ M_{k-1}), one v_bitop3.
__device__ __forceinline__ uint32_t bytes_below(int s) {  // s = 32 - 8 (m - 4 j), any value
    const int c = min(max(s, 0), 32);
    return uint32_t(0xffffffffull >> c);
}
__device__ __forceinline__ uint4 chunk_start_mask(uint4 d, int m) {
    const int s = 32 - 8 * m;
    const uint32_t mm1 = bytes_below(s - 32), m0 = bytes_below(s), m1 = bytes_below(s + 32),
                   m2 = bytes_below(s + 64), m3 = bytes_below(s + 96);
    return make_uint4(~m0 & (d.x ^ mm1), ~m1 & (d.y ^ m0), ~m2 & (d.z ^ m1), ~m3 & (d.w ^ m2));
}

// Keep masks of a lane's 16-byte piece whose chunk starts at position m of
// it (m may be < 0 or > 15): dword j keeps its bytes with index >= m - 4 j,
// i.e. K_j = ~(0xffffffff >> clamp(32 - 8 (m - 4 j), 0, 32)).  Chunk bytes
// before position 0 are the zero prefix of the chunk's first virtual block
// (leading zeros do not change lin; crc = lin ^ crc(0, zeros(n)) for a chunk
// of n bytes, so no pre-inversion needs to reach the data).
__device__ __forceinline__ uint32_t keep_from(int s) { return ~bytes_below(s); }
__device__ __forceinline__ uint4 keep_masks(int m) {
    const int s = 32 - 8 * m;
    return make_uint4(keep_from(s), keep_from(s + 32), keep_from(s + 64), keep_from(s + 96));
}
// x & (K | ~f) per dword (one v_bitop3 each): the masks apply where f = ~0.
__device__ __forceinline__ void apply_keep(uint4 &x, const uint4 &k, uint32_t f) {
    x.x &= k.x | ~f;
    x.y &= k.y | ~f;
    x.z &= k.z | ~f;
    x.w &= k.w | ~f;
}

// General subtile pieces: the bytes before a chunk's start in its first
// block are zeroed.  The chunk starts at position pad_c - 16 q of lane q's
// piece of the chunk's first block; every full chunk has the same pad, so
// the lane's keep masks kp (keep_masks(pad - 16 q)) are computed once per
// item and a piece only selects them by its block's start bit (5 VALU).  The
// tail chunk (at most one start per item) takes its own masks in the piece
// row that holds its first block (a wave-uniform branch).  Unpadded items
// (bpc = 512 k, tail a multiple of 512) need nothing.
template <int DIAG, bool S4, int IMG>
__device__ __forceinline__ void gsub_pieces(const uint8_t *lds, const GShape &g, const GSub &gs, const uint4 &kp,
                                            uint4 v[8], uint32_t pc[8], int lane) {
    if (DIAG & 4) {  // DIAGNOSTIC (debug variants only, wrong results): no chunk-start masks
        tile_pieces<DIAG, S4, IMG>(lds, v, pc, lane, NoPrep{});
        return;
    }
    const uint32_t h = uint32_t(lane) >> 5, q = uint32_t(lane) & 31u;
    const uint32_t tst = g.padt ? gs.start & gs.tailm : 0u;  // the tail's first block (uniform)
    const uint32_t tsh = tst >> h;
    const int mt = int(g.padt) - int(16u * q);
    if (g.pad) {
        const uint32_t sfh = gs.sfull >> h;
        tile_pieces<DIAG, S4, IMG>(lds, v, pc, lane, [&](int i, uint4 &x) {
            apply_keep(x, kp, 0u - ((sfh >> (2 * i)) & 1u));
            if ((tst >> (2 * i)) & 3u)  // (uniform)
                apply_keep(x, keep_masks(mt), 0u - ((tsh >> (2 * i)) & 1u));
        });
    } else if (g.padt) {
        // Only the tail chunk is padded (a power-of-two or 512 k packet with a short tail).
        tile_pieces<DIAG, S4, IMG>(lds, v, pc, lane, [&](int i, uint4 &x) {
            if ((tst >> (2 * i)) & 3u) apply_keep(x, keep_masks(mt), 0u - ((tsh >> (2 * i)) & 1u));
        });
    } else {
        tile_pieces<DIAG, S4, IMG>(lds, v, pc, lane, NoPrep{});
    }
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_zero(uint32_t v) {  // lanes without a source read 0
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, 0xF, 0xF, true));
}

// A general item: for every subtile the power-of-two reduce-scatter gives
// each block's lin (block_lin); the blocks are permuted into block order
// (one ds_bpermute) and gathered, subtile s into 16-lane row s mod GROUP, so
// with GROUP = 4 one 64-lane vector holds up to 4 subtiles' 64 blocks.  Per
// group of GROUP subtiles (or the item's last, partial group): block b is shifted by
// Z^(512 dist_b) to its chunk's end (one nibble-table application for all
// 64 blocks), prefix-XORed over the 64 lanes (DPP row_shr within rows, then
// row_bcast across them), and lane c adds the XOR of its chunk's blocks in
// the group as P[hi - 1] ^ P[lo - 1].  After the last group lane c holds
// chunk c's lin, and crc = lin ^ crc(0, zeros(n)) for its n bytes.  GROUP
// = 1 is round 3's per-subtile gather (each block shifted before the
// permute, a prefix per 16-lane row).  The general-tiles-only build takes
// GROUP = 4 (bpc 1536: 49.6 -> 48.1 us), the builds with both paths GROUP =
// 2 (padded chunks, two subtiles per item when k divides 16: bpc 700 72.1
// -> 69.7 us, bpc 1000 58.1 -> 57.3; with 4, bpc 1000's verify had run
// 61.8 -> 63.5).  Each subtile's loads are issued
// after the previous one's lookups.
// (returns lane c's chunk checksum, defined for c < the item's chunks;
// payload / table_s4 as in KParams: also the resident kernel's)
template <int AUX, int DIAG, bool COMPDIAG, bool S4, int IMG, uint32_t GROUP = 1, bool HOIST = false>
__device__ __forceinline__ uint32_t gtile_crc(const uint8_t *payload, const uint8_t *table_s4, const uint8_t *lds,
                                              FastTile t, uint4 v[8], int lane) {
    const GShape g = gshape(t);
    const uint32_t c = uint32_t(lane);
    const uint32_t nout = g.nch + (g.kt ? 1u : 0u);
    // lane c's chunk: virtual blocks [lo, hi)
    const uint32_t lo = c < g.nch ? c * g.k : g.nfb;
    const uint32_t hi = c < g.nch ? lo + g.k : (c < nout ? g.nb : lo);
    const uint32_t from = block_lane(uint32_t(lane) & 15u) << 2;
    const uint32_t row = uint32_t(lane) >> 4, col = uint32_t(lane) & 15u;
    const uint32_t nsub = (g.nb + 15u) >> 4;
    // lane c's affine constant crc(0, zeros(n)), n = bpc or tl (scalar loads)
    typedef const __attribute__((address_space(4))) uint32_t *ConstU32;
    const ConstU32 zc = (ConstU32)(table_s4 + hdfs_crc::kZeroCrcOff);
    const uint32_t cf = zc[g.bpc], ct = zc[g.tl];
    const uint4 kp = keep_masks(int(g.pad) - int(16u * (uint32_t(lane) & 31u)));
    GState st;
    uint32_t acc = 0;
    uint32_t comb = 0;  // row r: subtile 4 q + r's blocks, in block order
    uint32_t shv = 0;   // ... and each block's distance to its chunk's end
    // (HOIST, the both-paths build: subtile s + 1's facts are computed right
    // after subtile s's loads are issued, so their scalar loads overlap its
    // lookups and a padded subtile's loads need not wait for them; the
    // general-tiles-only build measured 0.1-0.7 % slower with it, round 5)
    GSub gsn = HOIST ? gsub(g, 0, st) : GSub{};
    for (uint32_t s = 0; s < nsub; ++s) {
        // Unpadded items' loads need no block facts: issue them before the
        // subtile's pattern-table fetches (two dependent scalar loads).
        const bool contiguous = COMPDIAG || (g.pad == 0 && g.padt == 0);
        if (contiguous) load_gsub<AUX, COMPDIAG>(payload, g, GSub{}, s, lane, v);
        const GSub gs = HOIST ? gsn : gsub(g, s, st);
        if (!contiguous) load_gsub<AUX, COMPDIAG>(payload, g, gs, s, lane, v);
        if (HOIST) {
            gstate_next(g, gs, st);
            if (s + 1u < nsub) gsn = gsub(g, s + 1u, st);
        }
        uint32_t pc[8];
        gsub_pieces<DIAG, S4, IMG>(lds, g, gs, kp, v, pc, lane);
        const uint32_t x = block_lin(pc, lane);
        if (!HOIST) gstate_next(g, gs, st);
        if (DIAG & 2) {  // DIAGNOSTIC (debug variants only, wrong results): no per-subtile gather
            acc ^= x;
            continue;
        }
        if constexpr (GROUP == 1) {  // round 3's form: shift, then permute, per subtile
            const uint32_t blk = rep_block(lane);
            const uint32_t half = blk < 8u ? uint32_t(gs.dist) : uint32_t(gs.dist >> 32);
            const uint32_t sh = __builtin_amdgcn_ubfe(half, 4u * (blk & 7u), 4u);
            uint32_t xs = x;
            if (sh) xs = zshift<S4, IMG>(lds, sh, xs);
            uint32_t y = uint32_t(__builtin_amdgcn_ds_bpermute(int(from), int(xs)));  // lane l: block l & 15
            y ^= dpp_zero<0x111>(y);  // row_shr:1
            y ^= dpp_zero<0x112>(y);  // row_shr:2
            y ^= dpp_zero<0x114>(y);  // row_shr:4
            y ^= dpp_zero<0x118>(y);  // row_shr:8: lane l holds blocks 0 .. l & 15
            const int base = int(16u * s);
            const int l1 = min(max(int(lo) - base, 0), 16), h1 = min(max(int(hi) - base, 0), 16);
            const uint32_t ph = uint32_t(__builtin_amdgcn_ds_bpermute((max(h1, 1) - 1) << 2, int(y)));
            const uint32_t pl = uint32_t(__builtin_amdgcn_ds_bpermute((max(l1, 1) - 1) << 2, int(y)));
            if (h1 > l1) acc ^= ph ^ (l1 ? pl : 0u);
            continue;
        }
        const uint32_t r = s % GROUP;  // (uniform)
        const uint32_t y = uint32_t(__builtin_amdgcn_ds_bpermute(int(from), int(x)));  // lane l: block l & 15
        if (row == r) {
            comb = y;
            shv = __builtin_amdgcn_ubfe(col < 8u ? uint32_t(gs.dist) : uint32_t(gs.dist >> 32), 4u * (col & 7u), 4u);
        }
        if (r != GROUP - 1u && s + 1u != nsub) continue;
        // the group: subtiles 4 q .. s, blocks [64 q, 64 q + 16 (r + 1)); rows past r hold zeros
        uint32_t z = comb;
        if (shv) z = zshift<S4, IMG>(lds, shv, z);
        z ^= dpp_zero<0x111>(z);  // row_shr:1
        z ^= dpp_zero<0x112>(z);  // row_shr:2
        z ^= dpp_zero<0x114>(z);  // row_shr:4
        z ^= dpp_zero<0x118>(z);  // row_shr:8: lane l holds its row's blocks 0 .. l & 15
        // row_bcast:15 -- rows 1 and 3 add the last lane of rows 0 and 2;
        // row_bcast:31 -- rows 2 and 3 add lane 31 (rows 0 and 1 in all)
        z ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(z), 0x142, 0xA, 0xF, false));
        if (GROUP > 2)
            z ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(z), 0x143, 0xC, 0xF, false));
        const int base = int(16u * GROUP * (s / GROUP)), span = int(16u * GROUP);
        const int l1 = min(max(int(lo) - base, 0), span), h1 = min(max(int(hi) - base, 0), span);
        const uint32_t ph = uint32_t(__builtin_amdgcn_ds_bpermute((max(h1, 1) - 1) << 2, int(z)));
        const uint32_t pl = uint32_t(__builtin_amdgcn_ds_bpermute((max(l1, 1) - 1) << 2, int(z)));
        if (h1 > l1) acc ^= ph ^ (l1 ? pl : 0u);
        comb = 0;
        shv = 0;
    }
    return acc ^ (c < g.nch ? cf : ct);
}

template <int AUX, int DIAG, bool COMPDIAG, bool S4, bool VERIFY, int IMG, uint32_t GROUP = 1, bool HOIST = false>
__device__ __forceinline__ void finish_gtile(const KParams &p, const uint8_t *lds, uint32_t *vacc, FastTile t,
                                             uint4 v[8], uint32_t ev, int lane) {
    const uint32_t crc = gtile_crc<AUX, DIAG, COMPDIAG, S4, IMG, GROUP, HOIST>(p.payload, p.table_s4, lds, t, v, lane);
    const GShape g = gshape(t);
    if (uint32_t(lane) < g.nch + (g.kt ? 1u : 0u)) emit<VERIFY>(p, vacc, t.out + uint32_t(lane), crc, ev);
}

}  // namespace hdfs_crc_dev
