// crc32c_items.h -- the CRC32C kernel's non-tile work items: GenItem
// chunks (half a wave per chunk of any length / alignment), SegItem chunks
// assembled from several buffers, and ConstRun checksums known at plan time.
// Internal to crc32c_device.h, which includes it after the tile helpers.
#pragma once

namespace hdfs_crc_dev {

// ---- general path: half a wave per chunk of any length / alignment -------
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

// lin() of the half-wave's GenItem g (chunk at payload + g.src), in every
// lane of the half-wave: the chunk right-aligned into zero-prefixed virtual
// 512-byte blocks, Horner-combined with Z^512.  Both half-waves take part
// (the reduction and the loop bound span the wave).  Also the resident
// kernel's (resident_engine.h).
template <bool S4, int IMG>
__device__ __forceinline__ uint32_t gen_item_lin(const uint8_t *payload, const uint8_t *lds, const GenItem &g,
                                                 int lane) {
    const uint32_t q = uint32_t(lane) & 31u;
    const uint32_t r = g.len;
    const uint32_t nbv = (r + 511u) >> 9;  // virtual 512-byte blocks
    const uint32_t nmax = max(__builtin_amdgcn_readlane(nbv, 0), __builtin_amdgcn_readlane(nbv, 32));
    const int64_t pad = int64_t(nbv) * 512 - int64_t(r);
    const uintptr_t cbeg = reinterpret_cast<uintptr_t>(payload) + g.src;
    const uintptr_t cend = cbeg + r;
    const uintptr_t ffend = r >= 4 ? cbeg + 4 : cbeg;
    const LaneCols cols = lane_cols<IMG>(q);
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
            lin = piece<S4, 0, IMG>(lds, funnel(w, uint32_t(a & 15u)), cols);
        }
        lin = allreduce32(lin);
        if (m < nbv) acc = zshift<S4, IMG>(lds, 1, acc) ^ lin;
    }
    return acc;
}

template <bool S4, bool VERIFY, int IMG>
__device__ __forceinline__ void gen_pair(const KParams &p, const uint8_t *lds, uint32_t *vacc, uint32_t pair,
                                         int lane) {
    const uint32_t h = uint32_t(lane) >> 5, q = uint32_t(lane) & 31u;
    const uint32_t idx = 2u * pair + h;
    const bool valid = idx < p.ngen;
    GenItem g{0, 0, 0};
    if (valid) g = p.gen[idx];
    const uint32_t acc = gen_item_lin<S4, IMG>(p.payload, lds, g, lane);
    if (valid && q == 0) {
        const uint32_t r = g.len;
        const uint32_t crc = acc ^ (r >= 4 ? 0xffffffffu : p.c_small[r]);
        emit<VERIFY>(p, vacc, g.out, crc, VERIFY ? p.expect[g.out] : 0u);
    }
}

// A chunk assembled from several buffers (SegItem): like gen_pair, but each
// lane's 16-byte window (chunk positions o .. o+15) is filled from every data
// piece it overlaps; positions no piece covers are zero fill.
template <bool S4, bool VERIFY, int IMG>
__device__ __forceinline__ void seg_pair(const KParams &p, const uint8_t *lds, uint32_t *vacc, uint32_t pair,
                                         int lane) {
    const uint32_t h = uint32_t(lane) >> 5, q = uint32_t(lane) & 31u;
    const uint32_t idx = 2u * pair + h;
    const bool valid = idx < p.nseg;
    SegItem s{0, 0, 0, 0};
    if (valid) s = p.seg[idx];
    const uint32_t r = s.len;
    const uint32_t nbv = (r + 511u) >> 9;
    const uint32_t nmax = max(__builtin_amdgcn_readlane(nbv, 0), __builtin_amdgcn_readlane(nbv, 32));
    const int64_t pad = int64_t(nbv) * 512 - int64_t(r);
    const uintptr_t base = reinterpret_cast<uintptr_t>(p.payload);
    const LaneCols cols = lane_cols<IMG>(q);
    uint32_t acc = 0;
    for (uint32_t m = 0; m < nmax; ++m) {
        uint32_t lin = 0;
        if (m < nbv) {
            const int64_t o = int64_t(m) * 512 + int64_t(16 * q) - pad;  // chunk position of the window
            uint4 d = make_uint4(0, 0, 0, 0);
            for (uint32_t u = 0; u < s.npieces; ++u) {
                const GenPiece g = p.pieces[s.first + u];
                if (o >= int64_t(g.start) + g.len || o + 16 <= int64_t(g.start)) continue;
                const uintptr_t cbeg = base + g.src, cend = cbeg + g.len;
                const uintptr_t a = cbeg + uintptr_t(o - int64_t(g.start));
                const uintptr_t a0 = a & ~uintptr_t(15);
                uint32_t w[8];
                load_piece(a0, cbeg, cend, cbeg, w);
                load_piece(a0 + 16, cbeg, cend, cbeg, w + 4);
                const uint4 f = funnel(w, uint32_t(a & 15u));
                d = make_uint4(d.x | f.x, d.y | f.y, d.z | f.z, d.w | f.w);
            }
            if (r >= 4) d = chunk_start_mask(d, int(-o));  // (o + 16 > 0 here: nothing before the chunk is loaded)
            lin = piece<S4, 0, IMG>(lds, d, cols);
        }
        lin = allreduce32(lin);
        if (m < nbv) acc = zshift<S4, IMG>(lds, 1, acc) ^ lin;
    }
    if (valid && q == 0) {
        const uint32_t crc = acc ^ (r >= 4 ? 0xffffffffu : p.c_small[r]);
        emit<VERIFY>(p, vacc, s.out, crc, VERIFY ? p.expect[s.out] : 0u);
    }
}

// Checksums known at plan time (chunks of zero fill only): stored (or compared).
template <bool VERIFY>
__device__ __forceinline__ void const_run(const KParams &p, uint32_t *vacc, uint32_t i, int lane) {
    const ConstRuns c = (ConstRuns)(p.consts) + i;
    const uint32_t out = c->out, count = c->count, value = c->value;
    for (uint32_t k = uint32_t(lane); k < count; k += 64u)
        emit<VERIFY>(p, vacc, out + k, value, VERIFY ? p.expect[out + k] : 0u);
}

}  // namespace hdfs_crc_dev
