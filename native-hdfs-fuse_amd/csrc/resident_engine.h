// resident_engine.h -- the RESIDENT checksum kernel for concurrent block
// writes (crc32c_blocks_create_resident, include/hdfs_crc32c.h section 3b;
// the debug library's crc32c_debug_resident_* A/B shapes use it too).
//
// libfuse writes one 4 MiB block per hadoop_fuse_write_block call on many
// worker threads (src/fuse.c:336-449, fuse.c:1771).  One launch per block
// costs ~4.3 us of fixed work per launch (kernel boundary, table staging,
// tail: DESIGN.md section 5), which caps 16 writers with one block each at
// 1.8 us per block through the group-commit queue (crc32c_blocks).  Here the
// kernel stays on the GPU instead: tables staged ONCE per launch, blocks
// pulled from a ring the submitting threads fill, completion written to
// host memory -- no launch per block at all.
//
// Protocol (all host words in pinned, device-mapped, coherent memory):
//  * submit (host): ticket t = an atomic counter; slot t % kRing is reused
//    only once block t - kRing is complete; the slot's words (payload
//    pointer, out pointer and, for a block of another plan than the
//    queue's, its plan's ResShape record, kernel_abi.h) each carry t's tag,
//    so one read of the slot tells a complete entry from a stale or
//    half-written one.
//  * shapes: any plan of power-of-two tiles, general tiles and GenItems
//    (bpc 512 << k; a trimmed first packet of an append at an unaligned
//    block offset, hadooprpc.c:832-840, and packet tails), at any payload
//    alignment.  A block whose shape is "simple" (power-of-two tiles only,
//    16-byte aligned) runs the aligned tile loop; any other takes, per unit,
//    the shifted loads of crc32c_device.h for tiles off 16-byte alignment,
//    crc32c_general.h's gtile_crc for general tiles and gen_item_lin for
//    GenItems (half a wave each).
//  * forwarder (workgroup 0's last wave): reads 64 host slots per poll (one
//    PCIe round trip per poll, not per block) and copies the ready ones into
//    a device ring, tags and all (agent scope).
//  * collector (workgroup 1's last wave): block t is complete when all
//    workgroups' flags for its slot hold t + 1 (one 1 KiB load per check);
//    blocks complete in ticket order, hdone[slot] = t + 1 (system scope).
//  * workers (every other wave): block t is run by phase t % P (P blocks in
//    flight); within a phase PER waves per workgroup take its tiles (a 4 MiB
//    block is 512 tiles = 2 per CU: one each, or both by one wave with both
//    loaded first); a workgroup's phase workers count themselves in LDS and
//    the last one stores the workgroup's flag.  Checksums are stored
//    write-through (system scope), and every store has completed before the
//    flag.
//  * lifetime: the forwarder exits on the host's stop word, after idle_us
//    with nothing queued, or after kStuckMs without progress while blocks are
//    outstanding (a workgroup that never got a CU); on exit it raises the
//    device stop word that every worker polls; the collector records where
//    it stopped (exit_col) so a relaunch resumes there.  The host relaunches
//    the kernel on demand (submit, or a waiter that waits long), never while
//    one runs.  Workers have their own bound (kWorkerMs without a block).
//    Every wave therefore exits, whatever the host does.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "crc32c_device.h"
#include "hdfs_crc32c.h"
#include "runtime_internal.h"

namespace hdfs_crc_res {

using namespace hdfs_crc_dev;
using hdfs_crc::FastTile;

constexpr uint32_t kRing = 64;       // tickets in flight at most
// (the kernel is a template on WAVES per workgroup -- one workgroup per CU,
// 152 KiB of LDS --, PHASES, the blocks processed at once, and PER, the
// worker waves per workgroup and phase that take tiles (2: one 8 KiB tile
// each; 1: both tiles of the workgroup, both loaded before the first one's
// lookups, so twice the phases fit).  The product instantiates 16 / 7 / 2
// (crc32c_resident.hip); the debug library the other shapes, as A/B.)
constexpr uint32_t kMaxWg = 256;     // one flag lane-dword per workgroup (64 lanes x 4)
constexpr uint64_t kTicksPerUs = 100;  // s_memrealtime: 100 MHz
constexpr uint64_t kStuckMs = 50;
// Trace (HDFS_CRC32C_RESIDENT_STAMPS=1 at create): per ticket t % kStampRing,
// s_memrealtime when the forwarder forwarded it, when workgroup 0's worker
// of its phase saw it, when that worker's tiles were stored, and when the
// collector completed it; plus the forwarder's host-slot poll round trips.
constexpr uint32_t kStampRing = 4096;
constexpr uint64_t kWorkerMs = 200;

// A host slot is two 64-bit words, payload and out pointer (48-bit GPU
// addresses), each tagged in bits 48-62 with the low 15 bits of ticket + 1:
// a reader that sees both with matching tags has the block's pointers (no
// separate sequence word, no order between the stores).  Bit 63 of the out
// word: the block is of another plan than the queue's -- its shape record's
// address (tagged the same way) is in shape[slot], which the forwarder then
// loads too (a second round trip, only for such blocks: the common block
// costs the poll two loads per lane, not three).  The device ring holds all
// three words (shape 0: the queue's plan).
constexpr int kTagShift = 48;
constexpr uint64_t kAddrMask = (1ull << kTagShift) - 1;
constexpr uint64_t kTagMask = 0x7fffull << kTagShift;
constexpr uint64_t kShapeFlag = 1ull << 63;
__host__ __device__ constexpr uint64_t tag_of(uint64_t ticket) { return ((ticket + 1) & 0x7fffull) << kTagShift; }
constexpr uint32_t kSlotW = 3;  // (device ring) payload, out, shape

struct HostRing {
    uint64_t slot[kRing][2];  // host: the ticket's tagged payload / out pointers
    uint64_t shape[kRing];    // host: its tagged shape record (out word's kShapeFlag)
    uint64_t done[kRing];     // kernel: ticket + 1 once the block's checksums are stored
    uint32_t stop;            // host: exit now
    uint32_t pad0[15];
    uint64_t exit_col;        // kernel (at exit): tickets below this are complete
    uint64_t exits;           // kernel: launches that have exited
};

struct DevRing {
    uint64_t slot[kRing][kSlotW];
    uint32_t flag[kRing][kMaxWg];  // per slot and workgroup: ticket + 1 once its workers are done
    uint64_t fwd;                  // forwarder: tickets below this are forwarded
    uint64_t col;                  // collector: tickets below this are complete
    uint32_t stop;                 // forwarder: every wave exits
    uint64_t rtt_sum, rtt_n;       // trace: forwarder poll round trips (ticks), count
};

// The block's shape (wave-uniform: scalar loads of its plan's ResShape).
struct Shape {
    const FastTile *tiles;
    const GenItem *gen;
    uint32_t ntiles, ngen, simple;
};

struct RParams {
    HostRing *h;
    DevRing *d;
    // the queue plan's shape: a block of the queue's plan (the common case,
    // no kShapeFlag) needs no load of its record before its tiles
    Shape def;
    const uint8_t *table_s4;
    uint32_t flags;
    uint32_t c_lg[5];
    uint32_t c_small[4];
    uint64_t first;       // first ticket this launch forwards
    uint64_t idle_ticks;  // forwarder: exit after this long with nothing queued
    uint64_t *stamps;     // trace (nullptr: off), 4 per ticket % kStampRing
};

template <typename T>
__device__ __forceinline__ T ld_sys(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ T ld_dev(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_sys(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ void st_dev(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ Shape shape_at(uint64_t addr) {
    typedef const __attribute__((address_space(4))) hdfs_crc::ResShape *CS;
    const CS r = (CS)(addr);
    return Shape{r->tiles, r->gen, r->ntiles, r->ngen, r->simple};
}
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    const uint32_t lo = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(v))));
    const uint32_t hi = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(v >> 32))));
    return uint64_t(hi) << 32 | lo;
}

// One power-of-two tile of a block (offsets relative to the block's payload
// / checksum array): the production tile's loads, lookups and reduce,
// stores write-through.
__device__ __forceinline__ FastTile rtile(const FastTile *tiles, uint32_t idx) {
    typedef const __attribute__((address_space(4))) FastTile *CT;
    const CT tp = (CT)(tiles) + idx;
    return FastTile{tp->src, tp->out, tp->meta};
}
__device__ __forceinline__ void rtile_load(const uint8_t *payload, const FastTile &t, int lane, uint4 v[8]) {
    const uint32_t nb = t.meta & 0xffu;
    const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(payload + t.src, nb * 512u);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const auto r = __builtin_amdgcn_raw_buffer_load_b128(rsrc, 16u * uint32_t(lane) + 1024u * i, 0, 2);
        v[i] = make_uint4(r[0], r[1], r[2], r[3]);
    }
}
// A checksum of the block, write-through (system scope: the waiter's next
// stream work or copy may run on any XCD or engine).
__device__ __forceinline__ void rstore(uint32_t *out, uint32_t idx, uint32_t v) {
    typedef __attribute__((address_space(1))) uint32_t *GU32;  // (a global store, not a flat one)
    __hip_atomic_store((GU32)(out + idx), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void rtile_reduce(const RParams &p, const uint8_t *lds, uint32_t *out, const FastTile &t,
                                             const uint32_t pc[8], int lane) {
    const uint32_t nb = t.meta & 0xffu, lg = (t.meta >> 8) & 0xffu;
    uint32_t x = block_lin(pc, lane);
    const uint32_t blk = rep_block(lane);
    if (lg) {
        const uint32_t nbc = 1u << lg;
        const uint32_t s = nbc - 1u - (blk & (nbc - 1u));
        if (s) x = zshift<true, kImgFull>(lds, s, x);
        x ^= static_cast<uint32_t>(__shfl_xor(static_cast<int>(x), 32));
        if (lg >= 2) x ^= dpp<kDppXor8>(x);
        if (lg >= 3) x ^= dpp<kDppXor2>(x);
        if (lg >= 4) x ^= dpp<kDppXor1>(x);
    }
    if (rep_lane(lane, blk, nb, lg)) rstore(out, t.out + (blk >> lg), out_order(x ^ p.c_lg[lg], p.flags));
}
__device__ __forceinline__ void rtile_finish(const RParams &p, const uint8_t *lds, uint32_t *out, const FastTile &t,
                                             uint4 v[8], int lane) {
    uint32_t pc[8];
    tile_pieces<0, true, kImgFull>(lds, v, pc, lane, NoPrep{});
    rtile_reduce(p, lds, out, t, pc, lane);
}
__device__ __forceinline__ void run_tile(const RParams &p, const uint8_t *lds, const uint8_t *payload,
                                         uint32_t *out, const FastTile *tiles, uint32_t idx, int lane) {
    const FastTile t = rtile(tiles, idx);
    uint4 v[8];
    rtile_load(payload, t, lane, v);
    __builtin_amdgcn_sched_barrier(0);
    rtile_finish(p, lds, out, t, v, lane);
}
// Two tiles by one wave: both tiles' loads first, so the second one's
// latency hides under the first one's lookups.
__device__ __forceinline__ void run_tile_pair(const RParams &p, const uint8_t *lds, const uint8_t *payload,
                                              uint32_t *out, const FastTile *tiles, uint32_t ia, uint32_t ib,
                                              int lane) {
    const FastTile ta = rtile(tiles, ia), tb = rtile(tiles, ib);
    uint4 va[8], vb[8];
    rtile_load(payload, ta, lane, va);
    rtile_load(payload, tb, lane, vb);
    __builtin_amdgcn_sched_barrier(0);
    rtile_finish(p, lds, out, ta, va, lane);
    rtile_finish(p, lds, out, tb, vb, lane);
}

// A power-of-two tile of a block of any alignment: the aligned loads, or
// the shifted loads of crc32c_device.h when it starts off 16-byte alignment.
__device__ __forceinline__ void run_ptile(const RParams &p, const uint8_t *lds, const uint8_t *payload, uint32_t *out,
                                          const FastTile &t, int lane) {
    const uint32_t r = uint32_t(reinterpret_cast<uintptr_t>(payload + t.src)) & 15u;  // (uniform)
    if (!r) {
        uint4 v[8];
        rtile_load(payload, t, lane, v);
        __builtin_amdgcn_sched_barrier(0);
        rtile_finish(p, lds, out, t, v, lane);
        return;
    }
    uint4 v[9];
    load_shifted_raw<2>(payload, t, r, lane, v);
    __builtin_amdgcn_sched_barrier(0);
    uint32_t pc[8];
    const uint32_t b = r & 3u, li = ((t.meta & 0xffu) - 1u) >> 1;
    const int ll = int(((t.meta & 0xffu) - 1u) & 1u) * 32 + 31;
    switch (r >> 2) {
        case 0: tile_pieces<0, true, kImgFull>(lds, v, pc, lane, ShiftPrep<0>{v, b, lane, li, ll}); break;
        case 1: tile_pieces<0, true, kImgFull>(lds, v, pc, lane, ShiftPrep<1>{v, b, lane, li, ll}); break;
        case 2: tile_pieces<0, true, kImgFull>(lds, v, pc, lane, ShiftPrep<2>{v, b, lane, li, ll}); break;
        default: tile_pieces<0, true, kImgFull>(lds, v, pc, lane, ShiftPrep<3>{v, b, lane, li, ll}); break;
    }
    rtile_reduce(p, lds, out, t, pc, lane);
}

// GenItem chunks: half a wave each (gen_item_lin), the half-wave's item
// `g` (valid: it has one).
__device__ __forceinline__ void run_gen_item(const RParams &p, const uint8_t *lds, const uint8_t *payload,
                                             uint32_t *out, const GenItem &g, bool valid, int lane) {
    const uint32_t acc = gen_item_lin<true, kImgFull>(payload, lds, g, lane);
    if (valid && (lane & 31) == 0)
        rstore(out, g.out, out_order(acc ^ (g.len >= 4 ? 0xffffffffu : p.c_small[g.len]), p.flags));
}

// A general tile of a block (kGeneralTile: a packet's tail chunk behind up
// to 16 full chunks).  The resident queue takes only those of unpadded
// chunks of 2^lg blocks (bytesPerChecksum 512 << lg: crc32c_resident.hip
// checks), so the full chunks run as power-of-two tiles of 16 blocks and
// the tail as a GenItem -- no general-item gather code in this kernel.
__device__ __forceinline__ void run_gtile(const RParams &p, const uint8_t *lds, const uint8_t *payload, uint32_t *out,
                                          const FastTile &t, int lane) {
    const GShape g = gshape(t);
    const uint32_t lg = 31u - uint32_t(__builtin_clz(g.k));
    for (uint32_t s = 0; 16u * s < g.nfb; ++s) {
        const uint32_t nb = min(g.nfb - 16u * s, 16u);
        run_ptile(p, lds, payload, out, FastTile{g.src + 8192u * s, t.out + ((16u * s) >> lg), nb | (lg << 8)}, lane);
    }
    if (g.tl) {
        const GenItem gi{g.src + uint64_t(g.nch) * g.bpc, t.out + g.nch, g.tl};
        const bool valid = (lane >> 5) == 0;  // (the lower half-wave; the upper runs an empty item)
        run_gen_item(p, lds, payload, out, valid ? gi : GenItem{0, 0, 0}, valid, lane);
    }
}

// Unit `idx` of a block of any shape: tile idx, or, past the tiles, the
// GenItem pair idx - ntiles.
__device__ __forceinline__ void run_unit(const RParams &p, const uint8_t *lds, const uint8_t *payload, uint32_t *out,
                                         const Shape &sh, uint32_t idx, int lane) {
    if (idx < sh.ntiles) {
        const FastTile t = rtile(sh.tiles, idx);
        if (t.meta & hdfs_crc::kGeneralTile)
            run_gtile(p, lds, payload, out, t, lane);
        else
            run_ptile(p, lds, payload, out, t, lane);
        return;
    }
    const uint32_t gi = 2u * (idx - sh.ntiles) + (uint32_t(lane) >> 5);
    const bool valid = gi < sh.ngen;
    GenItem g{0, 0, 0};
    if (valid) g = sh.gen[gi];
    run_gen_item(p, lds, payload, out, g, valid, lane);
}

// A block of any shape: units first, first + stride, ... (tiles, then
// GenItem pairs).
__device__ __forceinline__ void run_units(const RParams &p, const uint8_t *lds, const uint8_t *payload,
                                                    uint32_t *out, Shape sh, uint32_t first, uint32_t stride,
                                                    int lane) {
    const uint32_t units = sh.ntiles + (sh.ngen + 1u) / 2u;
    for (uint32_t idx = first; idx < units; idx += stride) run_unit(p, lds, payload, out, sh, idx, lane);
}

// Forwarder (workgroup 0's last wave): the host ring -> the device ring.
// One PCIe round trip per poll covers the next 64 tickets.  Decides the
// launch's end: the host's stop word, idle_ticks with nothing outstanding,
// or kStuckMs without the collector advancing while blocks are outstanding.
// The aligned-only build (GENERAL false) never forwards a block that needs
// the general code (kShapeFlag): at the first one it stops forwarding and
// ends the launch (its blocks before that complete), and the host launches
// the general build for it.
template <bool GENERAL>
static inline __device__ void forwarder(const RParams &p, int lane) {
    HostRing *h = p.h;
    DevRing *d = p.d;
    uint64_t fwd = p.first, col = p.first;
    uint64_t last = now();
    uint64_t rtt_sum = 0, rtt_n = 0;
    for (;;) {
        bool progress = false;
        const uint64_t t_poll = p.stamps ? now() : 0;
        // the next 64 tickets' host slots, one load per lane (ring reuse:
        // ticket t only once t - kRing is complete; `col` from the previous
        // pass, so the collector's word and the host slots load together)
        const uint64_t cand = fwd + uint64_t(lane);
        const bool room = cand < col + kRing;
        const uint32_t sl = uint32_t(cand % kRing);
        const uint64_t w0 = room ? ld_sys(&h->slot[sl][0]) : 0, w1 = room ? ld_sys(&h->slot[sl][1]) : 0;
        const uint64_t c = ld_dev(&d->col);
        if (c != col) {
            col = c;
            progress = true;
        }
        const uint64_t tg = tag_of(cand);
        bool ok = room && (w0 & kTagMask) == tg && (w1 & kTagMask) == tg;
        uint64_t w2 = 0;
        const bool need = ok && (w1 & kShapeFlag);
        bool handoff = false;
        if (const uint64_t flagged = __ballot(need)) {  // (blocks needing the general build: their shape words)
            if (GENERAL) {
                w2 = need ? ld_sys(&h->shape[sl]) : 0;
                ok = ok && (!need || (w2 & kTagMask) == tg);
            } else {
                // forward up to the first such block, then end the launch
                const uint64_t before = ~__ballot(ok);
                if (!before || __builtin_ctzll(flagged) <= __builtin_ctzll(before)) {
                    ok = ok && uint32_t(lane) < uint32_t(__builtin_ctzll(flagged));
                    handoff = true;
                }
            }
        }
        const uint64_t ready = __ballot(ok);
        if (p.stamps) {  // (the ballot waited for the host loads)
            rtt_sum += now() - t_poll;
            ++rtt_n;
        }
        const uint32_t n = ~ready ? uint32_t(__builtin_ctzll(~ready)) : 64u;  // consecutive ready tickets from fwd
        if (n) {
            if (uint32_t(lane) < n) {
                st_dev(&d->slot[sl][0], w0);
                st_dev(&d->slot[sl][1], w1);
                st_dev(&d->slot[sl][2], w2);
                if (p.stamps) st_dev(&p.stamps[4 * (cand % kStampRing)], now());
            }
            fwd += n;
            if (lane == 0) st_dev(&d->fwd, fwd);
            progress = true;
        }
        if (handoff) break;  // (after forwarding the blocks before it)
        const uint64_t t = now();
        if (progress) {
            last = t;
            continue;
        }
        if (ld_sys(&h->stop)) break;
        if (col == fwd && t - last > p.idle_ticks) break;                  // idle
        if (col < fwd && t - last > kStuckMs * 1000 * kTicksPerUs) break;  // no progress: give up
        __builtin_amdgcn_s_sleep(2);
    }
    if (lane == 0) {
        st_dev(&d->stop, 1u);
        if (p.stamps) {
            st_dev(&d->rtt_sum, ld_dev(&d->rtt_sum) + rtt_sum);
            st_dev(&d->rtt_n, ld_dev(&d->rtt_n) + rtt_n);
        }
    }
}

// Collector (workgroup 1's last wave): block t is complete when every
// workgroup's flag for its slot holds t + 1; the (up to 8) oldest
// outstanding blocks' flags are loaded together and completed in ticket
// order (hdone[slot] = t + 1 in host memory).  Ends once the forwarder has
// stopped and nothing it forwarded is outstanding (or kStuckMs later), then
// records where it stopped for the next launch.
static inline __device__ void collector(const RParams &p, int lane) {
    HostRing *h = p.h;
    DevRing *d = p.d;
    uint64_t col = p.first;
    uint64_t last = now();
    const uint32_t ng = gridDim.x;
    for (;;) {
        const uint32_t stop = ld_dev(&d->stop);
        const uint64_t fwd = ld_dev(&d->fwd);
        bool progress = false;
        constexpr uint32_t kCheck = 8;
        const uint64_t nout = fwd > col ? fwd - col : 0;
        uint32_t f[kCheck][4];
#pragma unroll
        for (uint32_t c = 0; c < kCheck; ++c)
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const uint32_t wg = 4u * uint32_t(lane) + k;
                f[c][k] = (c < nout && wg < ng) ? ld_dev(&d->flag[(col + c) % kRing][wg]) : 0u;
            }
#pragma unroll
        for (uint32_t c = 0; c < kCheck; ++c) {
            if (c >= nout) break;
            const uint32_t want = uint32_t(col + 1);
            bool ok = true;
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k)
                if (4u * uint32_t(lane) + k < ng && f[c][k] != want) ok = false;
            if (__ballot(!ok)) break;
            if (lane == 0) {
                st_sys(&h->done[col % kRing], col + 1);
                if (p.stamps) st_dev(&p.stamps[4 * (col % kStampRing) + 3], now());
            }
            ++col;
            progress = true;
        }
        if (progress) {
            if (lane == 0) st_dev(&d->col, col);
            last = now();
            continue;
        }
        if (stop && col >= fwd) break;
        if (stop && now() - last > kStuckMs * 1000 * kTicksPerUs) break;
        if (now() - last > kWorkerMs * 1000 * kTicksPerUs) break;  // (the forwarder is gone)
        __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) {
        st_sys(&h->exit_col, col);
        wait_vmem();
        st_sys(&h->exits, ld_sys(&h->exits) + 1);
    }
}

template <uint32_t kWaves, uint32_t kPhases, uint32_t kPer, bool GENERAL = false>
__global__ __launch_bounds__(kWaves * 64, kWaves / 4) void resident_kernel(RParams p) {
    constexpr uint32_t kWorkers = kWaves - 1;
    constexpr uint32_t kStage = kS4StageBytes;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kStage + 4 * kRing];
    uint32_t *lcnt = reinterpret_cast<uint32_t *>(lds + kStage);  // per slot: this workgroup's workers done
    const int lane = int(threadIdx.x & 63u);
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr uint32_t kChunks = kStage / 1024u;
    const uint32_t rot = (blockIdx.x * 37u) % kChunks;
    for (uint32_t i = wv; i < kChunks; i += kWaves) {
        const uint32_t c = i + rot < kChunks ? i + rot : i + rot - kChunks;
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void *)(p.table_s4 + c * 1024u + 16u * uint32_t(lane)),
            (__attribute__((address_space(3))) void *)(lds + c * 1024u), 16, 0, 0);
    }
    if (threadIdx.x < kRing) lcnt[threadIdx.x] = 0;
    __syncthreads();
    if (wv == kWaves - 1) {
        if (blockIdx.x == 0) forwarder<GENERAL>(p, lane);
        if (blockIdx.x == 1) collector(p, lane);
        return;
    }
    // Worker: phase (b + w) % P; the workgroup's waves of a phase rank in
    // wave order; the first kPer take tiles kPer b + rank (+ kPer G, ...).
    const uint32_t b = blockIdx.x, G = gridDim.x;
    const uint32_t phase = (b + wv) % kPhases;
    uint32_t rank = 0, expect = 0;
    for (uint32_t w = 0; w < kWorkers; ++w)
        if ((b + w) % kPhases == phase) {
            if (w < wv) ++rank;
            ++expect;
        }
    DevRing *d = p.d;
    uint64_t j = p.first + (phase + kPhases - uint32_t(p.first % kPhases)) % kPhases;  // first block of the phase
    uint64_t last = now();
    for (;;) {
        const uint32_t sl = uint32_t(j % kRing);
        bool stop = false;
        uint64_t w0 = 0, w1 = 0, w2 = 0;
        const uint64_t tg = tag_of(j);
        for (uint32_t polls = 0;; ++polls) {
            w0 = ld_dev(&d->slot[sl][0]);
            w1 = ld_dev(&d->slot[sl][1]);
            if ((w0 & kTagMask) == tg && (w1 & kTagMask) == tg) {
                if (!GENERAL || !(w1 & kShapeFlag)) break;
                w2 = ld_dev(&d->slot[sl][2]);  // (a block of another plan: its shape word too)
                if ((w2 & kTagMask) == tg) break;
            }
            if ((polls & 15u) == 15u && (ld_dev(&d->stop) || now() - last > kWorkerMs * 1000 * kTicksPerUs)) {
                stop = true;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (stop) break;
        const bool stamp = p.stamps && b == 0 && lane == 0;
        if (stamp) st_dev(&p.stamps[4 * (j % kStampRing) + 1], now());
        const uint8_t *payload = reinterpret_cast<const uint8_t *>(uniform64(w0) & kAddrMask);
        uint32_t *out = reinterpret_cast<uint32_t *>(uniform64(w1) & kAddrMask);
        const Shape sh = GENERAL && (w1 & kShapeFlag) ? shape_at(uniform64(w2) & kAddrMask) : p.def;
        // (aligned tiles only: the round-4 loop; any other block, general
        // build only: units = its tiles, then its GenItem pairs)
        const bool simple = !GENERAL || !(w1 & kShapeFlag);
        if (!simple) {
            if (kPer == 1 || rank < kPer)
                run_units(p, lds, payload, out, sh, kPer == 1 ? b : kPer * b + rank, kPer * G, lane);
        } else if (kPer == 1) {  // (rank 0: this workgroup's tiles b, b + G, ..., two at a time)
            for (uint32_t idx = b; idx < sh.ntiles; idx += 2u * G) {
                if (idx + G < sh.ntiles)
                    run_tile_pair(p, lds, payload, out, sh.tiles, idx, idx + G, lane);
                else
                    run_tile(p, lds, payload, out, sh.tiles, idx, lane);
            }
        } else if (rank < kPer) {
            for (uint32_t idx = kPer * b + rank; idx < sh.ntiles; idx += kPer * G)
                run_tile(p, lds, payload, out, sh.tiles, idx, lane);
        }
        wait_vmem();  // (this wave's checksum stores have completed)
        if (stamp && rank == 0) st_dev(&p.stamps[4 * (j % kStampRing) + 2], now());
        if (lane == 0) {
            const uint32_t old = atomicAdd(&lcnt[sl], 1u);
            if (old + 1u == expect) {
                lcnt[sl] = 0;
                st_dev(&d->flag[sl][b], uint32_t(j + 1));
            }
        }
        j += kPhases;
        last = now();
    }
}

}  // namespace hdfs_crc_res
