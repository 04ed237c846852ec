// plan.cpp -- see plan.h.
#include <cstdlib>
#include "plan.h"
#include "hdfs_crc32c.h"

#include <algorithm>
#include <cerrno>
#include <cstring>

#include "crc_math.h"
#include "hdfs_crc32c_debug.h"

namespace hdfs_crc {

static int fast_lg(uint32_t bpc) {
    for (int lg = 0; lg <= 4; ++lg)
        if (bpc == (kBlockBytes << lg)) return lg;
    return -1;
}

void HostPlan::clear() {
    tiles.clear();
    gen.clear();
    seg.clear();
    pieces.clear();
    consts.clear();
    nchecksums = payload_bytes = 0;
}

uint64_t HostPlan::items() const {
    return uint64_t(tiles.size()) + (gen.size() + 1) / 2 + (seg.size() + 1) / 2 + consts.size();
}

static void push_gen(HostPlan *plan, uint64_t src, uint64_t out, uint32_t len) {
    GenItem g;
    g.src = src;
    g.out = uint32_t(out);
    g.len = len;
    plan->gen.push_back(g);
}


// Full chunks per general item of k blocks per chunk: when k divides 16,
// whole chunks filling two subtiles (round 3: one; measured, same box:
// bpc 1000 60.3 -> 58.5 us, bpc 700 73.6 -> 70.2, bpc 4000 62.3 -> 59.8),
// else kGeneralChunks = 16 (bpc 1536: 3 subtiles, the best of 5-31 chunks;
// bpc 2560 / 3000 slower or equal with fewer).  A/B knobs:
// HDFS_CRC32C_GBLOCKS (about that many blocks per item; 0: round 3's sizes),
// HDFS_CRC32C_GCHUNKS (k not dividing 16) and HDFS_CRC32C_GCHUNKS_DIV (k
// dividing 16, a multiple of 16 / k) override it.  At most 31 (the
// descriptor's field).
static long env_long(const char *name) {
    const char *e = std::getenv(name);
    return e ? std::atol(e) : -1L;
}
static uint64_t item_chunks(uint32_t k) {
    static const long blocks = env_long("HDFS_CRC32C_GBLOCKS"), ch = env_long("HDFS_CRC32C_GCHUNKS"),
                      div = env_long("HDFS_CRC32C_GCHUNKS_DIV");
    const uint64_t one = kTileBlocks % k == 0 ? kTileBlocks / k : 1;  // chunks that fill whole subtiles
    if (kTileBlocks % k == 0 && div >= 1 && div <= 31 && uint64_t(div) % one == 0) return uint64_t(div);
    if (kTileBlocks % k != 0 && ch >= 1 && ch <= 31) return uint64_t(ch);
    if (blocks < 0)  // the default: two subtiles of whole chunks when k divides 16, else 16 chunks
        return kTileBlocks % k == 0 ? (2 * one <= 31 ? 2 * one : one) : kGeneralChunks;
    const uint64_t target = uint64_t(blocks);
    if (target == 0) return kTileBlocks % k == 0 ? one : kGeneralChunks;  // round 3's sizes
    uint64_t n = std::max<uint64_t>(target / k, 1);
    n = std::max<uint64_t>(n / one, 1) * one;  // whole subtiles when k divides 16
    while (n > 31) n -= one;
    return n;
}

// Padded power-of-two tiles for bpc = 512 * 2^lg - pad (plan.h); A/B knob
// HDFS_CRC32C_PADDED_TILES=0 sends those chunks to general items instead.
static bool padded_tiles_on() {
    static const bool on = env_long("HDFS_CRC32C_PADDED_TILES") != 0;
    return on;
}
// Half tiles for bpc <= 256, 512 < bpc <= 768 (M = 1) and 1024 < bpc <= 1280
// (M = 2) (plan.h); A/B knob HDFS_CRC32C_HALF_TILES=0 sends those chunks to
// the forms above instead.
static bool half_tiles_on() {
    static const bool on = env_long("HDFS_CRC32C_HALF_TILES") != 0;
    return on;
}

// Whether a packet's tail chunk (tl >= 4 bytes) next to tiles of whole
// chunks goes alone into a GenItem rather than into a general item with the
// packet's last `last` full chunks (k virtual blocks each): when that item
// would not fit one 16-block subtile.  knob (an A/B environment variable): 1
// always a GenItem, 0 never, unset the rule.
static bool tail_alone(long knob, uint64_t last, uint32_t k, uint32_t tl) {
    if (knob == 1 || knob == 0) return knob == 1;
    return last * k + (tl + kBlockBytes - 1) / kBlockBytes > kTileBlocks;
}

int append_packet(const crc32c_packet &p, HostPlan *plan, bool absolute) {
    // A zero-length packet (the block's last-packet marker, hadooprpc.c:644,
    // 853-856) has no checksums whatever its bpc; any other needs bpc > 0.
    if (p.len == 0) return 0;
    if (p.bpc == 0) return -EINVAL;
    const uint64_t n = (uint64_t(p.len) + p.bpc - 1) / p.bpc;  // hadooprpc.c:639
    if (p.out_idx + n > (1ull << 32)) return -EINVAL;
    if (p.out_idx + n > plan->nchecksums) plan->nchecksums = p.out_idx + n;
    plan->payload_bytes += p.len;

    const uint64_t nfull = p.len / p.bpc;
    const uint32_t tail = p.len % p.bpc;
    const int lg = fast_lg(p.bpc);
    bool tail_done = false;
    if (lg >= 0) {
        // Any alignment: a tile off 16-byte alignment is read with unaligned
        // dwordx4 buffer loads (config 2 five bytes off: 55 instead of 42.5 us).
        const uint64_t blocks = nfull << lg;  // 512-byte blocks of full chunks
        for (uint64_t b = 0; b < blocks; b += kTileBlocks) {
            const uint64_t nb = blocks - b < kTileBlocks ? blocks - b : kTileBlocks;
            FastTile t;
            t.src = p.payload_off + b * kBlockBytes;
            t.out = uint32_t(p.out_idx + (b >> lg));
            t.meta = uint32_t(nb) | (uint32_t(lg) << 8);
            // A tail of at most one 512-byte block is a GenItem on its own
            // (the batch then keeps the power-of-two build: 412-byte tails,
            // same box, 46.25 -> 44.89 us, round 5); a longer one rides
            // behind the packet's last chunks in a general item, since a
            // GenItem runs its blocks one after another at the launch's end.
            // A/B knob HDFS_CRC32C_POW2_TAIL_GEN: 1 always a GenItem, 0 never.
            static const long pow2_tail_knob = env_long("HDFS_CRC32C_POW2_TAIL_GEN");
            const bool pow2_tail_gen = pow2_tail_knob == 1 || (pow2_tail_knob != 0 && tail <= kBlockBytes);
            if (b + nb == blocks && tail >= 4 && !pow2_tail_gen) {
                // the packet's short tail chunk rides behind its last chunks:
                // that tile becomes a general item (k = 2^lg, no pad)
                t.src |= uint64_t(tail) << 48;
                t.meta = general_meta(uint32_t(nb >> lg), 1u << lg, 0, (tail + kBlockBytes - 1) / kBlockBytes);
                tail_done = true;
            }
            plan->tiles.push_back(t);
        }
    } else if (p.bpc >= 4 && p.bpc <= kMaxTileBpc) {
        // General items: up to 16 chunks of k virtual blocks each, processed
        // as 16-block subtiles (a chunk may span two).  A padded item's
        // first loads start up to 15 bytes before its first chunk (masked to
        // zero): allowed when those bytes are in the same allocation
        // (offset >= 16) or, for device addresses, the same page.
        const uint32_t k = (p.bpc + kBlockBytes - 1) / kBlockBytes;
        const uint32_t pad = k * kBlockBytes - p.bpc;
        const auto early_ok = [&](uint64_t src) { return absolute ? (src & 4095u) >= 16 : src >= 16; };
        uint64_t c = 0;
        const int klg = fast_lg(k * kBlockBytes);
        const bool half = (p.bpc <= 256 || (p.bpc > 512 && p.bpc <= 768) || (p.bpc > 1024 && p.bpc <= 1280)) &&
                          half_tiles_on();
        if (half) {
            // Half tiles of up to 32 (bpc <= 256), 10 (M = 1) or 6 (M = 2)
            // chunks; a tail chunk rides in a general item with the last
            // chunks that did not fill a tile.
            const uint32_t m = p.bpc / 512u, padh = 256u - (p.bpc - 512u * m);
            const uint64_t cpt = m == 0 ? 32 : m == 1 ? 10 : 6;
            // (as next to padded tiles: the tail alone a GenItem when the
            // general item would span two subtiles; A/B knob
            // HDFS_CRC32C_HALF_TAIL_GEN: 1 always, 0 never)
            static const long half_tail_knob = env_long("HDFS_CRC32C_HALF_TAIL_GEN");
            const uint64_t last = nfull % cpt ? nfull % cpt : cpt;
            const bool tail_gen = tail_alone(half_tail_knob, last, k, tail);
            uint64_t upto = nfull;
            if (tail >= 4 && nfull && !tail_gen) upto = nfull - last;
            while (c < upto) {
                const uint64_t src = p.payload_off + c * p.bpc;
                if (!early_ok(src)) {
                    push_gen(plan, src, p.out_idx + c, p.bpc);
                    ++c;
                    continue;
                }
                const uint64_t nch = std::min(cpt, upto - c);
                FastTile t;
                t.src = src;
                t.out = uint32_t(p.out_idx + c);
                t.meta = half_meta(uint32_t(nch), m, padh);
                plan->tiles.push_back(t);
                c += nch;
            }
        } else if (klg >= 0 && padded_tiles_on()) {
            // k a power of two: padded power-of-two tiles of 16 >> lg chunks.
            // A tail chunk (>= 4 bytes) rides in a general item with the last
            // 1 .. 16 >> lg full chunks before it when they fit one 16-block
            // subtile together; otherwise every full chunk goes into tiles
            // and the tail alone is a GenItem (round 5, same box: bpc 2000
            // 52.35 -> 51.37 us, bpc 4000 54.40 -> 51.92; bpc 1000, whose
            // item is 4 blocks, 52.00 -> 54.02 the other way).  A/B knob
            // HDFS_CRC32C_PADDED_TAIL_GEN: 1 always a GenItem, 0 never.
            static const long tail_knob = env_long("HDFS_CRC32C_PADDED_TAIL_GEN");
            const uint64_t cpt = kTileBlocks >> klg;
            const uint64_t last = nfull % cpt ? nfull % cpt : cpt;
            const bool tail_gen = tail_alone(tail_knob, last, k, tail);
            uint64_t upto = nfull;
            if (tail >= 4 && nfull && !tail_gen) upto = nfull - last;
            while (c < upto) {
                const uint64_t src = p.payload_off + c * p.bpc;
                if (!early_ok(src)) {
                    push_gen(plan, src, p.out_idx + c, p.bpc);
                    ++c;
                    continue;
                }
                const uint64_t nch = std::min(cpt, upto - c);
                FastTile t;
                t.src = src;
                t.out = uint32_t(p.out_idx + c);
                t.meta = padded_meta(uint32_t(nch << klg), uint32_t(klg), pad);
                plan->tiles.push_back(t);
                c += nch;
            }
        }
        // (k dividing 16: whole chunks fill subtiles exactly, and one subtile
        // per item keeps the item loop out of the way)
        const uint64_t per = item_chunks(k);
        while (c < nfull) {
            const uint64_t src = p.payload_off + c * p.bpc;
            if (pad && !early_ok(src)) {
                push_gen(plan, src, p.out_idx + c, p.bpc);
                ++c;
                continue;
            }
            const uint64_t nch = std::min(per, nfull - c);
            FastTile t;
            t.src = src;
            t.out = uint32_t(p.out_idx + c);
            t.meta = general_meta(uint32_t(nch), k, pad);
            // The packet's tail chunk rides in its last item: it starts
            // right after the item's full chunks, so its loads never reach
            // before the packet.
            const uint32_t kt = (tail + kBlockBytes - 1) / kBlockBytes;
            if (c + nch == nfull && tail >= 4) {
                t.src |= uint64_t(tail) << 48;
                t.meta = general_meta(uint32_t(nch), k, pad, kt);
                tail_done = true;
            }
            plan->tiles.push_back(t);
            c += nch;
        }
    } else {
        for (uint64_t c = 0; c < nfull; ++c) push_gen(plan, p.payload_off + c * p.bpc, p.out_idx + c, p.bpc);
    }
    if (tail && !tail_done) push_gen(plan, p.payload_off + nfull * p.bpc, p.out_idx + nfull, tail);
    return 0;
}

int build_plan(const crc32c_packet *pkts, size_t npkts, HostPlan *plan, bool absolute) {
    plan->clear();
    for (size_t i = 0; i < npkts; ++i) {
        const int rc = append_packet(pkts[i], plan, absolute);
        if (rc) return rc;
    }
    return 0;
}

namespace {

// crc(0, zeros(n)) for the polynomial: the register ~0 moved over n zero
// bytes, post-inverted (crc32c.c:84, 106 conditioning).
struct ZeroCrc {
    uint32_t poly;
    uint32_t last_len = 0, last = 0;
    uint32_t operator()(uint32_t n) {
        if (n != last_len || !last_len) {
            last = shift_zeros(0xffffffffu, n, poly) ^ 0xffffffffu;
            last_len = n;
        }
        return last;
    }
};

// n consecutive checksums out .. out + n - 1 of one constant value: extends
// the last run where it continues it, in runs of at most kConstRunMax.
void push_const(HostPlan *plan, uint64_t out, uint32_t value, uint64_t n = 1) {
    while (n) {
        if (!plan->consts.empty()) {
            ConstRun &r = plan->consts.back();
            if (r.value == value && uint64_t(r.out) + r.count == out && r.count < kConstRunMax) {
                const uint64_t k = std::min<uint64_t>(n, kConstRunMax - r.count);
                r.count += uint32_t(k);
                out += k;
                n -= k;
                continue;
            }
        }
        const uint64_t k = std::min<uint64_t>(n, kConstRunMax);
        plan->consts.push_back(ConstRun{uint32_t(out), uint32_t(k), value, 0u});
        out += k;
        n -= k;
    }
}

}  // namespace

int build_write_plan(const crc32c_buffer *buffers, uint32_t n_buffers, uint64_t bufferoffset, uint64_t len,
                     uint64_t blockoffset, uint32_t packetsize, uint32_t bpc, uint32_t poly, HostPlan *plan) {
    plan->clear();
    if (bpc == 0 || packetsize == 0 || (n_buffers && !buffers)) return -EINVAL;
    std::vector<uint64_t> start(size_t(n_buffers) + 1, 0);  // stream offset of each buffer
    for (uint32_t i = 0; i < n_buffers; ++i) {
        if (buffers[i].len > UINT64_MAX - start[i]) return -EINVAL;
        start[i + 1] = start[i] + buffers[i].len;
    }
    if (bufferoffset > start[n_buffers] || len > start[n_buffers] - bufferoffset) return -EINVAL;

    ZeroCrc zero{poly};
    uint64_t out = 0, sent = 0;
    uint32_t bi = 0;  // buffer holding the current chunk's first byte
    crc32c_packet run{};  // consecutive chunks of one packet inside one data buffer
    bool in_run = false;
    uint32_t run_buf = 0;
    auto flush = [&]() -> int {
        if (!in_run) return 0;
        in_run = false;
        return append_packet(run, plan, true);
    };
    // Packet cutting of hadoop_rpc_send_packets (hadooprpc.c:827-857), as crc32c_packetize.
    for (;;) {
        uint64_t plen = len - sent < packetsize ? len - sent : packetsize;
        const uint64_t past = (blockoffset + sent) % bpc;
        if (plen > 0 && past != 0) plen = std::min<uint64_t>(bpc - past, len - sent);
        if (plen == 0) break;
        if (plen > UINT32_MAX) return -E2BIG;
        const uint64_t pos = bufferoffset + sent;  // stream offset of the packet
        const uint64_t nch = (plen + bpc - 1) / bpc;
        if (out + nch > (1ull << 32)) return -E2BIG;
        const uint64_t nfullp = plen / bpc;  // full-length chunks of the packet
        for (uint64_t c = 0; c < nch; ++c) {
            const uint64_t a = pos + c * bpc;
            while (bi + 1 < n_buffers && start[bi + 1] <= a) ++bi;
            // Bulk: the full chunks c .. c + nf - 1 lie wholly inside buffer bi
            // (O(packets), not O(chunks), for the common case).
            const uint64_t nf = c < nfullp ? std::min<uint64_t>(nfullp - c, (start[bi + 1] - a) / bpc) : 0;
            if (nf >= 2) {
                if (buffers[bi].data) {
                    const uint64_t addr = uint64_t(uintptr_t(buffers[bi].data)) + (a - start[bi]);
                    if (in_run && run_buf == bi && c > 0 && run.payload_off + run.len == addr) {
                        run.len += uint32_t(nf * bpc);
                    } else {
                        if (int rc = flush()) return rc;
                        run = crc32c_packet{addr, out + c, uint32_t(nf * bpc), bpc};
                        run_buf = bi;
                        in_run = true;
                    }
                } else {
                    if (int rc = flush()) return rc;
                    push_const(plan, out + c, zero(bpc), nf);
                }
                c += nf - 1;
                continue;
            }
            const uint32_t clen = uint32_t(std::min<uint64_t>(bpc, plen - c * bpc));
            const uint64_t b = a + clen;
            // (zero-length buffers are skipped by the loop above)
            if (b <= start[bi + 1]) {  // inside one buffer
                if (buffers[bi].data) {
                    const uint64_t addr = uint64_t(uintptr_t(buffers[bi].data)) + (a - start[bi]);
                    if (in_run && run_buf == bi && c > 0 && run.payload_off + run.len == addr) {
                        run.len += clen;
                    } else {
                        if (int rc = flush()) return rc;
                        run = crc32c_packet{addr, out + c, clen, bpc};
                        run_buf = bi;
                        in_run = true;
                    }
                } else {
                    if (int rc = flush()) return rc;
                    push_const(plan, out + c, zero(clen));
                }
                continue;
            }
            // spans buffers: one SegItem with a piece per data buffer
            if (int rc = flush()) return rc;
            SegItem s{uint32_t(plan->pieces.size()), 0u, uint32_t(out + c), clen};
            for (uint32_t j = bi; j < n_buffers && start[j] < b; ++j) {
                const uint64_t lo = std::max(a, start[j]), hi = std::min(b, start[j + 1]);
                if (hi <= lo || !buffers[j].data) continue;
                GenPiece pc;
                pc.src = uint64_t(uintptr_t(buffers[j].data)) + (lo - start[j]);
                pc.start = uint32_t(lo - a);
                pc.len = uint32_t(hi - lo);
                plan->pieces.push_back(pc);
                ++s.npieces;
            }
            if (s.npieces == 0)
                push_const(plan, out + c, zero(clen));
            else
                plan->seg.push_back(s);
        }
        if (int rc = flush()) return rc;
        out += nch;
        sent += plen;
    }
    // append_packet counted the runs; the totals cover every chunk.
    plan->nchecksums = out;
    plan->payload_bytes = len;
    return 0;
}

void rebase_plan(HostPlan *plan, uint64_t *base) {
    uint64_t lo = UINT64_MAX;
    for (const FastTile &t : plan->tiles) lo = std::min(lo, t.src & kSrcMask);  // (bits 48-63: a tail length)
    for (const GenItem &g : plan->gen) lo = std::min(lo, g.src);
    for (const GenPiece &p : plan->pieces) lo = std::min(lo, p.src);
    lo = lo == UINT64_MAX ? 0 : lo & ~uint64_t(15);
    for (FastTile &t : plan->tiles) t.src -= lo;
    for (GenItem &g : plan->gen) g.src -= lo;
    for (GenPiece &p : plan->pieces) p.src -= lo;
    *base = lo;
}

}  // namespace hdfs_crc

extern "C" int crc32c_debug_plan(const crc32c_packet *pkts, size_t npkts, void *tiles, size_t tiles_cap, void *gen,
                                 size_t gen_cap, uint64_t *ntiles, uint64_t *ngen) {
    hdfs_crc::HostPlan plan;
    const int rc = hdfs_crc::build_plan(pkts, npkts, &plan);
    if (rc) return rc;
    if (ntiles) *ntiles = plan.tiles.size();
    if (ngen) *ngen = plan.gen.size();
    if (tiles && tiles_cap)
        std::memcpy(tiles, plan.tiles.data(),
                    sizeof(hdfs_crc::FastTile) * (plan.tiles.size() < tiles_cap ? plan.tiles.size() : tiles_cap));
    if (gen && gen_cap)
        std::memcpy(gen, plan.gen.data(),
                    sizeof(hdfs_crc::GenItem) * (plan.gen.size() < gen_cap ? plan.gen.size() : gen_cap));
    return 0;
}

extern "C" int crc32c_debug_write_plan(const crc32c_buffer *buffers, uint32_t n_buffers, uint64_t bufferoffset,
                                       uint64_t len, uint64_t blockoffset, uint32_t packetsize, uint32_t bpc,
                                       uint64_t counts[6]) {
    hdfs_crc::HostPlan plan;
    const int rc = hdfs_crc::build_write_plan(buffers, n_buffers, bufferoffset, len, blockoffset, packetsize, bpc,
                                              hdfs_crc::kPoly, &plan);
    if (rc) return rc;
    if (counts) {
        counts[0] = plan.tiles.size();
        counts[1] = plan.gen.size();
        counts[2] = plan.seg.size();
        counts[3] = plan.pieces.size();
        counts[4] = plan.consts.size();
        counts[5] = plan.nchecksums;
    }
    return 0;
}

extern "C" size_t crc32c_debug_lds_image(void *dst, size_t cap, uint32_t *c_lg, uint32_t *c_small) {
    if (dst && cap >= hdfs_crc::kLdsBytes) hdfs_crc::build_lds_image(static_cast<uint8_t *>(dst));
    if (c_lg && c_small) hdfs_crc::affine_constants(c_lg, c_small);
    return hdfs_crc::kLdsBytes;
}

extern "C" size_t crc32c_debug_lds_image_s4(void *dst, size_t cap, uint32_t flags) {
    const uint32_t poly = (flags & CRC32C_TYPE_CRC32) ? hdfs_crc::kPolyIeee : hdfs_crc::kPoly;
    if (dst && cap >= hdfs_crc::kS4Bytes) hdfs_crc::build_lds_image_s4(static_cast<uint8_t *>(dst), poly);
    return hdfs_crc::kS4Bytes;
}

extern "C" void crc32c_debug_affine_constants(uint32_t flags, uint32_t *c_lg, uint32_t *c_small) {
    const uint32_t poly = (flags & CRC32C_TYPE_CRC32) ? hdfs_crc::kPolyIeee : hdfs_crc::kPoly;
    hdfs_crc::affine_constants(c_lg, c_small, poly);
}
