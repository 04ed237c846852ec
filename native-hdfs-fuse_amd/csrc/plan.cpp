// plan.cpp -- see plan.h.
#include "plan.h"
#include "hdfs_crc32c.h"

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

int build_plan(const crc32c_packet *pkts, size_t npkts, HostPlan *plan) {
    plan->tiles.clear();
    plan->gen.clear();
    plan->nchecksums = plan->payload_bytes = plan->payload_extent = 0;
    for (size_t i = 0; i < npkts; ++i) {
        const crc32c_packet &p = pkts[i];
        if (p.bpc == 0) return -EINVAL;
        if (p.len == 0) continue;  // last-packet marker: no checksums (hadooprpc.c:644, 666)
        const uint64_t n = (uint64_t(p.len) + p.bpc - 1) / p.bpc;  // hadooprpc.c:639
        if (p.out_idx + n > (1ull << 32)) return -EINVAL;
        if (p.out_idx + n > plan->nchecksums) plan->nchecksums = p.out_idx + n;
        plan->payload_bytes += p.len;
        if (p.payload_off + p.len > plan->payload_extent) plan->payload_extent = p.payload_off + p.len;

        const uint64_t nfull = p.len / p.bpc;
        const uint32_t tail = p.len % p.bpc;
        const int lg = fast_lg(p.bpc);
        // Any alignment: a tile off 16-byte alignment is read with unaligned
        // dwordx4 buffer loads (config 2 five bytes off: 55 instead of 42.5
        // us; through the general path it took 220 us).
        if (lg >= 0) {
            const uint64_t blocks = nfull << lg;  // 512-byte blocks of full chunks
            for (uint64_t b = 0; b < blocks; b += kTileBlocks) {
                const uint64_t nb = blocks - b < kTileBlocks ? blocks - b : kTileBlocks;
                FastTile t;
                t.src = p.payload_off + b * kBlockBytes;
                t.out = uint32_t(p.out_idx + (b >> lg));
                t.meta = uint32_t(nb) | (uint32_t(lg) << 8);
                plan->tiles.push_back(t);
            }
        } else {
            for (uint64_t c = 0; c < nfull; ++c) {
                GenItem g;
                g.src = p.payload_off + c * p.bpc;
                g.out = uint32_t(p.out_idx + c);
                g.len = p.bpc;
                plan->gen.push_back(g);
            }
        }
        if (tail) {
            GenItem g;
            g.src = p.payload_off + nfull * p.bpc;
            g.out = uint32_t(p.out_idx + nfull);
            g.len = tail;
            plan->gen.push_back(g);
        }
    }
    return 0;
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
