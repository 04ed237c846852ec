// plan.h -- host-side work decomposition of a packet batch for the GPU.
//
// A batch of packets (crc32c_packet: payload_off, len, bpc, out_idx) is cut
// the way hadoop_rpc_send_packet cuts each packet into chunks
// (hadooprpc.c:639, 733-742) and then regrouped into GPU work items:
//
//  * FastTile: up to 16 consecutive 512-byte blocks (8 KiB, one wave-tile)
//    of FULL chunks of one packet whose bpc is 512 << lg (lg = 0..4), at any
//    alignment.  A tile never straddles a chunk, so a wave finishes every
//    chunk it starts.
//  * GenItem: one chunk of any length / alignment (the short tail chunk of a
//    packet, or every chunk of a packet whose bpc does not fit the fast
//    tile), processed by half a wave.
#pragma once
#include <cstdint>
#include <vector>

#include "hdfs_crc32c.h"

namespace hdfs_crc {

constexpr uint32_t kTileBlocks = 16;  // 512-byte blocks per fast tile
constexpr uint32_t kBlockBytes = 512;

struct FastTile {
    uint64_t src;   // payload byte offset of the tile's first block
    uint32_t out;   // checksum index of the tile's first chunk
    uint32_t meta;  // bits 0-7: blocks in tile (1..16); bits 8-15: lg = log2(bpc / 512)
};
static_assert(sizeof(FastTile) == 16, "FastTile is 16 bytes");

struct GenItem {
    uint64_t src;  // payload byte offset of the chunk
    uint32_t out;  // checksum index
    uint32_t len;  // chunk length in bytes (>= 1)
};
static_assert(sizeof(GenItem) == 16, "GenItem is 16 bytes");

struct HostPlan {
    std::vector<FastTile> tiles;
    std::vector<GenItem> gen;
    uint64_t nchecksums = 0;     // max(out_idx + nchunks)
    uint64_t payload_bytes = 0;  // sum of packet lengths
    uint64_t payload_extent = 0; // max(payload_off + len)
};

// 0 or -EINVAL (bpc == 0, checksum index beyond 2^32).
int build_plan(const crc32c_packet *pkts, size_t npkts, HostPlan *plan);

}  // namespace hdfs_crc
