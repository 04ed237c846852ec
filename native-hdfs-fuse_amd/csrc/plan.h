// plan.h -- host-side work decomposition of a packet batch for the GPU.
//
// A batch of packets (crc32c_packet: payload_off, len, bpc, out_idx) is cut
// the way hadoop_rpc_send_packet cuts each packet into chunks
// (hadooprpc.c:639, 733-742) and then regrouped into GPU work items:
//
//  * FastTile, power-of-two form: up to 16 consecutive 512-byte blocks (8 KiB,
//    one wave-tile) of FULL chunks of one packet whose bpc is 512 << lg
//    (lg = 0..4), at any alignment.  A tile never straddles a chunk, so a
//    wave finishes every chunk it starts.
//  * FastTile, padded power-of-two form (pad bits set, bit 31 clear): up to
//    16 >> lg FULL chunks of one packet whose bpc is 512 << lg minus a pad
//    of 1..511 bytes (lg = 0..4: bpc 4..511, 513..1023, 1537..2047,
//    3585..4095, 7681..8191).  Each chunk is right-aligned into its 2^lg
//    virtual 512-byte blocks behind pad leading zeros, so the tile runs the
//    power-of-two reduce (no per-subtile gather): only the lanes of each
//    chunk's first block are masked, and the affine constant is bpc's.
//  * FastTile, half form (meta bit 30): up to 32 (M = 0: bpc 4..256), 10
//    (M = 1: bpc 513..768) or 6 (M = 2: bpc 1025..1280) FULL chunks of one
//    packet, each M whole 512-byte
//    blocks after a partial part of r = bpc - 512 M bytes right-aligned into
//    a 256-byte half block behind padh = 256 - r zeros; two chunks' partial
//    parts share one block (crc32c_device.h, half tiles).
//  * FastTile, general form (meta bit 31): a general item of up to 16 FULL
//    chunks of one packet with any other bpc in [4, 8192], k = ceil(bpc /
//    512) virtual 512-byte blocks per chunk.  Each chunk is right-aligned
//    into its k blocks (pad = 512 k - bpc leading zero bytes, which do not
//    change the CRC's linear part), so every block is a whole 512-byte
//    load.  The last item of a packet also carries the packet's short tail
//    chunk (tl >= 4 bytes, kt = ceil(tl / 512) more blocks).  One wave runs
//    the item's nch k + kt blocks as consecutive 16-block subtiles, so a
//    chunk may span two subtiles (bpc 1536: 16 chunks in exactly 3).
//  * GenItem: one chunk of any length / alignment (the short tail chunk of a
//    packet, or every chunk whose bpc fits neither tile form), processed by
//    half a wave.
//  * SegItem: one chunk whose bytes come from several buffers (a packet
//    assembled from Hadoop_Fuse_Buffers, hadooprpc.c:666-725), as a list of
//    GenPieces; zero-filled buffers (data == NULL) are simply absent.
//  * ConstRun: `count` consecutive checksums that all equal one value known
//    at plan time -- chunks made only of zero-fill buffers (ftruncate
//    extension, fuse.c:1137-1142): no payload byte is read for them.
#pragma once
#include <cstdint>
#include <vector>

#include "hdfs_crc32c.h"

namespace hdfs_crc {

constexpr uint32_t kTileBlocks = 16;  // 512-byte blocks per tile
constexpr uint32_t kBlockBytes = 512;
constexpr uint32_t kMaxTileBpc = kTileBlocks * kBlockBytes;  // 8192
constexpr uint32_t kGeneralTile = 0x80000000u;
constexpr uint32_t kHalfTile = 0x40000000u;

struct FastTile {
    // payload byte offset of the tile's first chunk (bits 0-47); general
    // form: bits 48-63 = tl, the length of a tail chunk after the nch full
    // ones (0 = none)
    uint64_t src;
    uint32_t out;   // checksum index of the tile's first chunk
    // power-of-two form: bits 0-7 = blocks in tile (1..16), bits 8-15 = lg = log2(bpc / 512);
    // padded power-of-two form: the same, bits 8-15 = lg = log2(k) and bits 18-26 = pad = 512 k - bpc;
    // half form: bit 30, bits 0-7 = chunks, bits 8-15 = M, bits 18-26 = padh = 256 - (bpc - 512 M);
    // general form: bit 31, bits 0-7 = subtiles ceil((nch * k + kt) / 16), bits 8-12 = k, bits 13-17 = nch
    //               (full chunks in the item, 1..16), bits 18-26 = pad = 512 k - bpc
    uint32_t meta;
};
static_assert(sizeof(FastTile) == 16, "FastTile is 16 bytes");
constexpr uint64_t kSrcMask = (1ull << 48) - 1;
constexpr uint32_t kGeneralChunks = 16;  // full chunks per general item

inline uint32_t padded_meta(uint32_t nb, uint32_t lg, uint32_t pad) { return nb | (lg << 8) | (pad << 18); }
inline uint32_t half_meta(uint32_t n, uint32_t m, uint32_t padh) { return kHalfTile | n | (m << 8) | (padh << 18); }
// pad of a power-of-two tile (0: unpadded; general tiles keep their own at the same bits)
inline uint32_t tile_pad_bits(uint32_t meta) { return (meta >> 18) & 511u; }

inline uint32_t general_meta(uint32_t nch, uint32_t k, uint32_t pad, uint32_t kt = 0) {
    return kGeneralTile | ((nch * k + kt + kTileBlocks - 1) / kTileBlocks) | (k << 8) | (nch << 13) | (pad << 18);
}

struct GenItem {
    uint64_t src;  // payload byte offset of the chunk
    uint32_t out;  // checksum index
    uint32_t len;  // chunk length in bytes (>= 1)
};
static_assert(sizeof(GenItem) == 16, "GenItem is 16 bytes");

struct GenPiece {
    uint64_t src;    // payload byte offset of the piece's first byte
    uint32_t start;  // chunk-relative position of that byte
    uint32_t len;    // bytes (>= 1)
};
static_assert(sizeof(GenPiece) == 16, "GenPiece is 16 bytes");

struct SegItem {
    uint32_t first;    // index of the chunk's first GenPiece
    uint32_t npieces;  // data pieces (zero-fill pieces are not listed); may be 0
    uint32_t out;      // checksum index
    uint32_t len;      // chunk length in bytes (>= 1)
};
static_assert(sizeof(SegItem) == 16, "SegItem is 16 bytes");

struct ConstRun {
    uint32_t out;    // first checksum index
    uint32_t count;  // checksums
    uint32_t value;  // the checksum (host order)
    uint32_t pad;
};
static_assert(sizeof(ConstRun) == 16, "ConstRun is 16 bytes");

// Checksums per ConstRun at most (a wave writes 64 per store).
constexpr uint32_t kConstRunMax = 1024;

struct HostPlan {
    std::vector<FastTile> tiles;
    std::vector<GenItem> gen;
    std::vector<SegItem> seg;
    std::vector<GenPiece> pieces;
    std::vector<ConstRun> consts;
    uint64_t nchecksums = 0;     // max(out_idx + nchunks)
    uint64_t payload_bytes = 0;  // sum of packet lengths (zero-fill bytes included)
    void clear();
    uint64_t items() const;      // work items of a launch (tiles, gen / seg pairs, const runs)
};

// 0 or -EINVAL (bpc == 0, checksum index beyond 2^32).  `absolute`: the
// payload offsets are device addresses (the plan is rebased afterwards); it
// only changes which chunks may take the padded general tile, whose loads
// start up to 15 bytes before a chunk (same 4 KiB page required then, else a
// payload offset >= 16).
int build_plan(const crc32c_packet *pkts, size_t npkts, HostPlan *plan, bool absolute = false);

// Appends one packet's work items (no reset; updates the totals).
int append_packet(const crc32c_packet &p, HostPlan *plan, bool absolute = false);

// hadoop_rpc_send_packets over a Hadoop_Fuse_Buffer_Pos (hadooprpc.c:815-860,
// 666-725): packetize `len` bytes written at `blockoffset`, then checksum every
// chunk of every packet in order (out index 0, 1, ...).  Buffer addresses are
// absolute (device addresses; NULL = zero fill).  Chunks inside one data
// buffer become tiles / gen items, chunks spanning buffers SegItems, chunks
// made of zero fill ConstRuns.  `poly` selects the CRC (for the constants).
// 0, -EINVAL (bad sizes, range beyond the buffers) or -E2BIG.
int build_write_plan(const crc32c_buffer *buffers, uint32_t n_buffers, uint64_t bufferoffset, uint64_t len,
                     uint64_t blockoffset, uint32_t packetsize, uint32_t bpc, uint32_t poly, HostPlan *plan);

// Rebases every payload address of an absolute plan to offsets from *base
// (the lowest address read, rounded down to 16; 0 when nothing is read).
void rebase_plan(HostPlan *plan, uint64_t *base);

}  // namespace hdfs_crc
