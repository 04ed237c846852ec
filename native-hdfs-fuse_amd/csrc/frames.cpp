// frames.cpp -- the read side's packet stream ("next"
// row 1).  A DataNode answering OP_READ_BLOCK with sendChecksums sends, per
// packet, PLEN (u32 BE) | HLEN (u16 BE) | PacketHeaderProto | checksums
// (u32 BE each) | data (hadoop_rpc_receive_packets reads it field by field,
// src/hadooprpc.c:497-584; PLEN = 4 + checksums + data, hadooprpc.c:640).
// The reads start at ReadOpChecksumInfoProto.chunkOffset, the requested
// offset aligned backwards to a chunk boundary (datatransfer.proto:218-227).
//
//  * crc32c_parse_frames: the frames of a receive buffer (whole frames only,
//    so a caller can resume when more bytes arrive), header fields decoded.
//  * crc32c_verify_frames_host: parses a run of frames and verifies every
//    data chunk against the checksums interleaved in front of it on the GPU
//    (crc32c_verify_host over the frame buffer itself: the data is read in
//    place, only the 4-byte checksums are gathered into an array).
#include <cerrno>
#include <cstring>
#include <vector>

#include "errors.h"
#include "hdfs_crc32c.h"

using hdfs_crc::fail;

namespace {

inline uint32_t get_be32(const uint8_t *p) {
    return uint32_t(p[0]) << 24 | uint32_t(p[1]) << 16 | uint32_t(p[2]) << 8 | uint32_t(p[3]);
}

inline uint64_t get_le(const uint8_t *p, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; ++i) v |= uint64_t(p[i]) << (8 * i);
    return v;
}

// Protobuf varint at p (< end): the value, or false when malformed.
bool varint(const uint8_t *&p, const uint8_t *end, uint64_t *v) {
    uint64_t r = 0;
    for (int s = 0; s < 64; s += 7) {
        if (p >= end) return false;
        const uint8_t b = *p++;
        r |= uint64_t(b & 0x7f) << s;
        if (!(b & 0x80)) {
            *v = r;
            return true;
        }
    }
    return false;
}

// PacketHeaderProto (datatransfer.proto:184-191): offsetInBlock, seqno,
// lastPacketInBlock and dataLen are required; unknown fields are skipped.
bool parse_header(const uint8_t *p, size_t n, crc32c_frame_info *f) {
    const uint8_t *end = p + n;
    unsigned seen = 0;
    while (p < end) {
        uint64_t key;
        if (!varint(p, end, &key)) return false;
        const uint32_t field = uint32_t(key >> 3), wt = uint32_t(key & 7);
        uint64_t v = 0;
        switch (wt) {
        case 0:
            if (!varint(p, end, &v)) return false;
            break;
        case 1:
            if (end - p < 8) return false;
            v = get_le(p, 8);
            p += 8;
            break;
        case 5:
            if (end - p < 4) return false;
            v = get_le(p, 4);
            p += 4;
            break;
        case 2: {
            uint64_t len;
            if (!varint(p, end, &len) || len > uint64_t(end - p)) return false;
            p += len;
            continue;
        }
        default:
            return false;
        }
        if (field == 1 && wt == 1) f->offset_in_block = int64_t(v), seen |= 1;
        if (field == 2 && wt == 1) f->seqno = int64_t(v), seen |= 2;
        if (field == 3 && wt == 0) f->last = v ? 1 : 0, seen |= 4;
        if (field == 4 && wt == 5) f->data_len = uint32_t(v), seen |= 8;
    }
    return seen == 15 && int32_t(f->data_len) >= 0;
}

}  // namespace

extern "C" int64_t crc32c_parse_frames(const void *frames, size_t bytes, crc32c_frame_info *info, size_t cap,
                                       uint64_t *consumed) {
    const uint8_t *b = static_cast<const uint8_t *>(frames);
    size_t o = 0;
    int64_t n = 0;
    if (consumed) *consumed = 0;
    if (bytes && !b) return fail(-EINVAL, "frames == NULL");
    while (bytes - o >= 6) {
        const uint32_t plen = get_be32(b + o);
        const uint32_t hlen = uint32_t(b[o + 4]) << 8 | b[o + 5];
        if (plen < 4) return fail(-EBADMSG, "frame %lld at %zu: PLEN %u < 4", (long long)n, o, plen);
        const uint64_t total = 6ull + hlen + (plen - 4ull);
        if (bytes - o < total) break;  // the rest has not arrived yet
        crc32c_frame_info f;
        std::memset(&f, 0, sizeof f);
        if (!parse_header(b + o + 6, hlen, &f))
            return fail(-EBADMSG, "frame %lld at %zu: malformed PacketHeaderProto", (long long)n, o);
        if (f.data_len > plen - 4u)
            return fail(-EBADMSG, "frame %lld at %zu: dataLen %u > PLEN - 4", (long long)n, o, f.data_len);
        const uint32_t sum_bytes = plen - 4u - f.data_len;
        if (sum_bytes % 4)
            return fail(-EBADMSG, "frame %lld at %zu: %u checksum bytes", (long long)n, o, sum_bytes);
        f.frame_off = o;
        f.sums_off = o + 6 + hlen;
        f.data_off = f.sums_off + sum_bytes;
        f.nsums = sum_bytes / 4;
        if (info && size_t(n) < cap) info[n] = f;
        ++n;
        o += total;
        if (consumed) *consumed = o;
        if (f.last) break;  // lastPacketInBlock: nothing of this block follows
    }
    return n;
}

extern "C" int crc32c_verify_frames_host(crc32c_ctx *ctx, const void *frames, size_t bytes, uint32_t bpc,
                                         uint64_t chunk_offset, uint32_t flags, crc32c_frames_result *res) {
    if (!res || !bpc || (flags & ~(CRC32C_TYPE_CRC32 | CRC32C_CPU_FALLBACK)))
        return fail(-EINVAL, "res == NULL, bytesPerChecksum == 0 or unknown flags");
    std::memset(res, 0, sizeof *res);
    res->first_bad = UINT64_MAX;
    res->first_bad_offset = -1;
    uint64_t consumed = 0;
    const int64_t n = crc32c_parse_frames(frames, bytes, nullptr, 0, &consumed);
    if (n < 0) return int(n);
    std::vector<crc32c_frame_info> info;
    info.resize(size_t(n));
    crc32c_parse_frames(frames, bytes, info.data(), info.size(), &consumed);
    const uint8_t *b = static_cast<const uint8_t *>(frames);
    std::vector<crc32c_packet> pkts;
    std::vector<uint32_t> expected;
    std::vector<int64_t> chunk_pos;  // offsetInBlock of each checksum's chunk
    int64_t next = int64_t(chunk_offset);
    for (const crc32c_frame_info &f : info) {
        res->packets++;
        if (f.last) res->last_packet = 1;
        if (f.data_len == 0) continue;
        // Every data packet starts on a chunk boundary, the first at
        // chunkOffset, the others where the previous one ended.
        if (f.offset_in_block != next || uint64_t(f.offset_in_block) % bpc)
            return fail(-EBADMSG, "packet seqno %lld: offsetInBlock %lld, expected %lld on a %u-byte chunk boundary",
                        (long long)f.seqno, (long long)f.offset_in_block, (long long)next, bpc);
        const uint64_t nch = crc32c_nchunks(f.data_len, bpc);
        if (f.nsums != nch)
            return fail(-EBADMSG, "packet seqno %lld: %u checksums for %u bytes (%llu expected)", (long long)f.seqno,
                        f.nsums, f.data_len, (unsigned long long)nch);
        crc32c_packet p;
        p.payload_off = f.data_off;
        p.out_idx = expected.size();
        p.len = f.data_len;
        p.bpc = bpc;
        pkts.push_back(p);
        for (uint64_t k = 0; k < nch; ++k) {
            uint32_t v;
            std::memcpy(&v, b + f.sums_off + 4 * k, 4);  // wire order, compared as such
            expected.push_back(v);
            chunk_pos.push_back(f.offset_in_block + int64_t(k * bpc));
        }
        res->data_bytes += f.data_len;
        next = f.offset_in_block + f.data_len;
    }
    res->checksums = expected.size();
    res->consumed = consumed;
    if (pkts.empty()) return 0;
    uint64_t first = UINT64_MAX;
    const uint32_t vflags = (flags & (CRC32C_TYPE_CRC32 | CRC32C_CPU_FALLBACK)) | CRC32C_BIG_ENDIAN;
    const int64_t bad = crc32c_verify_host(ctx, frames, pkts.data(), pkts.size(), expected.data(), vflags, &first);
    if (bad < 0) return int(bad);
    res->mismatches = uint64_t(bad);
    res->first_bad = first;
    if (first != UINT64_MAX) res->first_bad_offset = chunk_pos[size_t(first)];
    return 0;
}
