// framing.cpp -- host-side companions of the checksum path (SURVEY.md
// section 8f, "next" rows 2 and 4):
//
//  * crc32c_frame_packets: the per-packet prefix hadoop_rpc_send_packet
//    writes with 1 + 1 + 1 + n separate sendto calls (src/hadooprpc.c:596-664,
//    733-748) -- PLEN, HLEN, the PacketHeaderProto, the n checksums -- built
//    for a whole batch in one pass, so that each packet goes out as one
//    sendmsg of two iovecs (prefix, data).
//  * crc32c_block_md5: OpBlockChecksumResponseProto.md5 (datatransfer.proto:
//    262-267), the MD5 of a block's big-endian checksum bytes.
#include <cstring>

#include "hdfs_crc32c.h"

namespace {

inline void put_be32(uint8_t *p, uint32_t v) {
    p[0] = uint8_t(v >> 24);
    p[1] = uint8_t(v >> 16);
    p[2] = uint8_t(v >> 8);
    p[3] = uint8_t(v);
}

inline void put_le(uint8_t *p, uint64_t v, int n) {
    for (int i = 0; i < n; ++i) p[i] = uint8_t(v >> (8 * i));
}

// PacketHeaderProto (datatransfer.proto:184-191) in protobuf wire format.
// Every field is fixed-length, so the header is always 25 bytes: keys
// 0x09 / 0x11 (fields 1, 2: sfixed64), 0x18 (field 3: bool varint), 0x25
// (field 4: sfixed32); syncBlock is optional and left unset, as the
// reference does (hadooprpc.c:641-644).
constexpr uint32_t kHeaderLen = 25;

void put_header(uint8_t *p, int64_t offset_in_block, int64_t seqno, bool last, int32_t data_len) {
    p[0] = 0x09;
    put_le(p + 1, uint64_t(offset_in_block), 8);
    p[9] = 0x11;
    put_le(p + 10, uint64_t(seqno), 8);
    p[18] = 0x18;
    p[19] = last ? 1 : 0;
    p[20] = 0x25;
    put_le(p + 21, uint32_t(data_len), 4);
}

// ---- MD5 (RFC 1321), for crc32c_block_md5 ----------------------------------
struct Md5 {
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    uint64_t nbytes = 0;
    uint8_t buf[64];
    size_t fill = 0;

    static uint32_t rotl(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }

    void block(const uint8_t *p) {
        static const uint32_t K[64] = {
            0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
            0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
            0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
            0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
            0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
            0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
            0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
            0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
        static const int S[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
        uint32_t m[16];
        for (int i = 0; i < 16; ++i)
            m[i] = uint32_t(p[4 * i]) | uint32_t(p[4 * i + 1]) << 8 | uint32_t(p[4 * i + 2]) << 16 |
                   uint32_t(p[4 * i + 3]) << 24;
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
        for (int i = 0; i < 64; ++i) {
            uint32_t f;
            int g;
            if (i < 16) {
                f = (b & c) | (~b & d);
                g = i;
            } else if (i < 32) {
                f = (d & b) | (~d & c);
                g = (5 * i + 1) & 15;
            } else if (i < 48) {
                f = b ^ c ^ d;
                g = (3 * i + 5) & 15;
            } else {
                f = c ^ (b | ~d);
                g = (7 * i) & 15;
            }
            const uint32_t t = d;
            d = c;
            c = b;
            b = b + rotl(a + f + K[i] + m[g], S[(i >> 4) * 4 + (i & 3)]);
            a = t;
        }
        h[0] += a;
        h[1] += b;
        h[2] += c;
        h[3] += d;
    }

    void update(const uint8_t *p, size_t n) {
        nbytes += n;
        while (n) {
            const size_t k = fill + n < 64 ? n : 64 - fill;
            std::memcpy(buf + fill, p, k);
            fill += k;
            p += k;
            n -= k;
            if (fill == 64) {
                block(buf);
                fill = 0;
            }
        }
    }

    void finish(uint8_t out[16]) {
        const uint64_t bits = nbytes * 8;
        const uint8_t pad = 0x80;
        update(&pad, 1);
        const uint8_t zero = 0;
        while (fill != 56) update(&zero, 1);
        uint8_t len[8];
        put_le(len, bits, 8);
        update(len, 8);
        for (int i = 0; i < 4; ++i) put_le(out + 4 * i, h[i], 4);
    }
};

}  // namespace

extern "C" size_t crc32c_frame_packets(const crc32c_packet *pkts, size_t npkts, const uint32_t *sums,
                                       uint32_t flags, uint64_t block_offset, int64_t first_seqno,
                                       uint32_t checksum_len, uint8_t *out, size_t cap, uint64_t *prefix_off) {
    if (npkts && !pkts) return 0;
    if (checksum_len != 0 && checksum_len != 4) return 0;
    size_t need = 0;
    for (size_t i = 0; i < npkts; ++i)
        need += 4 + 2 + kHeaderLen + size_t(checksum_len) * crc32c_nchunks(pkts[i].len, pkts[i].bpc);
    if (!out || cap < need) return need;
    if (checksum_len && need && !sums) return 0;
    size_t o = 0;
    const uint64_t base = npkts ? pkts[0].payload_off : 0;
    for (size_t i = 0; i < npkts; ++i) {
        const crc32c_packet &p = pkts[i];
        const uint64_t n = checksum_len ? crc32c_nchunks(p.len, p.bpc) : 0;
        if (prefix_off) prefix_off[i] = o;
        // PLEN counts itself, the checksums and the data (hadooprpc.c:640)
        put_be32(out + o, uint32_t(4 + n * checksum_len + p.len));
        out[o + 4] = uint8_t(kHeaderLen >> 8);
        out[o + 5] = uint8_t(kHeaderLen);
        put_header(out + o + 6, int64_t(block_offset + (p.payload_off - base)), first_seqno + int64_t(i), p.len == 0,
                   int32_t(p.len));
        uint8_t *c = out + o + 6 + kHeaderLen;
        for (uint64_t k = 0; k < n; ++k) {
            const uint32_t v = sums[p.out_idx + k];
            if (flags & CRC32C_BIG_ENDIAN)
                std::memcpy(c + 4 * k, &v, 4);  // already wire order
            else
                put_be32(c + 4 * k, v);
        }
        o += 6 + kHeaderLen + n * checksum_len;
    }
    if (prefix_off) prefix_off[npkts] = o;
    return o;
}

extern "C" void crc32c_block_md5(const uint32_t *sums, size_t n, uint32_t flags, uint8_t md5[16]) {
    Md5 m;
    uint8_t be[4 * 256];
    size_t k = 0;
    while (k < n) {
        const size_t c = n - k < 256 ? n - k : 256;
        for (size_t j = 0; j < c; ++j) {
            if (flags & CRC32C_BIG_ENDIAN)
                std::memcpy(be + 4 * j, sums + k + j, 4);
            else
                put_be32(be + 4 * j, sums[k + j]);
        }
        m.update(be, 4 * c);
        k += c;
    }
    m.finish(md5);
}
