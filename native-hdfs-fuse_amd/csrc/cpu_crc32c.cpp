// cpu_crc32c.cpp -- the drop-in scalar export `crc32c(crc, buf, len)`.
//
// Replaces src/crc32c.c:333-343 with identical semantics: `crc` is a finished
// CRC32C (pre-inverted on entry, post-inverted on exit, crc32c.c:237/312),
// any alignment, len == 0 returns crc, thread-safe, cannot fail.  It is the
// host path for single calls; batches go to the GPU (crc32c_runtime.hip).
//
// Two host implementations, chosen once by CPUID:
//  * SSE4.2 `crc32` instruction (3-cycle latency, 1 per cycle): the buffer
//    is consumed in groups of three consecutive stripes, run as three
//    independent register chains and merged with precomputed "append S zero
//    bytes" operators (crc32c.c:249-289 uses the same idea with two stripe
//    sizes, 8192 and 256).  A cascade of stripe sizes 8192 / 1024 / 336 /
//    168 also covers the sizes the checksum loop actually passes: a 512-byte
//    chunk is three 168-byte chains + 8 bytes, about half the latency of one
//    64-step chain (the reference's path for 512 B, crc32c.c:293-299).
//  * portable slicing-by-8 tables (crc32c.c:78-107's fallback role).
#include <algorithm>
#include <cerrno>
#include <cstring>
#include <mutex>

#include "crc_math.h"
#include "hdfs_crc32c.h"

namespace {

using hdfs_crc::Gf2Op;

constexpr size_t kStripes[] = {8192, 1024, 336, 168};
constexpr int kNumStripes = 4;

uint32_t g_slice[8][256];
uint32_t g_stripe_shift[kNumStripes][4][256];  // Z^stripe applied to byte k of a register
bool g_have_sse42 = false;
std::once_flag g_once;

void init_once() {
    const uint32_t *t0 = hdfs_crc::byte_table();
    for (int b = 0; b < 256; ++b) {
        g_slice[0][b] = t0[b];
        for (int k = 1; k < 8; ++k) g_slice[k][b] = (g_slice[k - 1][b] >> 8) ^ t0[g_slice[k - 1][b] & 0xffu];
    }
    for (int s = 0; s < kNumStripes; ++s) {
        const Gf2Op z = hdfs_crc::op_zeros(kStripes[s]);
        for (int k = 0; k < 4; ++k)
            for (uint32_t b = 0; b < 256; ++b) g_stripe_shift[s][k][b] = z.apply(b << (8 * k));
    }
#if defined(__x86_64__) || defined(__i386__)
    __builtin_cpu_init();
    g_have_sse42 = __builtin_cpu_supports("sse4.2");
#endif
}

inline uint32_t stripe_shift(int s, uint32_t r) {
    const uint32_t(&t)[4][256] = g_stripe_shift[s];
    return t[0][r & 0xff] ^ t[1][(r >> 8) & 0xff] ^ t[2][(r >> 16) & 0xff] ^ t[3][r >> 24];
}

// Register update over raw bytes (no conditioning), portable.
uint32_t reg_update_sw(uint32_t r, const uint8_t *p, size_t n) {
    for (; n && (reinterpret_cast<uintptr_t>(p) & 7u); --n) r = (r >> 8) ^ g_slice[0][(r ^ *p++) & 0xffu];
    for (; n >= 8; n -= 8, p += 8) {
        uint64_t w;
        std::memcpy(&w, p, 8);
        w ^= r;
        r = g_slice[7][w & 0xff] ^ g_slice[6][(w >> 8) & 0xff] ^ g_slice[5][(w >> 16) & 0xff] ^
            g_slice[4][(w >> 24) & 0xff] ^ g_slice[3][(w >> 32) & 0xff] ^ g_slice[2][(w >> 40) & 0xff] ^
            g_slice[1][(w >> 48) & 0xff] ^ g_slice[0][w >> 56];
    }
    for (; n; --n) r = (r >> 8) ^ g_slice[0][(r ^ *p++) & 0xffu];
    return r;
}

#if defined(__x86_64__)
// Three chains over the stripes [p, p+S), [p+S, p+2S), [p+2S, p+3S); the
// first continues r, the other two start from 0 and are shifted into place.
template <int SI>
__attribute__((target("sse4.2"))) inline uint64_t three_stripes(uint64_t r, const uint8_t *p) {
    constexpr size_t S = kStripes[SI];
    uint64_t a = r, b = 0, c = 0;
    for (size_t i = 0; i < S; i += 8) {
        uint64_t wa, wb, wc;
        std::memcpy(&wa, p + i, 8);
        std::memcpy(&wb, p + S + i, 8);
        std::memcpy(&wc, p + 2 * S + i, 8);
        a = __builtin_ia32_crc32di(a, wa);
        b = __builtin_ia32_crc32di(b, wb);
        c = __builtin_ia32_crc32di(c, wc);
    }
    return stripe_shift(SI, stripe_shift(SI, uint32_t(a)) ^ uint32_t(b)) ^ uint32_t(c);
}

// Software prefetch distance of three_chunks, in groups of three chunks
// beyond the next one.
constexpr size_t kPrefetchGroups = 1;

// Three whole chunks of `bpc` bytes (a multiple of 8) at p, p + bpc, p + 2 bpc,
// each from crc = 0: three independent crc32q chains interleaved, so the
// instruction's 3-cycle latency is hidden without any merge step (the
// reference runs one dependent chain per 512-byte chunk, crc32c.c:293-299).
__attribute__((target("sse4.2"))) void three_chunks(const uint8_t *p, size_t bpc, uint32_t out[3]) {
    uint64_t a = 0xffffffffu, b = 0xffffffffu, c = 0xffffffffu;
    const uint8_t *next = p + 3 * bpc + 3 * kPrefetchGroups * bpc;
    for (size_t i = 0; i < bpc; i += 8) {
        if ((i & 63) == 0) {  // the hardware prefetchers miss three interleaved streams
            __builtin_prefetch(next + i);
            __builtin_prefetch(next + bpc + i);
            __builtin_prefetch(next + 2 * bpc + i);
        }
        uint64_t wa, wb, wc;
        std::memcpy(&wa, p + i, 8);
        std::memcpy(&wb, p + bpc + i, 8);
        std::memcpy(&wc, p + 2 * bpc + i, 8);
        a = __builtin_ia32_crc32di(a, wa);
        b = __builtin_ia32_crc32di(b, wb);
        c = __builtin_ia32_crc32di(c, wc);
    }
    out[0] = ~uint32_t(a);
    out[1] = ~uint32_t(b);
    out[2] = ~uint32_t(c);
}

__attribute__((target("sse4.2"))) uint32_t reg_update_hw(uint32_t r32, const uint8_t *p, size_t n) {
    uint64_t r = r32;
    for (; n && (reinterpret_cast<uintptr_t>(p) & 7u); --n) r = __builtin_ia32_crc32qi(uint32_t(r), *p++);
    for (; n >= 3 * kStripes[0]; n -= 3 * kStripes[0], p += 3 * kStripes[0]) r = three_stripes<0>(r, p);
    for (; n >= 3 * kStripes[1]; n -= 3 * kStripes[1], p += 3 * kStripes[1]) r = three_stripes<1>(r, p);
    for (; n >= 3 * kStripes[2]; n -= 3 * kStripes[2], p += 3 * kStripes[2]) r = three_stripes<2>(r, p);
    for (; n >= 3 * kStripes[3]; n -= 3 * kStripes[3], p += 3 * kStripes[3]) r = three_stripes<3>(r, p);
    for (; n >= 8; n -= 8, p += 8) {
        uint64_t w;
        std::memcpy(&w, p, 8);
        r = __builtin_ia32_crc32di(r, w);
    }
    for (; n; --n) r = __builtin_ia32_crc32qi(uint32_t(r), *p++);
    return uint32_t(r);
}
#endif

}  // namespace

extern "C" uint32_t crc32c(uint32_t crc, const void *buf, size_t len) {
    std::call_once(g_once, init_once);
    const uint8_t *p = static_cast<const uint8_t *>(buf);
    uint32_t r = ~crc;
#if defined(__x86_64__)
    if (g_have_sse42) return ~reg_update_hw(r, p, len);
#endif
    return ~reg_update_sw(r, p, len);
}

namespace {
uint32_t g_ieee[8][256];
std::once_flag g_ieee_once;

void init_ieee() {
    const uint32_t *t0 = hdfs_crc::byte_table(hdfs_crc::kPolyIeee);
    for (int b = 0; b < 256; ++b) {
        g_ieee[0][b] = t0[b];
        for (int k = 1; k < 8; ++k) g_ieee[k][b] = (g_ieee[k - 1][b] >> 8) ^ t0[g_ieee[k - 1][b] & 0xffu];
    }
}
}  // namespace

extern "C" uint32_t hdfs_crc32(uint32_t crc, const void *buf, size_t len) {
    // Slicing-by-8 over the IEEE tables (x86 has no CRC32 instruction for
    // this polynomial); little-endian host, as crc32c.c:75-77 assumes too.
    std::call_once(g_ieee_once, init_ieee);
    const uint8_t *p = static_cast<const uint8_t *>(buf);
    uint32_t r = ~crc;
    size_t n = len;
    for (; n && (reinterpret_cast<uintptr_t>(p) & 7u); --n) r = (r >> 8) ^ g_ieee[0][(r ^ *p++) & 0xffu];
    for (; n >= 8; n -= 8, p += 8) {
        uint64_t w;
        std::memcpy(&w, p, 8);
        w ^= r;
        r = g_ieee[7][w & 0xff] ^ g_ieee[6][(w >> 8) & 0xff] ^ g_ieee[5][(w >> 16) & 0xff] ^
            g_ieee[4][(w >> 24) & 0xff] ^ g_ieee[3][(w >> 32) & 0xff] ^ g_ieee[2][(w >> 40) & 0xff] ^
            g_ieee[1][(w >> 48) & 0xff] ^ g_ieee[0][w >> 56];
    }
    for (; n; --n) r = (r >> 8) ^ g_ieee[0][(r ^ *p++) & 0xffu];
    return ~r;
}

extern "C" int crc32c_chunks_cpu(const void *packet, size_t len, uint32_t bpc, uint32_t *out, uint32_t flags) {
    // hadooprpc.c:733-742 on the host: chunk i = crc32c(0, packet + i*bpc,
    // min(bpc, len - i*bpc)), htonl'd with CRC32C_BIG_ENDIAN (71-75).
    if (bpc == 0 || (flags & ~uint32_t(CRC32C_BIG_ENDIAN | CRC32C_TYPE_CRC32))) return -EINVAL;
    if (len && (!packet || !out)) return -EINVAL;
    const uint8_t *p = static_cast<const uint8_t *>(packet);
    const size_t n = (len + bpc - 1) / bpc;
    size_t i = 0;
    if (flags & CRC32C_TYPE_CRC32) {
        for (; i < n; ++i) out[i] = hdfs_crc32(0, p + i * bpc, std::min<size_t>(bpc, len - i * bpc));
    } else {
        std::call_once(g_once, init_once);
#if defined(__x86_64__)
        if (g_have_sse42 && bpc % 8 == 0)
            for (; i + 3 <= len / bpc; i += 3) three_chunks(p + i * bpc, bpc, out + i);
#endif
        for (; i < n; ++i) out[i] = crc32c(0, p + i * bpc, std::min<size_t>(bpc, len - i * bpc));
    }
    if (flags & CRC32C_BIG_ENDIAN)
        for (size_t k = 0; k < n; ++k) out[k] = __builtin_bswap32(out[k]);
    return 0;
}

extern "C" uint64_t crc32c_nchunks(uint64_t len, uint32_t bpc) {
    // roundup(len, bpc) (hadooprpc.c:639, roundup.h:7-11).
    return bpc ? (len + bpc - 1) / bpc : 0;
}

extern "C" uint64_t crc32c_batch_nchecksums(const crc32c_packet *pkts, size_t npkts) {
    uint64_t n = 0;
    for (size_t i = 0; pkts && i < npkts; ++i)
        if (pkts[i].len) {
            // (len > 0 with bpc == 0 is an invalid packet, which every batch
            // entry point refuses with -EINVAL; it counts nothing here)
            const uint64_t end = pkts[i].out_idx + crc32c_nchunks(pkts[i].len, pkts[i].bpc);
            if (end > n) n = end;
        }
    return n;
}

extern "C" uint64_t crc32c_packetize(uint64_t len, uint64_t blockoffset, uint32_t packetsize, uint32_t bpc,
                                     uint64_t *lens, uint64_t max) {
    // hadooprpc.c:827-857.  A packet that would start off a chunk boundary
    // only finishes that chunk (832-840); a zero-length packet ends the
    // block (644, 853-856).
    if (bpc == 0 || packetsize == 0) return 0;
    uint64_t sent = 0, n = 0;
    for (;;) {
        uint64_t plen = len - sent < packetsize ? len - sent : packetsize;
        const uint64_t past = (blockoffset + sent) % bpc;
        if (plen > 0 && past != 0) {
            plen = bpc - past;
            // The reference only asserts that the trimmed packet fits the
            // remaining bytes (hadooprpc.c:622); clamp instead of overrunning.
            if (plen > len - sent) plen = len - sent;
        }
        if (lens && n < max) lens[n] = plen;
        ++n;
        if (plen == 0) break;
        sent += plen;
    }
    return n;
}
