// Host-code sanitizer run (TEST INFRASTRUCTURE): the host-only sources of
// libhdfs_crc32c.so (crc_math.cpp, cpu_crc32c.cpp, plan.cpp, framing.cpp,
// frames.cpp)
// built with -fsanitize=address,undefined and driven over randomized inputs
// whose buffers are heap blocks of exactly the size the ABI promises to touch,
// so a read or write one byte past them aborts.  Results are compared with the
// oracle restatement (oracle/crc32c_oracle.c) as the checker.  GPU code is not
// sanitized here (no GPU sanitizer on this pool); built and run by
// tests/test_host_sanitize.py.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <random>
#include <vector>

#include "crc_math.h"
#include "hdfs_crc32c.h"
#include "plan.h"

extern "C" {
uint32_t oracle_crc32c_bytewise(uint32_t crc, const void *buf, size_t len);
uint64_t oracle_chunks(const void *packet, uint64_t len, uint32_t bpc, uint32_t *out, int big_endian);
uint64_t oracle_packetize(uint64_t len, uint64_t blockoffset, uint32_t packetsize, uint32_t bpc, uint64_t *lens,
                          uint64_t max);
int crc32c_debug_plan(const crc32c_packet *pkts, size_t npkts, void *tiles, size_t tiles_cap, void *gen,
                      size_t gen_cap, uint64_t *ntiles, uint64_t *ngen);
size_t crc32c_debug_lds_image_s4(void *dst, size_t cap, uint32_t flags);
size_t crc32c_debug_lds_image(void *dst, size_t cap, uint32_t *c_lg, uint32_t *c_small);

// frames.cpp verifies through the GPU runtime, which is not part of this
// host-only build: only its parser is exercised here.
int64_t crc32c_verify_host(crc32c_ctx *, const void *, const crc32c_packet *, size_t, const uint32_t *, uint32_t,
                           uint64_t *) {
    return -19;
}
}

namespace {

int g_fail = 0;
#define CHECK(cond, ...)                                         \
    do {                                                         \
        if (!(cond)) {                                           \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);                   \
            std::fprintf(stderr, "\n");                          \
            if (++g_fail > 20) std::exit(1);                     \
        }                                                        \
    } while (0)

// zlib's crc32, bit by bit (the CRC32 type's checker).
uint32_t crc32_bitwise(uint32_t crc, const uint8_t *p, size_t n) {
    crc = ~crc;
    for (size_t i = 0; i < n; ++i) {
        crc ^= p[i];
        for (int k = 0; k < 8; ++k) crc = (crc >> 1) ^ (0xedb88320u & (0u - (crc & 1u)));
    }
    return ~crc;
}

uint8_t *exact_bytes(std::mt19937_64 &rng, size_t n) {
    uint8_t *p = static_cast<uint8_t *>(std::malloc(n ? n : 1));
    for (size_t i = 0; i < n; ++i) p[i] = uint8_t(rng());
    return p;
}

void scalar_and_chunks(std::mt19937_64 &rng) {
    const uint32_t bpcs[] = {1, 3, 7, 100, 511, 512, 513, 1024, 1536, 4096, 65536};
    for (int it = 0; it < 3000; ++it) {
        const size_t len = (it % 10 == 0) ? rng() % 40 : rng() % 70000;
        uint8_t *buf = exact_bytes(rng, len);
        // crc32c in two incremental pieces == the oracle in one
        const size_t cut = len ? rng() % (len + 1) : 0;
        const uint32_t a = crc32c(crc32c(0, buf, cut), buf + cut, len - cut);
        CHECK(a == oracle_crc32c_bytewise(0, buf, len), "crc32c len %zu cut %zu", len, cut);
        CHECK(hdfs_crc32(hdfs_crc32(0, buf, cut), buf + cut, len - cut) == crc32_bitwise(0, buf, len),
              "hdfs_crc32 len %zu", len);
        // per-packet loop into an exactly sized checksum array
        const uint32_t bpc = bpcs[rng() % (sizeof(bpcs) / sizeof(bpcs[0]))];
        const uint32_t flags = uint32_t(rng() % 4);  // BIG_ENDIAN | TYPE_CRC32
        const uint64_t n = crc32c_nchunks(len, bpc);
        uint32_t *out = static_cast<uint32_t *>(std::malloc(n ? 4 * n : 1));
        uint32_t *want = static_cast<uint32_t *>(std::malloc(n ? 4 * n : 1));
        CHECK(crc32c_chunks_cpu(buf, len, bpc, out, flags) == 0, "chunks_cpu rc");
        if (flags & CRC32C_TYPE_CRC32) {
            for (uint64_t i = 0; i < n; ++i) {
                const size_t at = size_t(i) * bpc, m = len - at < bpc ? len - at : bpc;
                const uint32_t c = crc32_bitwise(0, buf + at, m);
                want[i] = (flags & CRC32C_BIG_ENDIAN) ? __builtin_bswap32(c) : c;
            }
        } else {
            CHECK(oracle_chunks(buf, len, bpc, want, int(flags & CRC32C_BIG_ENDIAN)) == n, "oracle n");
        }
        CHECK(n == 0 || std::memcmp(out, want, 4 * n) == 0, "chunks_cpu len %zu bpc %u flags %u", len, bpc,
              flags);
        std::free(out);
        std::free(want);
        std::free(buf);
    }
    CHECK(crc32c_chunks_cpu(nullptr, 1, 512, nullptr, 0) < 0, "NULL buffers rejected");
    uint32_t o;
    CHECK(crc32c_chunks_cpu(&o, 1, 0, &o, 0) < 0, "bpc 0 rejected");
}

void packetize(std::mt19937_64 &rng) {
    for (int it = 0; it < 2000; ++it) {
        const uint64_t len = rng() % (1u << 23);
        const uint64_t off = rng() % (1u << 22);
        const uint32_t bpcs[] = {512, 1024, 4096, 100};
        const uint32_t bpc = bpcs[rng() % 4];
        const uint32_t psize = (rng() % 2) ? 65536u : uint32_t(bpc * (1 + rng() % 64));
        const uint64_t n = oracle_packetize(len, off, psize, bpc, nullptr, 0);
        std::vector<uint64_t> want(n);
        oracle_packetize(len, off, psize, bpc, want.data(), n);
        uint64_t *got = static_cast<uint64_t *>(std::malloc(8 * n));
        CHECK(crc32c_packetize(len, off, psize, bpc, got, n) == n, "packetize count");
        CHECK(std::memcmp(got, want.data(), 8 * n) == 0, "packetize len %llu off %llu", (unsigned long long)len,
              (unsigned long long)off);
        // a short output array is never overrun
        const uint64_t cap = n / 2;
        uint64_t *part = static_cast<uint64_t *>(std::malloc(cap ? 8 * cap : 1));
        CHECK(crc32c_packetize(len, off, psize, bpc, part, cap) == n, "packetize short cap");
        std::free(part);
        std::free(got);
    }
}

std::vector<crc32c_packet> random_batch(std::mt19937_64 &rng, uint64_t *extent) {
    const uint32_t bpcs[] = {512, 1024, 2048, 4096, 8192, 100, 1536, 7};
    const size_t npkts = 1 + rng() % 64;
    std::vector<crc32c_packet> pk(npkts);
    uint64_t off = 0, out = 0;
    for (auto &p : pk) {
        off += rng() % 3 == 0 ? rng() % 97 : 0;  // some unaligned packets
        p.payload_off = off;
        p.len = uint32_t(rng() % 4 == 0 ? rng() % 3000 : 65536 - (rng() % 2) * (rng() % 700));
        p.bpc = bpcs[rng() % 8];
        p.out_idx = out;
        out += crc32c_nchunks(p.len, p.bpc);
        off += p.len;
    }
    *extent = off;
    return pk;
}

void plans_and_framing(std::mt19937_64 &rng) {
    for (int it = 0; it < 300; ++it) {
        uint64_t extent = 0;
        const std::vector<crc32c_packet> pk = random_batch(rng, &extent);
        uint64_t nt = 0, ng = 0;
        CHECK(crc32c_debug_plan(pk.data(), pk.size(), nullptr, 0, nullptr, 0, &nt, &ng) == 0, "plan rc");
        auto *tiles = static_cast<hdfs_crc::FastTile *>(std::malloc(nt ? 16 * nt : 1));
        auto *gen = static_cast<hdfs_crc::GenItem *>(std::malloc(ng ? 16 * ng : 1));
        CHECK(crc32c_debug_plan(pk.data(), pk.size(), tiles, nt, gen, ng, &nt, &ng) == 0, "plan rc 2");
        // every chunk is covered exactly once by a tile or a general item
        const uint64_t nsums = crc32c_batch_nchecksums(pk.data(), pk.size());
        std::vector<int> seen(nsums, 0);
        for (uint64_t i = 0; i < nt; ++i) {
            const uint32_t meta = tiles[i].meta;
            const uint64_t src = tiles[i].src & hdfs_crc::kSrcMask;
            const uint32_t tl = uint32_t(tiles[i].src >> 48), kt = (tl + 511u) / 512u;
            uint32_t nch, bpc;
            if ((meta & 0xC0000000u) == hdfs_crc::kHalfTile) {  // half tile: n chunks of 512 M + r bytes
                const uint32_t m = (meta >> 8) & 0xffu, padh = (meta >> 18) & 511u;
                nch = meta & 0xffu;
                bpc = 512u * m + 256u - padh;
                CHECK(m <= 2 && nch >= 1 && nch <= (m == 0 ? 32u : m == 1 ? 10u : 6u) && padh < 256 && tl == 0 &&
                          bpc >= 4,
                      "half tile meta %x", meta);
                CHECK(padh == 0 || src >= 16, "half tile too close to the payload start");
            } else if (meta & hdfs_crc::kGeneralTile) {
                const uint32_t k = (meta >> 8) & 31u, pad = (meta >> 18) & 511u;
                nch = (meta >> 13) & 31u;
                bpc = k * 512u - pad;
                CHECK(nch >= 1 && nch <= 16 && (meta & 0xffu) == (nch * k + kt + 15) / 16 && bpc >= 4,
                      "general tile meta %x", meta);
                CHECK(pad == 0 || src >= 16, "padded tile too close to the payload start");
                CHECK(tl == 0 || (tl >= 4 && tl < bpc), "tail chunk length %u", tl);
            } else {
                // (bits 18-26: the pad of a padded power-of-two tile, bpc = (512 << lg) - pad)
                const uint32_t nb = meta & 0xffu, lg = (meta >> 8) & 0xffu, pad = (meta >> 18) & 511u;
                CHECK(nb >= 1 && nb <= 16 && lg <= 4 && (nb % (1u << lg)) == 0 && tl == 0, "tile meta %x", meta);
                CHECK((meta & ~(0xffffu | (511u << 18))) == 0, "tile meta %x", meta);
                nch = nb >> lg;
                bpc = (512u << lg) - pad;
                CHECK(bpc >= 4 && (pad == 0 || src >= 16), "padded tile meta %x src %llu", meta,
                      (unsigned long long)src);
            }
            CHECK(src + uint64_t(bpc) * nch + tl <= extent, "tile past the payload");
            for (uint32_t c = 0; c < nch + (tl ? 1u : 0u); ++c)
                if (tiles[i].out + c < nsums) seen[tiles[i].out + c]++;
        }
        for (uint64_t i = 0; i < ng; ++i) {
            CHECK(gen[i].len >= 1 && gen[i].src + gen[i].len <= extent, "gen item range");
            if (gen[i].out < nsums) seen[gen[i].out]++;
        }
        for (uint64_t i = 0; i < nsums; ++i) CHECK(seen[i] == 1, "chunk %llu covered %d times", (unsigned long long)i, seen[i]);
        std::free(tiles);
        std::free(gen);

        // framing into exactly the size it asks for
        std::vector<uint32_t> sums(nsums ? nsums : 1);
        for (auto &s : sums) s = uint32_t(rng());
        const uint32_t flags = uint32_t(rng() % 2);
        const uint32_t cl = (rng() % 4 == 0) ? 0u : 4u;
        const size_t need = crc32c_frame_packets(pk.data(), pk.size(), sums.data(), flags, rng() % 4096, 0, cl,
                                                 nullptr, 0, nullptr);
        CHECK(need > 0, "frame size");
        uint8_t *fr = static_cast<uint8_t *>(std::malloc(need));
        uint64_t *po = static_cast<uint64_t *>(std::malloc(8 * (pk.size() + 1)));
        CHECK(crc32c_frame_packets(pk.data(), pk.size(), sums.data(), flags, 0, 0, cl, fr, need, po) == need,
              "frame bytes");
        CHECK(po[0] == 0 && po[pk.size()] == need, "prefix offsets");
        for (size_t i = 0; i < pk.size(); ++i) {
            CHECK(po[i + 1] > po[i], "prefix offsets increase");
            const uint32_t plen = (uint32_t(fr[po[i]]) << 24) | (uint32_t(fr[po[i] + 1]) << 16) |
                                  (uint32_t(fr[po[i] + 2]) << 8) | fr[po[i] + 3];
            const uint64_t n = cl ? crc32c_nchunks(pk[i].len, pk[i].bpc) : 0;
            CHECK(plen == 4 + cl * n + pk[i].len, "PLEN of packet %zu", i);  // hadooprpc.c:640
        }
        CHECK(crc32c_frame_packets(pk.data(), pk.size(), sums.data(), flags, 0, 0, cl, fr, need - 1, po) == need,
              "short cap writes nothing, returns the size");
        std::free(po);
        std::free(fr);

        uint8_t md5[16];
        uint32_t *s = static_cast<uint32_t *>(std::malloc(4 * (nsums ? nsums : 1)));
        std::memcpy(s, sums.data(), 4 * nsums);
        crc32c_block_md5(s, nsums, flags, md5);
        std::free(s);
    }
}

// crc(0, chunk) of one HostPlan item evaluated on the CPU from its
// descriptor alone (addresses absolute: host pointers of the test).
uint32_t crc_at(uint64_t addr, uint32_t len) {
    return oracle_crc32c_bytewise(0, reinterpret_cast<const void *>(uintptr_t(addr)), len);
}

// Packet assembly (build_write_plan) over random buffer lists of exactly
// sized heap blocks (NULL = zero fill): every item is evaluated from its
// descriptor and compared with the oracle over the assembled stream, cut
// into packets and chunks as hadooprpc.c:815-860 / 733-742 do.
void write_plans(std::mt19937_64 &rng) {
    for (int it = 0; it < 300; ++it) {
        const uint32_t nb = 1 + uint32_t(rng() % 5);
        std::vector<crc32c_buffer> bufs(nb);
        std::vector<uint8_t *> owned;
        std::vector<uint8_t> stream;
        for (auto &b : bufs) {
            b.len = (rng() % 4 == 0) ? rng() % 50 : rng() % 90000;
            if (rng() % 3 == 0) {
                b.data = nullptr;
                stream.insert(stream.end(), size_t(b.len), 0);
            } else {
                uint8_t *p = exact_bytes(rng, size_t(b.len));
                owned.push_back(p);
                b.data = p;
                stream.insert(stream.end(), p, p + b.len);
            }
        }
        const uint64_t total = stream.size();
        const uint64_t boff = total ? rng() % (total + 1) : 0;
        const uint64_t len = total - boff ? rng() % (total - boff + 1) : 0;
        const uint32_t bpcs[] = {512, 1024, 4096, 100, 1536, 3};
        const uint32_t bpc = bpcs[rng() % 6];
        const uint64_t blockoffset = rng() % 3 ? 0 : rng() % 100000;
        const uint32_t psize = rng() % 2 ? 65536u : bpc * uint32_t(1 + rng() % 8);
        hdfs_crc::HostPlan hp;
        CHECK(hdfs_crc::build_write_plan(bufs.data(), nb, boff, len, blockoffset, psize, bpc, hdfs_crc::kPoly, &hp) == 0,
              "write plan rc");
        // expected: the assembled bytes, packetized and chunked
        std::vector<uint32_t> want;
        const uint64_t np = crc32c_packetize(len, blockoffset, psize, bpc, nullptr, 0);
        std::vector<uint64_t> lens(np);
        crc32c_packetize(len, blockoffset, psize, bpc, lens.data(), np);
        uint64_t pos = boff;
        for (uint64_t pl : lens) {
            for (uint64_t c = 0; c * bpc < pl; ++c) {
                const uint32_t cl = uint32_t(std::min<uint64_t>(bpc, pl - c * bpc));
                want.push_back(oracle_crc32c_bytewise(0, stream.data() + pos + c * bpc, cl));
            }
            pos += pl;
        }
        CHECK(hp.nchecksums == want.size(), "write plan checksums %llu vs %zu", (unsigned long long)hp.nchecksums,
              want.size());
        std::vector<uint32_t> got(want.size(), 0xdeadbeefu);
        std::vector<int> seen(want.size(), 0);
        auto put = [&](uint64_t i, uint32_t v) {
            if (i < got.size()) {
                got[i] = v;
                seen[i]++;
            }
        };
        for (const auto &t : hp.tiles) {
            uint32_t nch, tb;
            const uint64_t src = t.src & hdfs_crc::kSrcMask;
            const uint32_t tl = uint32_t(t.src >> 48);
            if ((t.meta & 0xC0000000u) == hdfs_crc::kHalfTile) {
                nch = t.meta & 0xffu;
                tb = 512u * ((t.meta >> 8) & 0xffu) + 256u - ((t.meta >> 18) & 511u);
                CHECK(((t.meta >> 18) & 511u) == 0 || (src & 4095u) >= 16, "half tile page rule");
            } else if (t.meta & hdfs_crc::kGeneralTile) {
                nch = (t.meta >> 13) & 31u;
                tb = ((t.meta >> 8) & 31u) * 512u - ((t.meta >> 18) & 511u);
                CHECK(((t.meta >> 18) & 511u) == 0 || (src & 4095u) >= 16, "padded tile page rule");
            } else {  // (padded power-of-two tiles: bpc = (512 << lg) - pad)
                nch = (t.meta & 0xffu) >> ((t.meta >> 8) & 0xffu);
                tb = (512u << ((t.meta >> 8) & 0xffu)) - ((t.meta >> 18) & 511u);
                CHECK(tl == 0, "tail on a power-of-two tile");
                CHECK(((t.meta >> 18) & 511u) == 0 || (src & 4095u) >= 16, "padded tile page rule");
            }
            for (uint32_t c = 0; c < nch; ++c) put(t.out + c, crc_at(src + uint64_t(c) * tb, tb));
            if (tl) put(t.out + nch, crc_at(src + uint64_t(nch) * tb, tl));
        }
        for (const auto &g : hp.gen) put(g.out, crc_at(g.src, g.len));
        for (const auto &sg : hp.seg) {
            std::vector<uint8_t> chunk(sg.len, 0);
            for (uint32_t u = 0; u < sg.npieces; ++u) {
                const auto &pc = hp.pieces[sg.first + u];
                CHECK(pc.start + uint64_t(pc.len) <= sg.len && pc.len >= 1, "piece range");
                std::memcpy(chunk.data() + pc.start, reinterpret_cast<const void *>(uintptr_t(pc.src)), pc.len);
            }
            put(sg.out, oracle_crc32c_bytewise(0, chunk.data(), sg.len));
        }
        for (const auto &cr : hp.consts)
            for (uint32_t k = 0; k < cr.count; ++k) put(cr.out + k, cr.value);
        for (size_t i = 0; i < want.size(); ++i) {
            CHECK(seen[i] == 1, "write chunk %zu covered %d times", i, seen[i]);
            CHECK(got[i] == want[i], "write chunk %zu: %08x vs %08x", i, got[i], want[i]);
        }
        for (uint8_t *p : owned) std::free(p);
    }
}

// Received frames (frames.cpp): frames built by crc32c_frame_packets with
// the data behind each prefix parse back to the same fields, into an
// exactly sized buffer; a truncated buffer yields only its whole frames.
void frames_parse(std::mt19937_64 &rng) {
    for (int it = 0; it < 200; ++it) {
        const size_t np = 1 + rng() % 20;
        std::vector<crc32c_packet> pk(np);
        uint64_t off = 0, out = 0;
        for (size_t i = 0; i < np; ++i) {
            pk[i].payload_off = off;
            pk[i].len = i + 1 == np ? 0 : uint32_t(rng() % 70000);
            pk[i].bpc = 512;
            pk[i].out_idx = out;
            out += crc32c_nchunks(pk[i].len, 512);
            off += pk[i].len;
        }
        std::vector<uint32_t> sums(out ? out : 1, 0x12345678u);
        const size_t need = crc32c_frame_packets(pk.data(), np, sums.data(), 0, 4096, 0, 4, nullptr, 0, nullptr);
        std::vector<uint8_t> prefix(need);
        std::vector<uint64_t> po(np + 1);
        crc32c_frame_packets(pk.data(), np, sums.data(), 0, 4096, 0, 4, prefix.data(), need, po.data());
        const size_t total = need + off;
        uint8_t *buf = static_cast<uint8_t *>(std::malloc(total));
        size_t w = 0;
        for (size_t i = 0; i < np; ++i) {
            std::memcpy(buf + w, prefix.data() + po[i], po[i + 1] - po[i]);
            w += po[i + 1] - po[i];
            std::memset(buf + w, int(i), pk[i].len);
            w += pk[i].len;
        }
        std::vector<crc32c_frame_info> info(np);
        uint64_t used = 0;
        CHECK(crc32c_parse_frames(buf, total, info.data(), np, &used) == int64_t(np) && used == total, "parse all");
        for (size_t i = 0; i < np; ++i) {
            CHECK(info[i].data_len == pk[i].len && info[i].offset_in_block == int64_t(4096 + pk[i].payload_off) &&
                      info[i].seqno == int64_t(i) && info[i].last == (i + 1 == np) &&
                      info[i].nsums == crc32c_nchunks(pk[i].len, 512),
                  "frame %zu fields", i);
        }
        const size_t cut = rng() % total;
        uint8_t *part = static_cast<uint8_t *>(std::malloc(cut ? cut : 1));
        std::memcpy(part, buf, cut);
        const int64_t k = crc32c_parse_frames(part, cut, info.data(), np, &used);
        CHECK(k >= 0 && k < int64_t(np) && used <= cut, "partial parse");
        std::free(part);
        std::free(buf);
    }
}

void table_images() {
    const size_t n4 = crc32c_debug_lds_image_s4(nullptr, 0, 0);
    for (uint32_t flags : {0u, uint32_t(CRC32C_TYPE_CRC32)}) {
        uint8_t *img = static_cast<uint8_t *>(std::malloc(n4));
        CHECK(crc32c_debug_lds_image_s4(img, n4, flags) == n4, "s4 image size");
        std::free(img);
    }
    uint32_t clg[5], csm[4];
    const size_t n = crc32c_debug_lds_image(nullptr, 0, nullptr, nullptr);
    uint8_t *img = static_cast<uint8_t *>(std::malloc(n));
    CHECK(crc32c_debug_lds_image(img, n, clg, csm) == n, "nibble image size");
    std::free(img);
}

// shift_zeros (register * x^(8 n) mod P, what plan building uses for
// zero-fill constants) equals the 32x32 operator op_zeros(n) for both
// polynomials: every n below 1100, powers of two and random n up to 2^40.
void zero_shifts(std::mt19937_64 &rng) {
    for (uint32_t poly : {hdfs_crc::kPoly, hdfs_crc::kPolyIeee}) {
        std::vector<uint64_t> ns;
        for (uint64_t n = 0; n < 1100; ++n) ns.push_back(n);
        for (int k = 0; k < 41; ++k) ns.push_back(uint64_t(1) << k);
        for (int i = 0; i < 60; ++i) ns.push_back(rng() % (uint64_t(1) << 40));
        for (uint64_t n : ns) {
            const uint32_t r = uint32_t(rng());
            const hdfs_crc::Gf2Op op = hdfs_crc::op_zeros(n, poly);
            CHECK(hdfs_crc::shift_zeros(r, n, poly) == op.apply(r), "shift_zeros(%08x, %llu) poly %08x", r,
                  (unsigned long long)n, poly);
            CHECK(hdfs_crc::shift_zeros(0xffffffffu, n, poly) == op.apply(0xffffffffu), "shift_zeros(~0, %llu)",
                  (unsigned long long)n);
        }
    }
}

}  // namespace

int main() {
    std::mt19937_64 rng(0x9E3779B97F4A7C15ull);
    scalar_and_chunks(rng);
    packetize(rng);
    plans_and_framing(rng);
    write_plans(rng);
    frames_parse(rng);
    table_images();
    zero_shifts(rng);
    if (g_fail) {
        std::fprintf(stderr, "%d failures\n", g_fail);
        return 1;
    }
    std::printf("host sanitizer run clean\n");
    return 0;
}
