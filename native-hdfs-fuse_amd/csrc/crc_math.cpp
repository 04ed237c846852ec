// crc_math.cpp -- see crc_math.h.
#include "crc_math.h"

#include <cstring>
#include <mutex>
#include <vector>

namespace hdfs_crc {

namespace {
struct PolyTable {
    uint32_t t[256];
    std::once_flag once;
};
PolyTable g_tab[2];  // kPoly, kPolyIeee

void init_t0(uint32_t poly, uint32_t *t) {
    // Eight reflected shift/xor steps per byte value (crc32c.c:54-65).
    for (uint32_t b = 0; b < 256; ++b) {
        uint32_t r = b;
        for (int i = 0; i < 8; ++i) r = (r >> 1) ^ (poly & (0u - (r & 1u)));
        t[b] = r;
    }
}
}  // namespace

const uint32_t *byte_table(uint32_t poly) {
    PolyTable &pt = g_tab[poly == kPolyIeee ? 1 : 0];
    std::call_once(pt.once, [&] { init_t0(poly == kPolyIeee ? kPolyIeee : kPoly, pt.t); });
    return pt.t;
}

uint32_t append_zero_byte(uint32_t reg, uint32_t poly) {
    const uint32_t *t = byte_table(poly);
    return (reg >> 8) ^ t[reg & 0xffu];
}

Gf2Op op_identity() {
    Gf2Op o;
    for (int j = 0; j < 32; ++j) o.col[j] = 1u << j;
    return o;
}

Gf2Op op_compose(const Gf2Op &a, const Gf2Op &b) {
    Gf2Op o;
    for (int j = 0; j < 32; ++j) o.col[j] = a.apply(b.col[j]);
    return o;
}

Gf2Op op_zeros(uint64_t nbytes, uint32_t poly) {
    // Square-and-multiply on the one-zero-byte operator.
    Gf2Op step, acc = op_identity();
    for (int j = 0; j < 32; ++j) step.col[j] = append_zero_byte(1u << j, poly);
    while (nbytes) {
        if (nbytes & 1u) acc = op_compose(step, acc);
        step = op_compose(step, step);
        nbytes >>= 1;
    }
    return acc;
}

namespace {
// a * b mod P in the register's reflected representation (bit 31 = x^0).
uint32_t mulmod(uint32_t a, uint32_t b, uint32_t poly) {
    uint32_t p = 0;
    for (uint32_t m = 1u << 31; m; m >>= 1) {
        if (a & m) p ^= b;
        b = (b & 1u) ? (b >> 1) ^ poly : b >> 1;
    }
    return p;
}
struct PowTable {  // x^(2^k) mod P, k = 0..63
    uint32_t t[64];
    explicit PowTable(uint32_t poly) {
        t[0] = 1u << 30;  // x^1
        for (int k = 1; k < 64; ++k) t[k] = mulmod(t[k - 1], t[k - 1], poly);
    }
};
}  // namespace

uint32_t shift_zeros(uint32_t reg, uint64_t nbytes, uint32_t poly) {
    static const PowTable c(kPoly), ieee(kPolyIeee);
    const PowTable &pt = poly == kPolyIeee ? ieee : c;
    // x^(8 n) = product of x^(2^k) over the set bits k of 8 n
    uint32_t x = 1u << 31;  // x^0
    for (int k = 3; nbytes && k < 64; ++k, nbytes >>= 1)
        if (nbytes & 1u) x = mulmod(pt.t[k], x, poly);
    return mulmod(x, reg, poly);
}

uint32_t lin_bytes(const uint8_t *p, size_t n, uint32_t reg, uint32_t poly) {
    const uint32_t *t = byte_table(poly);
    for (size_t i = 0; i < n; ++i) reg = (reg >> 8) ^ t[(reg ^ p[i]) & 0xffu];
    return reg;
}

void build_lds_image(uint8_t *dst, uint32_t poly) {
    std::memset(dst, 0, kLdsBytes);
    const uint32_t *t0 = byte_table(poly);
    // vals[x] = lin(x followed by d zero bytes) for the 32 nibble-basis bytes
    // (x = n for low nibbles, x = n << 4 for high nibbles), walked from d = 0
    // up to d = 511.  The byte at block offset o is followed by d = 511 - o.
    uint32_t lo[16], hi[16];
    for (int n = 0; n < 16; ++n) {
        lo[n] = t0[n];
        hi[n] = t0[n << 4];
    }
    auto put = [&](size_t off, uint32_t v) { std::memcpy(dst + off, &v, 4); };
    for (int d = 0; d < 512; ++d) {
        const int o = 511 - d;       // block offset of the byte
        const int q = o >> 4;        // lane column
        const int k = o & 15;        // byte within the lane's 16-byte piece
        for (int n = 0; n < 16; ++n) {
            put(size_t(k) * 4096 + size_t(n) * 256 + size_t(q) * 4, lo[n]);
            put(128 + size_t(k) * 256 + size_t(n) * 4096 + size_t(q) * 4, hi[n]);
        }
        for (int n = 0; n < 16; ++n) {
            lo[n] = append_zero_byte(lo[n], poly);
            hi[n] = append_zero_byte(hi[n], poly);
        }
    }
    const Gf2Op z512 = op_zeros(512, poly);
    Gf2Op zs = z512;
    for (int s = 1; s <= kMaxShift; ++s) {
        for (int tn = 0; tn < 8; ++tn)
            for (uint32_t n = 0; n < 16; ++n)
                put(kLdsShiftOff + size_t(s - 1) * 512 + size_t(tn) * 64 + n * 4, zs.apply(n << (4 * tn)));
        zs = op_compose(z512, zs);
    }
}

uint32_t s4_step(uint32_t u, uint32_t poly) {
    uint32_t r = u;
    for (int i = 0; i < 4; ++i) r = append_zero_byte(r, poly);
    return r;
}

void build_lds_image_s4(uint8_t *dst, uint32_t poly) {
    std::memset(dst, 0, kS4Bytes);
    auto put = [&](size_t off, uint32_t v) { std::memcpy(dst + off, &v, 4); };
    // T_m[b]: byte b followed by m zero bytes, from register 0.
    const uint32_t *t0 = byte_table(poly);
    for (uint32_t b = 0; b < 256; ++b) {
        uint32_t v = t0[b];
        for (int m = 0; m < 4; ++m) {
            for (int q = 0; q < 32; ++q) put(size_t(m >> 1) * 65536 + size_t(b) * 256 + size_t(m & 1) * 128 + q * 4, v);
            v = append_zero_byte(v, poly);
        }
    }
    // N_q(n << 4t) = Z_{16 (31 - q)}(S(n << 4t)).
    for (int q = 0; q < 32; ++q) {
        const Gf2Op zq = op_zeros(uint64_t(16) * uint64_t(31 - q), poly);
        for (int t = 0; t < 8; ++t)
            for (uint32_t n = 0; n < 16; ++n)
                put(kS4NibOff + size_t(t >> 1) * 4096 + n * 256 + size_t(t & 1) * 128 + q * 4,
                    zq.apply(s4_step(n << (4 * t), poly)));
    }
    // Z^(512 s), as in the nibble image.
    std::vector<uint8_t> nib(kLdsBytes);
    build_lds_image(nib.data(), poly);
    std::memcpy(dst + kS4ShiftOff, nib.data() + kLdsShiftOff, kMaxShift * 512);
}

void compact_s4_image(const uint8_t *full, uint8_t *dst) {
    std::memset(dst, 0, kS4CBytes);
    for (uint32_t m = 0; m < 4; ++m)
        for (uint32_t b = 0; b < 256; ++b)  // column 0 of T_m
            std::memcpy(dst + m * 1024u + 4u * b, full + (m >> 1) * 65536u + b * 256u + (m & 1u) * 128u, 4);
    std::memcpy(dst + kS4CNibOff, full + kS4NibOff, kS4Bytes - kS4NibOff);
}

void affine_constants(uint32_t c_lg[5], uint32_t c_small[4], uint32_t poly) {
    // crc(0, zeros(n)) = Z^n(0xffffffff) ^ 0xffffffff (crc32c.c:237, 312).
    for (int lg = 0; lg < 5; ++lg) c_lg[lg] = op_zeros(512ull << lg, poly).apply(0xffffffffu) ^ 0xffffffffu;
    for (int r = 0; r < 4; ++r) c_small[r] = op_zeros(r, poly).apply(0xffffffffu) ^ 0xffffffffu;
}

void zero_crc_table(uint32_t *dst, uint32_t poly) {
    // register ~0 (crc32c.c:237) through n zero bytes, ^ ~0 (crc32c.c:312)
    uint32_t reg = 0xffffffffu;
    for (uint32_t n = 0; n <= kZeroCrcMax; ++n) {
        dst[n] = reg ^ 0xffffffffu;
        reg = append_zero_byte(reg, poly);
    }
}

}  // namespace hdfs_crc
