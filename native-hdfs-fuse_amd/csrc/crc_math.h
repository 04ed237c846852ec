// crc_math.h -- host-side GF(2) machinery for CRC32C (Castagnoli, reflected).
//
// Everything the GPU needs that is data rather than code is derived here once
// per process: the byte table, "append n zero bytes" operators, the LDS image
// of positional nibble tables and zero-shift operators, and the affine
// constants.  Reference semantics followed: src/crc32c.c:43 (polynomial),
// 50-73 (byte table), 84/106 (pre/post inversion), 137-200 (zero operators
// used to combine CRCs of concatenated pieces).
#pragma once
#include <cstddef>
#include <cstdint>

namespace hdfs_crc {

constexpr uint32_t kPoly = 0x82f63b78u;      // CRC32C, Castagnoli (crc32c.c:43)
constexpr uint32_t kPolyIeee = 0xedb88320u;  // CRC32, IEEE 802.3 / zlib (Hadoop's CHECKSUM_CRC32)
// Both are reflected CRCs with init ~0 and final ~0; everything below takes
// the polynomial as a parameter (only these two are supported).

// 32x32 GF(2) matrix stored as the images of the 32 unit vectors.
struct Gf2Op {
    uint32_t col[32];
    uint32_t apply(uint32_t v) const {
        uint32_t r = 0;
        for (int j = 0; v; ++j, v >>= 1)
            if (v & 1u) r ^= col[j];
        return r;
    }
};

const uint32_t *byte_table(uint32_t poly = kPoly);            // T0[b]: register after byte b from register 0
uint32_t append_zero_byte(uint32_t reg, uint32_t poly = kPoly);  // linear register, one zero byte appended
Gf2Op op_identity();
Gf2Op op_compose(const Gf2Op &a, const Gf2Op &b);           // a after b
Gf2Op op_zeros(uint64_t nbytes, uint32_t poly = kPoly);      // append nbytes zero bytes
// The register after nbytes zero bytes, as op_zeros(nbytes).apply(reg) but
// in O(log nbytes) 32-step products (reg * x^(8 nbytes) mod P) instead of
// 32x32 operator compositions: what plan building uses per zero-fill chunk.
uint32_t shift_zeros(uint32_t reg, uint64_t nbytes, uint32_t poly = kPoly);

// Linear part of the CRC over bytes with register starting at 0 (no
// conditioning): crc(0, M) == lin(M) ^ crc(0, zeros(len)).
uint32_t lin_bytes(const uint8_t *p, size_t n, uint32_t reg = 0, uint32_t poly = kPoly);

// ---- the GPU's LDS image (see DESIGN.md "LDS layout") ----
// [0, 65536): positional nibble tables of one 512-byte block.  Lane column q
//   (0..31) owns the 16 bytes at block offset 16q .. 16q+15; byte k of that
//   piece, nibble value n:
//     low nibble  at  k*4096 + n*256  + q*4          (address bit 7 = 0)
//     high nibble at  128 + k*256 + n*4096 + q*4     (address bit 7 = 1)
//   entry = lin(byte followed by 511 - (16q + k) zero bytes).
// [65536, 65536 + 15*512): Z^(512*s), s = 1..15, as 8 nibble tables of 16
//   entries: (s-1)*512 + t*64 + n*4 holds Z^(512 s)(n << 4t).
constexpr size_t kLdsPosBytes = 65536;
constexpr size_t kLdsShiftOff = 65536;
constexpr int kMaxShift = 15;
constexpr size_t kLdsBytes = kLdsPosBytes + kMaxShift * 512;

// Fills `dst` (kLdsBytes) with the LDS image.
void build_lds_image(uint8_t *dst, uint32_t poly = kPoly);

// ---- the slicing-by-4 kernel's LDS image (see DESIGN.md "S4 kernel") ----
// A lane chains its 16-byte piece d0..d3 through the position-independent
// slicing-by-4 step S (u = S(S(S(d0) ^ d1) ^ d2) ^ d3) and finishes with one
// column-specific operator N_q = Z_{16 (31 - q)} o S on u.
// [0, 131072): byte tables T_m[b] = register after byte b then m zero bytes
//   (m = 0..3, crc32c.c:50-73's crc32c_table[m]), each replicated over the 32
//   lane columns: T_m[b] at (m >> 1) * 65536 + b * 256 + (m & 1) * 128 + q * 4.
// [131072, 147456): N_q on nibble t of u, value n:
//   131072 + (t >> 1) * 4096 + n * 256 + (t & 1) * 128 + q * 4.
// [147456, 147456 + 15 * 512): Z^(512 s), s = 1..15, laid out as in the
//   nibble image's shift section.
constexpr size_t kS4NibOff = 131072;
constexpr size_t kS4ShiftOff = 147456;
constexpr size_t kS4Bytes = kS4ShiftOff + kMaxShift * 512;

// The compact S4 image (small batches): T0..T3 once each (T_m[b] at
// m * 1024 + 4 b), then the N_q section and the Z^(512 s) section laid out as
// in the full image.
constexpr size_t kS4CNibOff = 4096;
constexpr size_t kS4CShiftOff = kS4CNibOff + (kS4ShiftOff - kS4NibOff);
constexpr size_t kS4CBytes = kS4CShiftOff + kMaxShift * 512;
// Fills `dst` (kS4CBytes) from a full S4 image.
void compact_s4_image(const uint8_t *full, uint8_t *dst);

// Fills `dst` (kS4Bytes) with the slicing-by-4 LDS image.
void build_lds_image_s4(uint8_t *dst, uint32_t poly = kPoly);
// S(u): the register after feeding the 4 bytes of u (little-endian) into register 0.
uint32_t s4_step(uint32_t u, uint32_t poly = kPoly);

// crc(0, zeros(512 << lg)) for lg = 0..4 and crc(0, zeros(r)) for r = 0..3.
void affine_constants(uint32_t c_lg[5], uint32_t c_small[4], uint32_t poly = kPoly);

// crc(0, zeros(n)) for n = 0 .. kZeroCrcMax: the affine constant of a chunk
// of n bytes (crc(0, M) = lin(M) ^ crc(0, zeros(n))), which general items
// add per chunk instead of folding the pre-inversion into the data.
constexpr uint32_t kZeroCrcMax = 8192;
void zero_crc_table(uint32_t *dst, uint32_t poly = kPoly);  // kZeroCrcMax + 1 entries

}  // namespace hdfs_crc
