// gf2.h -- GF(2)[x]/P arithmetic shared by the host side of the C ABI and the
// CDNA4 kernels.
//
// Conventions (the folly/zlib reflected CRC register):
//   * a 32-bit register r represents the polynomial sum_i r[31-i] x^i, so
//     x^0 == 0x80000000 and multiplying by x is a right shift with a
//     conditional xor of the reflected polynomial;
//   * raw(data, s)  = folly::crc32c(data, n, s): the register after feeding the
//     bytes from state s, no final xor (src/fbs/storage/Common.h:158);
//   * raw(A||B, s)  = raw(A, s) * x^(8|B|)  ^  lin(B), lin(B) = raw(B, 0);
//   * folly::crc32c_combine(c1, c2, n) = c1 * x^(8n) ^ c2 (Common.h:191).
// Everything here is integer arithmetic; there is no floating point anywhere
// on this path.
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define GF2_HD __host__ __device__
#else
#define GF2_HD
#endif

namespace hf3fs_crc {

constexpr uint32_t kPolyCrc32c = 0x82F63B78u;  // Castagnoli, reflected
constexpr uint32_t kPolyCrc32 = 0xEDB88320u;   // IEEE 802.3, reflected
constexpr uint32_t kOne = 0x80000000u;         // x^0

// Wire enum ChecksumType (Common.h:66-70).
constexpr uint8_t kTypeNone = 0, kTypeCrc32c = 1, kTypeCrc32 = 2;

// a * b mod P.  Branch-free, fixed 32 rounds: identical cost on every lane.
GF2_HD constexpr inline uint32_t gf_mul(uint32_t a, uint32_t b, uint32_t poly) {
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    p ^= b & (0u - (a >> 31));  // coefficient of x^i in a (bit 31 - i)
    a <<= 1;
    b = (b >> 1) ^ (poly & (0u - (b & 1u)));  // b *= x
  }
  return p;
}

// Carry-less 32 x 32 -> 64 product from 16 integer multiplies: the operand bits are split
// into their four residue classes mod 4, so one product's terms at a bit of its class number
// at most 8 and their carries stop short of the next bit of that class (masked off below).
GF2_HD inline uint64_t clmul32(uint32_t x, uint32_t y) {
  const uint32_t m0 = 0x11111111u, m1 = 0x22222222u, m2 = 0x44444444u, m3 = 0x88888888u;
  const uint32_t x0 = x & m0, x1 = x & m1, x2 = x & m2, x3 = x & m3;
  const uint32_t y0 = y & m0, y1 = y & m1, y2 = y & m2, y3 = y & m3;
  const uint64_t z0 = (uint64_t)x0 * y0 ^ (uint64_t)x1 * y3 ^ (uint64_t)x2 * y2 ^ (uint64_t)x3 * y1;
  const uint64_t z1 = (uint64_t)x0 * y1 ^ (uint64_t)x1 * y0 ^ (uint64_t)x2 * y3 ^ (uint64_t)x3 * y2;
  const uint64_t z2 = (uint64_t)x0 * y2 ^ (uint64_t)x1 * y1 ^ (uint64_t)x2 * y0 ^ (uint64_t)x3 * y3;
  const uint64_t z3 = (uint64_t)x0 * y3 ^ (uint64_t)x1 * y2 ^ (uint64_t)x2 * y1 ^ (uint64_t)x3 * y0;
  return (z0 & 0x1111111111111111ull) | (z1 & 0x2222222222222222ull) | (z2 & 0x4444444444444444ull) |
         (z3 & 0x8888888888888888ull);
}

// a * b mod P (reflected) as gf_mul, from clmul32: shifted left by one, the product's high
// word holds degrees 0..31 and its low word (reflected) * x^32, which one pass through the
// dword slicing tables dw[256 k + b] = (b << 8k) * x^32 (ShortTables::dw) reduces.
// ~62 VALU (16 of them v_mad_u64_u32) + 4 table reads against gf_mul's ~215 VALU: 2.07x the
// throughput on gfx950 with the tables in LDS (scripts/probe_gfmul.hip).
GF2_HD inline uint32_t gf_mul_dw(uint32_t a, uint32_t b, const uint32_t* dw) {
  const uint64_t z = clmul32(a, b) << 1;
  const uint32_t h = (uint32_t)(z >> 32), l = (uint32_t)z;
  return h ^ dw[l & 0xffu] ^ dw[256 + ((l >> 8) & 0xffu)] ^ dw[512 + ((l >> 16) & 0xffu)] ^ dw[768 + (l >> 24)];
}

// x^n mod P for a non-negative bit count n (compile-time friendly).
GF2_HD constexpr inline uint32_t xpow_bits(uint64_t n, uint32_t poly) {
  uint32_t result = kOne, base = kOne >> 1;  // base = x
  while (n) {
    if (n & 1) result = gf_mul(result, base, poly);
    base = gf_mul(base, base, poly);
    n >>= 1;
  }
  return result;
}

// x^-1 mod P: x * (x^31 + sum_{i>=1} p_i x^(i-1)) = P - 1 == 1.
GF2_HD constexpr inline uint32_t x_inverse(uint32_t poly) { return (poly << 1) | 1u; }

GF2_HD constexpr inline uint32_t xpow_neg_bits(uint64_t n, uint32_t poly) {
  uint32_t result = kOne, base = x_inverse(poly);
  while (n) {
    if (n & 1) result = gf_mul(result, base, poly);
    base = gf_mul(base, base, poly);
    n >>= 1;
  }
  return result;
}

// x^e for a signed bit count.
GF2_HD constexpr inline uint32_t xpow_signed_bits(int64_t e, uint32_t poly) {
  return e >= 0 ? xpow_bits((uint64_t)e, poly) : xpow_neg_bits((uint64_t)(-e), poly);
}

// x^(8 nbytes) mod P for any 64-bit byte count (the bit count 8 nbytes may not fit 64 bits).
GF2_HD constexpr inline uint32_t xpow_bytes(uint64_t nbytes, uint32_t poly) {
  uint32_t result = kOne, base = xpow_bits(8, poly);  // base = x^8
  while (nbytes) {
    if (nbytes & 1) result = gf_mul(result, base, poly);
    base = gf_mul(base, base, poly);
    nbytes >>= 1;
  }
  return result;
}

// crc fed `nbytes` zero bytes.
GF2_HD constexpr inline uint32_t shift_bytes(uint32_t crc, uint64_t nbytes, uint32_t poly) {
  return gf_mul(crc, xpow_bytes(nbytes, poly), poly);
}

// folly::crc32c_combine / crc32_combine and Rust crc32c::crc32c_combine (the
// finalized form obeys the same algebra).
GF2_HD constexpr inline uint32_t combine_raw(uint32_t c1, uint32_t c2, uint64_t len2, uint32_t poly) {
  return shift_bytes(c1, len2, poly) ^ c2;
}

GF2_HD constexpr inline uint32_t poly_of(uint8_t type) { return type == kTypeCrc32 ? kPolyCrc32 : kPolyCrc32c; }

static_assert(gf_mul(kOne, 0x12345678u, kPolyCrc32c) == 0x12345678u, "x^0 is the identity");
static_assert(gf_mul(kOne >> 1, x_inverse(kPolyCrc32c), kPolyCrc32c) == kOne, "x * x^-1 == 1");
static_assert(gf_mul(kOne >> 1, x_inverse(kPolyCrc32), kPolyCrc32) == kOne, "x * x^-1 == 1");

}  // namespace hf3fs_crc
