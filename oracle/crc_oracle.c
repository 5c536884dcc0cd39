/*
 * crc_oracle.c -- CPU restatement of the 3FS CRC32C/CRC32 chunk-integrity path.
 * TEST INFRASTRUCTURE ONLY (see crc_oracle.h for scope and citations).
 */
#include "crc_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* tables                                                                    */
/* ------------------------------------------------------------------------ */
static uint32_t T32C[8][256]; /* slicing-by-8, Castagnoli */
static uint32_t T32[8][256];  /* slicing-by-8, IEEE */
static uint32_t X2N_C[64];    /* x^(2^k) mod P, Castagnoli */
static uint32_t X2N_I[64];    /* x^(2^k) mod P, IEEE */
#define HW_LONG 8192
#define HW_SHORT 256
static uint32_t LONG_TBL[4][256];  /* multiply by x^(8*HW_LONG) */
static uint32_t SHORT_TBL[4][256]; /* multiply by x^(8*HW_SHORT) */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

uint32_t orc_gf2_mulmod(uint32_t a, uint32_t b, uint32_t poly) {
  /* reflected GF(2)[x]/P product; bit 31 holds x^0 (zlib multmodp form). */
  uint32_t m = 1u << 31, p = 0;
  if (a == 0 || b == 0) return 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ poly : b >> 1;
  }
  return p;
}

static void build_slicing(uint32_t t[8][256], uint32_t poly) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : c >> 1;
    t[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int k = 1; k < 8; ++k) t[k][i] = (t[k - 1][i] >> 8) ^ t[0][t[k - 1][i] & 0xff];
}

static void build_x2n(uint32_t *x2n, uint32_t poly) {
  x2n[0] = 1u << 30; /* x^1 */
  for (int k = 1; k < 64; ++k) x2n[k] = orc_gf2_mulmod(x2n[k - 1], x2n[k - 1], poly);
}

static uint32_t x8n_with(const uint32_t *x2n, uint64_t n, uint32_t poly) {
  uint32_t p = 1u << 31; /* x^0 */
  int k = 3;             /* x^(8n) = x^(n * 2^3) */
  while (n) {
    if (n & 1) {
      /* x^(2^k) for k >= 64 (n >= 2^61): squares of x^(2^63) -- the order of x mod P is not a
       * divisor of 2^64 - 1 (x^(2^31) == x for Castagnoli), so the table may not wrap */
      uint32_t f = x2n[k < 64 ? k : 63];
      for (int j = 63; j < k; ++j) f = orc_gf2_mulmod(f, f, poly);
      p = orc_gf2_mulmod(p, f, poly);
    }
    n >>= 1;
    ++k;
  }
  return p;
}

static void build_zeros_op(uint32_t t[4][256], uint64_t nbytes) {
  uint32_t x = x8n_with(X2N_C, nbytes, ORC_POLY_CRC32C);
  for (int k = 0; k < 4; ++k)
    for (uint32_t i = 0; i < 256; ++i) t[k][i] = orc_gf2_mulmod(i << (8 * k), x, ORC_POLY_CRC32C);
}

static void init_tables(void) {
  build_slicing(T32C, ORC_POLY_CRC32C);
  build_slicing(T32, ORC_POLY_CRC32);
  build_x2n(X2N_C, ORC_POLY_CRC32C);
  build_x2n(X2N_I, ORC_POLY_CRC32);
  build_zeros_op(LONG_TBL, HW_LONG);
  build_zeros_op(SHORT_TBL, HW_SHORT);
}
static inline void ensure_init(void) { pthread_once(&g_once, init_tables); }

uint32_t orc_x8n(uint64_t n, uint32_t poly) {
  ensure_init();
  return x8n_with(poly == ORC_POLY_CRC32 ? X2N_I : X2N_C, n, poly);
}

uint32_t orc_shift(uint32_t crc, uint64_t n, uint32_t poly) { return orc_gf2_mulmod(crc, orc_x8n(n, poly), poly); }

/* folly::crc32c_combine: crc of (A||B) from raw(A, s) and raw(B, 0) */
uint32_t orc_crc32c_combine(uint32_t c1, uint32_t c2, uint64_t len2) {
  return orc_shift(c1, len2, ORC_POLY_CRC32C) ^ c2;
}
uint32_t orc_crc32_combine(uint32_t c1, uint32_t c2, uint64_t len2) {
  return orc_shift(c1, len2, ORC_POLY_CRC32) ^ c2;
}

/* ------------------------------------------------------------------------ */
/* raw register updates                                                      */
/* ------------------------------------------------------------------------ */
uint32_t orc_crc_bitwise(uint32_t crc, const uint8_t *p, size_t n, uint32_t poly) {
  for (size_t i = 0; i < n; ++i) {
    crc ^= p[i];
    for (int k = 0; k < 8; ++k) crc = (crc & 1) ? (crc >> 1) ^ poly : crc >> 1;
  }
  return crc;
}

static uint32_t slicing8(const uint32_t t[8][256], uint32_t crc, const uint8_t *p, size_t n) {
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    w ^= crc;
    crc = t[7][w & 0xff] ^ t[6][(w >> 8) & 0xff] ^ t[5][(w >> 16) & 0xff] ^ t[4][(w >> 24) & 0xff] ^
          t[3][(w >> 32) & 0xff] ^ t[2][(w >> 40) & 0xff] ^ t[1][(w >> 48) & 0xff] ^ t[0][w >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) crc = (crc >> 8) ^ t[0][(crc ^ *p++) & 0xff];
  return crc;
}

uint32_t orc_crc32c_sw(uint32_t crc, const uint8_t *p, size_t n) {
  ensure_init();
  return slicing8(T32C, crc, p, n);
}
uint32_t orc_crc32_sw(uint32_t crc, const uint8_t *p, size_t n) {
  ensure_init();
  return slicing8(T32, crc, p, n);
}

int orc_have_sse42(void) {
#if defined(__x86_64__)
  return __builtin_cpu_supports("sse4.2");
#else
  return 0;
#endif
}

#if defined(__x86_64__)
#include <nmmintrin.h>
static inline uint32_t zeros_op(const uint32_t t[4][256], uint32_t c) {
  return t[0][c & 0xff] ^ t[1][(c >> 8) & 0xff] ^ t[2][(c >> 16) & 0xff] ^ t[3][c >> 24];
}
static inline uint64_t ld64(const uint8_t *p) {
  uint64_t w;
  memcpy(&w, p, 8);
  return w;
}
/* The SSE4.2 crc32 instruction stream with three interleaved streams whose
 * partial registers are merged by multiplication with x^(8*blk): the shape of
 * folly's hardware crc32c (the instruction is the reference's hot loop,
 * CMakeLists.txt:70-71 build it with -msse4.2). */
__attribute__((target("sse4.2"))) static uint32_t crc32c_sse42(uint32_t crc, const uint8_t *p, size_t n) {
  uint64_t c0 = crc;
  while (n && ((uintptr_t)p & 7)) {
    c0 = _mm_crc32_u8((uint32_t)c0, *p++);
    --n;
  }
  while (n >= 3 * HW_LONG) {
    uint64_t c1 = 0, c2 = 0;
    const uint8_t *end = p + HW_LONG;
    do {
      c0 = _mm_crc32_u64(c0, ld64(p));
      c1 = _mm_crc32_u64(c1, ld64(p + HW_LONG));
      c2 = _mm_crc32_u64(c2, ld64(p + 2 * HW_LONG));
      p += 8;
    } while (p < end);
    c0 = zeros_op(LONG_TBL, (uint32_t)c0) ^ (uint32_t)c1;
    c0 = zeros_op(LONG_TBL, (uint32_t)c0) ^ (uint32_t)c2;
    p += 2 * HW_LONG;
    n -= 3 * HW_LONG;
  }
  while (n >= 3 * HW_SHORT) {
    uint64_t c1 = 0, c2 = 0;
    const uint8_t *end = p + HW_SHORT;
    do {
      c0 = _mm_crc32_u64(c0, ld64(p));
      c1 = _mm_crc32_u64(c1, ld64(p + HW_SHORT));
      c2 = _mm_crc32_u64(c2, ld64(p + 2 * HW_SHORT));
      p += 8;
    } while (p < end);
    c0 = zeros_op(SHORT_TBL, (uint32_t)c0) ^ (uint32_t)c1;
    c0 = zeros_op(SHORT_TBL, (uint32_t)c0) ^ (uint32_t)c2;
    p += 2 * HW_SHORT;
    n -= 3 * HW_SHORT;
  }
  while (n >= 8) {
    c0 = _mm_crc32_u64(c0, ld64(p));
    p += 8;
    n -= 8;
  }
  while (n) {
    c0 = _mm_crc32_u8((uint32_t)c0, *p++);
    --n;
  }
  return (uint32_t)c0;
}
#endif

/* ------------------------------------------------------------------------ */
/* Carry-less-multiply folding (PCLMULQDQ / VPCLMULQDQ): the algorithm class  */
/* of folly's large-buffer crc32c dispatch on current x86 releases (its       */
/* folly/external/fast-crc32 kernels fold 128-bit lanes with clmul and mix in */
/* crc32 streams).  The folly commit the reference pins is unrecorded          */
/* (SURVEY.md 8c), so this leg is the CPU-speed bar, not a parity claim: its   */
/* output is checked against the SSE4.2 leg and the reference's known answers  */
/* (tests/test_oracle.py).                                                     */
/*                                                                             */
/* Algebra (reflected: register bit t <-> x^(31-t); a 16-byte little-endian    */
/* lane, bit k <-> x^(127-k) of the lane's polynomial).  A lane A = H x^64 + L */
/* (H = low qword, L = high qword) moved D bits towards the end is             */
/*   A x^D == clmul(H, K(64 + D)) ^ clmul(L, K(D)),  K(m) = (x^(m-1) mod P)<<32 */
/* (the clmul of two reflected operands carries one factor x, hence m - 1).    */
/* The folded 128-bit tail T finishes as crc32(crc32(0, T.lo), T.hi): the      */
/* crc32 instruction computes (message) x^32 mod P.  The start value is xor-ed */
/* into the first four bytes (raw(D, s) = lin(D ^ s||0...)).                   */
/* ------------------------------------------------------------------------ */
static uint32_t xbits_c(uint64_t m) { /* x^m mod P (Castagnoli), register form */
  uint32_t r = 1u << 31;
  for (int k = 0; m; ++k, m >>= 1)
    if (m & 1) r = orc_gf2_mulmod(r, X2N_C[k & 63], ORC_POLY_CRC32C);
  return r;
}
static inline uint64_t kfold(uint64_t m) { return (uint64_t)xbits_c(m - 1) << 32; }

int orc_have_clmul(void) {
#if defined(__x86_64__)
  return __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.2");
#else
  return 0;
#endif
}
int orc_have_vpclmul(void) {
#if defined(__x86_64__)
  return orc_have_clmul() && __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("vpclmulqdq");
#else
  return 0;
#endif
}

#if defined(__x86_64__)
#include <immintrin.h>
/* fold constants per lane distance (bytes), built once */
static uint64_t FOLD_K[17][2]; /* [j]: lane moved 16 j bytes: {K(64 + 128 j), K(128 j)}, j = 1..16 */
static uint64_t FOLD_K256[2], FOLD_K128[2];
static pthread_once_t g_fold_once = PTHREAD_ONCE_INIT;
static void init_fold(void) {
  ensure_init();
  for (int j = 1; j <= 16; ++j) {
    FOLD_K[j][0] = kfold(64 + 128 * (uint64_t)j);
    FOLD_K[j][1] = kfold(128 * (uint64_t)j);
  }
  FOLD_K256[0] = kfold(64 + 2048), FOLD_K256[1] = kfold(2048); /* 256 B: the zmm loop stride */
  FOLD_K128[0] = kfold(64 + 1024), FOLD_K128[1] = kfold(1024); /* 128 B: the xmm loop stride */
}

__attribute__((target("sse4.2,pclmul"))) static inline __m128i fold16(__m128i a, const uint64_t k[2]) {
  const __m128i K = _mm_set_epi64x((long long)k[1], (long long)k[0]);
  return _mm_xor_si128(_mm_clmulepi64_si128(a, K, 0x00), _mm_clmulepi64_si128(a, K, 0x11));
}

/* lanes[0..m) are consecutive 16-byte lanes ending at the same point: fold them into one */
__attribute__((target("sse4.2,pclmul"))) static __m128i fold_lanes(const __m128i *lanes, int m) {
  __m128i t = lanes[m - 1];
  for (int i = 0; i < m - 1; ++i) t = _mm_xor_si128(t, fold16(lanes[i], FOLD_K[m - 1 - i]));
  return t;
}

/* the folded head T, then the tail bytes (< 16 per lane step) through crc32 */
__attribute__((target("sse4.2,pclmul"))) static uint32_t finish(__m128i t, const uint8_t *p, size_t n) {
  while (n >= 16) {
    t = _mm_xor_si128(fold16(t, FOLD_K[1]), _mm_loadu_si128((const __m128i *)p));
    p += 16;
    n -= 16;
  }
  uint64_t c = _mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(t));
  c = _mm_crc32_u64(c, (uint64_t)_mm_extract_epi64(t, 1));
  while (n >= 8) {
    c = _mm_crc32_u64(c, ld64(p));
    p += 8;
    n -= 8;
  }
  while (n--) c = _mm_crc32_u8((uint32_t)c, *p++);
  return (uint32_t)c;
}

/* 8 xmm lanes, 128 bytes per step (PCLMULQDQ) */
__attribute__((target("sse4.2,pclmul"))) static uint32_t crc32c_pclmul(uint32_t crc, const uint8_t *p, size_t n) {
  if (n < 256) return crc32c_sse42(crc, p, n);
  pthread_once(&g_fold_once, init_fold);
  __m128i a[8];
  for (int i = 0; i < 8; ++i) a[i] = _mm_loadu_si128((const __m128i *)(p + 16 * i));
  a[0] = _mm_xor_si128(a[0], _mm_cvtsi32_si128((int)crc));
  p += 128;
  n -= 128;
  const __m128i K = _mm_set_epi64x((long long)FOLD_K128[1], (long long)FOLD_K128[0]);
  while (n >= 128) {
    for (int i = 0; i < 8; ++i)
      a[i] = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(a[i], K, 0x00), _mm_clmulepi64_si128(a[i], K, 0x11)),
                           _mm_loadu_si128((const __m128i *)(p + 16 * i)));
    p += 128;
    n -= 128;
  }
  return finish(fold_lanes(a, 8), p, n);
}

/* 4 zmm = 16 lanes, 256 bytes per step (AVX-512 VPCLMULQDQ) */
__attribute__((target("sse4.2,pclmul,avx512f,vpclmulqdq"))) static uint32_t crc32c_vpclmul(uint32_t crc,
                                                                                       const uint8_t *p, size_t n) {
  if (n < 512) return crc32c_pclmul(crc, p, n);
  pthread_once(&g_fold_once, init_fold);
  __m512i a0 = _mm512_loadu_si512(p), a1 = _mm512_loadu_si512(p + 64), a2 = _mm512_loadu_si512(p + 128),
          a3 = _mm512_loadu_si512(p + 192);
  a0 = _mm512_xor_si512(a0, _mm512_zextsi128_si512(_mm_cvtsi32_si128((int)crc)));
  p += 256;
  n -= 256;
  const __m512i K = _mm512_broadcast_i32x4(_mm_set_epi64x((long long)FOLD_K256[1], (long long)FOLD_K256[0]));
#define FOLD512(a, off)                                                                                       \
  a = _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(a, K, 0x00), _mm512_clmulepi64_epi128(a, K, 0x11),   \
                                _mm512_loadu_si512(p + (off)), 0x96)
  while (n >= 256) {
    FOLD512(a0, 0);
    FOLD512(a1, 64);
    FOLD512(a2, 128);
    FOLD512(a3, 192);
    p += 256;
    n -= 256;
  }
#undef FOLD512
  __m128i lanes[16];
  const __m512i acc[4] = {a0, a1, a2, a3};
  for (int k = 0; k < 4; ++k) {
    lanes[4 * k + 0] = _mm512_extracti32x4_epi32(acc[k], 0);
    lanes[4 * k + 1] = _mm512_extracti32x4_epi32(acc[k], 1);
    lanes[4 * k + 2] = _mm512_extracti32x4_epi32(acc[k], 2);
    lanes[4 * k + 3] = _mm512_extracti32x4_epi32(acc[k], 3);
  }
  return finish(fold_lanes(lanes, 16), p, n);
}
#endif

/* kind: 2 = best clmul form this CPU has (VPCLMULQDQ, else PCLMULQDQ, else SSE4.2) */
uint32_t orc_crc32c_clmul(uint32_t crc, const uint8_t *p, size_t n) {
  ensure_init();
#if defined(__x86_64__)
  if (orc_have_vpclmul()) return crc32c_vpclmul(crc, p, n);
  if (orc_have_clmul()) return crc32c_pclmul(crc, p, n);
#endif
  return orc_crc32c_hw(crc, p, n);
}
uint32_t orc_crc32c_pclmul128(uint32_t crc, const uint8_t *p, size_t n) {
  ensure_init();
#if defined(__x86_64__)
  if (orc_have_clmul()) return crc32c_pclmul(crc, p, n);
#endif
  return orc_crc32c_hw(crc, p, n);
}

uint32_t orc_crc32c_hw(uint32_t crc, const uint8_t *p, size_t n) {
  ensure_init();
#if defined(__x86_64__)
  if (orc_have_sse42()) return crc32c_sse42(crc, p, n);
#endif
  return slicing8(T32C, crc, p, n);
}

/* ------------------------------------------------------------------------ */
/* Rust crc32c 0.6.8: finalized convention                                  */
/* ------------------------------------------------------------------------ */
uint32_t orc_rs_crc32c(const uint8_t *p, size_t n) { return ~orc_crc32c_hw(~0u, p, n); }
uint32_t orc_rs_crc32c_append(uint32_t crc, const uint8_t *p, size_t n) { return ~orc_crc32c_hw(~crc, p, n); }
uint32_t orc_rs_crc32c_combine(uint32_t c1, uint32_t c2, size_t len2) {
  /* fin(A||B) = fin(A) * x^(8|B|) ^ fin(B): the same algebra as folly's. */
  return orc_shift(c1, len2, ORC_POLY_CRC32C) ^ c2;
}

/* ------------------------------------------------------------------------ */
/* ChecksumInfo (Common.h:113-202)                                           */
/* ------------------------------------------------------------------------ */
#define ORC_SLICE (1u << 20) /* ChecksumInfo::kChunkSize = 1_MB (Common.h:118) */

orc_checksum orc_checksum_create(uint8_t type, const uint8_t *p, size_t len, uint32_t start) {
  orc_checksum c = {type, start};
  if (type == ORC_NONE) {
    c.value = 0;
    return c;
  }
  /* MemoryDataIterator hands out <= 1 MiB slices (Common.h:126-144, 154-165). */
  size_t done = 0;
  while (done < len) {
    size_t n = len - done < ORC_SLICE ? len - done : ORC_SLICE;
    if (type == ORC_CRC32C)
      c.value = orc_crc32c_hw(c.value, p + done, n);
    else if (type == ORC_CRC32)
      c.value = orc_crc32_sw(c.value, p + done, n);
    done += n;
  }
  return c;
}

int orc_checksum_combine(orc_checksum *self, orc_checksum o, size_t len) {
  if (self->type != ORC_NONE && self->type != o.type) return ORC_CHECKSUM_MISMATCH; /* :180-183 */
  if (len == 0) return ORC_OK;                                                    /* :184 */
  switch (self->type) {
    case ORC_NONE:
      *self = o;
      return ORC_OK;
    case ORC_CRC32C:
      self->value = orc_crc32c_combine(~self->value, o.value, len);
      return ORC_OK;
    case ORC_CRC32:
      self->value = orc_crc32_combine(~self->value, o.value, len);
      return ORC_OK;
  }
  return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* ChunkReplica::updateChecksum (ChunkReplica.cc:319-394)                    */
/* ------------------------------------------------------------------------ */
/* *kase: the counter the reference bumps (ChunkReplica.cc:25-28): 1 checksum_none,
 * 2 checksum_reuse, 3 checksum_combine, 4 checksum_read_chunk. */
static int replica_update_impl(const uint8_t *chunk_after, uint32_t size_after, orc_checksum chunk_ck,
                               orc_checksum write_ck, uint32_t off, uint32_t len, int trunc_or_extend,
                               uint32_t size_before, int is_append, orc_checksum *out, int *kase) {
  int combine_ck = size_before > 0 && is_append;
  uint32_t value;
  int k;
  if (trunc_or_extend) { /* :328-332 */
    write_ck = orc_checksum_create(chunk_ck.type, NULL, 0, ~0u);
    off = size_after;
    len = 0;
  }
  if (write_ck.type == ORC_NONE || size_after == 0) { /* :334-336 */
    value = 0;
    k = 1;
  } else if (off == 0 && len == size_after) { /* :337-339 reuse */
    value = write_ck.value;
    k = 2;
  } else if (write_ck.type == chunk_ck.type && combine_ck) { /* :340-355 append */
    orc_checksum c = chunk_ck;
    int rc = orc_checksum_combine(&c, write_ck, len);
    if (rc) return rc;
    value = c.value;
    k = 3;
  } else { /* :356-389 prefix + payload + suffix */
    k = 4;
    if ((uint64_t)off > size_after) return ORC_INVALID_ARG;
    orc_checksum prefix = orc_checksum_create(write_ck.type, chunk_after, off, ~0u);
    uint32_t suffix_start = off + len < size_after ? off + len : size_after;
    uint32_t suffix_len = size_after - suffix_start;
    orc_checksum suffix = orc_checksum_create(write_ck.type, chunk_after + suffix_start, suffix_len, ~0u);
    orc_checksum_combine(&prefix, write_ck, len);
    orc_checksum_combine(&prefix, suffix, suffix_len);
    value = prefix.value;
  }
  out->type = write_ck.type; /* :392 */
  out->value = value;
  if (kase) *kase = k;
  return ORC_OK;
}

int orc_replica_update_checksum(const uint8_t *chunk_after, uint32_t size_after, orc_checksum chunk_ck,
                                orc_checksum write_ck, uint32_t off, uint32_t len, int trunc_or_extend,
                                uint32_t size_before, int is_append, orc_checksum *out) {
  return replica_update_impl(chunk_after, size_after, chunk_ck, write_ck, off, len, trunc_or_extend, size_before,
                             is_append, out, NULL);
}

int orc_replica_update_checksum_case(const uint8_t *chunk_after, uint32_t size_after, orc_checksum chunk_ck,
                                     orc_checksum write_ck, uint32_t off, uint32_t len, int trunc_or_extend,
                                     uint32_t size_before, int is_append, orc_checksum *out, int *kase) {
  *kase = 0;
  return replica_update_impl(chunk_after, size_after, chunk_ck, write_ck, off, len, trunc_or_extend, size_before,
                             is_append, out, kase);
}

/* ------------------------------------------------------------------------ */
/* chunk engine (chunk.rs:89-281, engine.rs:288-420), finalized convention    */
/* ------------------------------------------------------------------------ */
#define ENGINE_ALIGN 4096u /* utils/aligned.rs:4 */

/* *kase: the engine's checksum counter (chunk.rs:153,156,188,217,233,273): 1 none,
 * 2 checksum_reuse, 3 checksum_combine, 4 checksum_recalculate. */
static int engine_safe_write(uint8_t *buf, uint32_t *len, uint32_t *ck, const uint8_t *data, uint32_t dlen,
                             uint32_t off, uint32_t data_ck, int truncate, int *kase) {
  *kase = 1;
  if (truncate && off < *len) { /* chunk.rs:184-198 */
    *len = off;
    *ck = orc_rs_crc32c(buf, off);
    *kase = 4;
    return ORC_OK;
  }
  int aligned_buf = dlen == 0 || (((uintptr_t)data % ENGINE_ALIGN) == 0 && dlen % ENGINE_ALIGN == 0);
  if (*len % ENGINE_ALIGN == 0 && off % ENGINE_ALIGN == 0 && aligned_buf) { /* :200-237 */
    if (off > *len) {
      memset(buf + *len, 0, off - *len);
      *ck = orc_rs_crc32c_append(*ck, buf + *len, off - *len); /* :213 */
      *len = off;
      *kase = 3;
    }
    if (dlen) {
      if (off != *len) return ORC_INVALID_ARG;
      memcpy(buf + off, data, dlen);
      *len = off + dlen;
      *ck = orc_rs_crc32c_combine(*ck, data_ck, dlen); /* :229 */
      *kase = 3;
    }
  } else if (*len < off + dlen) { /* :238-277 indirect append */
    if (*len > off) return ORC_INVALID_ARG;
    if (*len < off) memset(buf + *len, 0, off - *len);
    if (dlen) memcpy(buf + off, data, dlen); /* data may be NULL when dlen == 0 (UBSan) */
    uint32_t new_len = off + dlen;
    *ck = orc_rs_crc32c_append(*ck, buf + *len, new_len - *len); /* :266 */
    *len = new_len;
    *kase = 3;
  } else if (dlen != 0) {
    return ORC_INVALID_ARG;
  }
  return ORC_OK;
}

int orc_engine_write_case(uint8_t *buf, uint32_t *len_io, uint32_t *ck_io, uint32_t capacity, const uint8_t *data,
                          uint32_t dlen, uint32_t off, uint32_t data_ck, int truncate, int is_syncing, int exists,
                          int *kase) {
  *kase = 0;
  if (dlen != 0 && orc_rs_crc32c(data, dlen) != data_ck) return ORC_CHECKSUM_MISMATCH; /* engine.rs:297-311 */
  if (!exists) {
    *len_io = 0;
    *ck_io = 0;
    return engine_safe_write(buf, len_io, ck_io, data, dlen, off, data_ck, truncate, kase);
  }
  if (is_syncing || (dlen > 0 && off < *len_io) || (uint64_t)off + dlen > capacity) { /* copy_on_write */
    uint32_t old_len = *len_io;
    uint32_t new_len = old_len > off + dlen ? old_len : off + dlen;
    int skip_read = is_syncing || (off == 0 && dlen >= old_len);
    if (old_len < off) memset(buf + old_len, 0, off - old_len);
    if (dlen) memcpy(buf + off, data, dlen);
    *ck_io = skip_read ? data_ck : orc_rs_crc32c(buf, new_len); /* chunk.rs:150-158 */
    *len_io = is_syncing ? off + dlen : new_len;
    *kase = skip_read ? 2 : 4;
    return ORC_OK;
  }
  return engine_safe_write(buf, len_io, ck_io, data, dlen, off, data_ck, truncate, kase);
}

int orc_engine_write(uint8_t *buf, uint32_t *len_io, uint32_t *ck_io, uint32_t capacity, const uint8_t *data,
                     uint32_t dlen, uint32_t off, uint32_t data_ck, int truncate, int is_syncing, int exists) {
  int kase;
  return orc_engine_write_case(buf, len_io, ck_io, capacity, data, dlen, off, data_ck, truncate, is_syncing, exists,
                               &kase);
}

/* ------------------------------------------------------------------------ */
/* AioReadJob::setResult (BatchReadJob.cc:24-63)                              */
/* ------------------------------------------------------------------------ */
int orc_read_result_checksum(uint8_t batch_type, orc_checksum chunk_ck, uint32_t read_off, uint32_t read_len,
                             uint32_t chunk_len, const uint8_t *read_data, const uint8_t *full_chunk,
                             int recalculate, orc_checksum *out) {
  if (batch_type == ORC_NONE) {
    out->type = ORC_NONE;
    out->value = 0;
  } else if (batch_type == chunk_ck.type && read_off == 0 && read_len == chunk_len) {
    *out = chunk_ck;
  } else {
    *out = orc_checksum_create(batch_type, read_data, read_len, ~0u);
  }
  if (recalculate && read_off == 0 && read_len == chunk_len) {
    orc_checksum real = orc_checksum_create(chunk_ck.type, full_chunk, read_len, ~0u);
    if (real.type != chunk_ck.type || real.value != chunk_ck.value) return ORC_CHECKSUM_MISMATCH;
  }
  return ORC_OK;
}

/* Checksum::calcSerde (MessageHeader.h:33-37): init 0, low byte = magic|compressed */
uint32_t orc_calc_serde(const uint8_t *p, size_t n, int compressed) {
  uint32_t c = orc_crc32c_hw(0, p, n);
  return (c & ~0xffu) | 0x86u | (compressed ? 1u : 0u);
}

/* ------------------------------------------------------------------------ */
/* batched CPU baseline                                                      */
/* ------------------------------------------------------------------------ */
typedef struct {
  const uint8_t *base;
  size_t stride, len, n, first, step;
  uint32_t *out;
  int kind;
} batch_job;

static void *batch_worker(void *arg) {
  batch_job *j = (batch_job *)arg;
  for (size_t i = j->first; i < j->n; i += j->step) {
    const uint8_t *p = j->base + i * j->stride;
    orc_checksum c;
    if (j->kind == 0) {
      c = orc_checksum_create(ORC_CRC32C, p, j->len, ~0u);
    } else if (j->kind == 2) { /* the clmul leg, 1 MiB slices as ChecksumInfo::create feeds them */
      c.value = ~0u;
      for (size_t d = 0; d < j->len; d += ORC_SLICE)
        c.value = orc_crc32c_clmul(c.value, p + d, j->len - d < ORC_SLICE ? j->len - d : ORC_SLICE);
    } else {
      c.value = ~0u;
      for (size_t d = 0; d < j->len; d += ORC_SLICE)
        c.value = orc_crc32c_sw(c.value, p + d, j->len - d < ORC_SLICE ? j->len - d : ORC_SLICE);
    }
    j->out[i] = c.value;
  }
  return NULL;
}

void orc_create_batch(const uint8_t *base, size_t stride, size_t len, size_t n, uint32_t *out, int threads,
                      int kind) {
  ensure_init();
  if (threads <= 1) {
    batch_job j = {base, stride, len, n, 0, 1, out, kind};
    batch_worker(&j);
    return;
  }
  pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  batch_job *jobs = (batch_job *)calloc((size_t)threads, sizeof(batch_job));
  for (int t = 0; t < threads; ++t) {
    batch_job j = {base, stride, len, n, (size_t)t, (size_t)threads, out, kind};
    jobs[t] = j;
    pthread_create(&tid[t], NULL, batch_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  free(tid);
  free(jobs);
}

/* CPU baselines of the other configs (d3 ragged updates, d5 KV-block verify):
 * the reference's per-IO work, spread over `threads` pthreads.               */
typedef struct {
  uint8_t *chunks;
  size_t chunk_stride;
  const uint8_t *payload;
  size_t payload_stride;
  uint32_t *sizes, *cks, *offs, *lens, *wcks;
  int32_t *status;
  size_t n, first, step;
} update_job;

/* ChunkReplica::update on host bytes (ChunkReplica.cc:132-394): verify the
 * payload CRC (:193-207), gap zero-fill + write (:281-292), updateChecksum
 * with the prefix and suffix re-hashed from the chunk (:356-389; CRC32C). */
static void *update_worker(void *arg) {
  update_job *j = (update_job *)arg;
  for (size_t i = j->first; i < j->n; i += j->step) {
    uint8_t *c = j->chunks + i * j->chunk_stride;
    const uint8_t *p = j->payload + i * j->payload_stride;
    const uint32_t off = j->offs[i], len = j->lens[i], s0 = j->sizes[i];
    if (orc_crc32c_hw(~0u, p, len) != j->wcks[i]) {
      j->status[i] = ORC_CHECKSUM_MISMATCH;
      continue;
    }
    if (off > s0) memset(c + s0, 0, off - s0);
    if (len) memcpy(c + off, p, len);
    const uint32_t s1 = off + len > s0 ? off + len : s0;
    orc_checksum out;
    const orc_checksum cck = {ORC_CRC32C, j->cks[i]}, wck = {ORC_CRC32C, j->wcks[i]};
    j->status[i] = orc_replica_update_checksum(c, s1, cck, wck, off, len, 0, s0, off == s0, &out);
    j->sizes[i] = s1;
    j->cks[i] = out.value;
  }
  return NULL;
}

void orc_replica_update_batch(uint8_t *chunks, size_t chunk_stride, const uint8_t *payload, size_t payload_stride,
                              uint32_t *sizes, uint32_t *cks, uint32_t *offs, uint32_t *lens, uint32_t *wcks,
                              int32_t *status, size_t n, int threads) {
  ensure_init();
  if (threads < 1) threads = 1;
  pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  update_job *jobs = (update_job *)calloc((size_t)threads, sizeof(update_job));
  for (int t = 0; t < threads; ++t) {
    update_job j = {chunks, chunk_stride, payload, payload_stride, sizes, cks, offs, lens, wcks, status,
                    n, (size_t)t, (size_t)threads};
    jobs[t] = j;
    pthread_create(&tid[t], NULL, update_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  free(tid);
  free(jobs);
}

typedef struct {
  const uint8_t *arena;
  const uint64_t *offs;
  const uint32_t *lens, *expected;
  uint8_t *mismatch;
  size_t n, first, step;
} verify_job;

static void *verify_worker(void *arg) {
  verify_job *j = (verify_job *)arg;
  for (size_t i = j->first; i < j->n; i += j->step)
    j->mismatch[i] = orc_crc32c_hw(~0u, j->arena + j->offs[i], j->lens[i]) != j->expected[i];
  return NULL;
}

/* client read verify of KV blocks (StorageClientImpl.cc:1720-1737) */
size_t orc_verify_blocks(const uint8_t *arena, const uint64_t *offs, const uint32_t *lens, const uint32_t *expected,
                         uint8_t *mismatch, size_t n, int threads) {
  ensure_init();
  if (threads < 1) threads = 1;
  pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  verify_job *jobs = (verify_job *)calloc((size_t)threads, sizeof(verify_job));
  for (int t = 0; t < threads; ++t) {
    verify_job j = {arena, offs, lens, expected, mismatch, n, (size_t)t, (size_t)threads};
    jobs[t] = j;
    pthread_create(&tid[t], NULL, verify_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  free(tid);
  free(jobs);
  size_t bad = 0;
  for (size_t i = 0; i < n; ++i) bad += mismatch[i];
  return bad;
}

/* ------------------------------------------------------------------------ */
/* synthetic data                                             */
/* ------------------------------------------------------------------------ */
static inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* ------------------------------------------------------------------------ */
/* FileWrapper::readFile's checksum fold (src/client/cli/admin/FileWrapper.cc: */
/* 119-164), per file or replica (Checksum.cc:43-88); as oracle.py file_digest */
/* ------------------------------------------------------------------------ */
/* create(CRC32C, zeros, need) (FileWrapper.cc:151-153): the reference hashes a
 * buffer of real zero bytes, 1 MiB slices at a time. */
static uint32_t crc32c_zeros(uint64_t need) {
  static uint8_t zeros[ORC_SLICE];
  uint32_t c = ~0u;
  for (uint64_t d = 0; d < need; d += ORC_SLICE) c = orc_crc32c_hw(c, zeros, need - d < ORC_SLICE ? need - d : ORC_SLICE);
  return c;
}

int orc_file_digest(const orc_block_digest *b, uint64_t nb, int fill_zero, orc_checksum *out) {
  orc_checksum acc = {ORC_NONE, 0};
  out->type = ORC_NONE;
  out->value = 0;
  for (uint64_t i = 0; i < nb; ++i) /* malformed blocks: kInvalidArg before the fold */
    if (b[i].type > ORC_CRC32 || (fill_zero && !b[i].missing && b[i].read_len > b[i].block_len)) return ORC_INVALID_ARG;
  for (uint64_t i = 0; i < nb; ++i) {
    uint64_t succ = b[i].read_len;
    orc_checksum ck = {b[i].type, b[i].checksum};
    if (b[i].missing) { /* :134-138 */
      if (!fill_zero) return ORC_CHUNK_NOT_FOUND;
      succ = 0;
      ck.type = ORC_NONE;
      ck.value = 0;
    }
    if (succ != b[i].block_len) { /* :151-160 */
      if (!fill_zero) return ORC_INVALID_FORMAT;
      const uint64_t need = b[i].block_len - succ;
      const orc_checksum z = {ORC_CRC32C, crc32c_zeros(need)};
      int rc = orc_checksum_combine(&ck, z, need);
      if (rc) return rc;
      succ = b[i].block_len;
    }
    int rc = orc_checksum_combine(&acc, ck, succ); /* :163 */
    if (rc) return rc;
  }
  *out = acc;
  return ORC_OK;
}

typedef struct {
  const orc_block_digest *blocks;
  const uint64_t *file_off;
  uint64_t nfiles, first, step;
  int fill_zero;
  orc_file_result *out;
} digest_job;

static void *digest_worker(void *arg) {
  digest_job *j = (digest_job *)arg;
  for (uint64_t f = j->first; f < j->nfiles; f += j->step) {
    const uint64_t b0 = j->file_off[f], b1 = j->file_off[f + 1];
    orc_checksum ck;
    orc_file_result *o = &j->out[f];
    o->status = orc_file_digest(j->blocks + b0, b1 - b0, j->fill_zero, &ck);
    o->type = o->status ? ORC_NONE : ck.type;
    o->value = o->status ? 0 : ck.value;
  }
  return NULL;
}

void orc_file_digest_batch(const orc_block_digest *blocks, const uint64_t *file_off, uint64_t nfiles, int fill_zero,
                           orc_file_result *out, int threads) {
  ensure_init();
  if (threads < 1) threads = 1;
  pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  digest_job *jobs = (digest_job *)calloc((size_t)threads, sizeof(digest_job));
  for (int t = 0; t < threads; ++t) {
    digest_job j = {blocks, file_off, nfiles, (uint64_t)t, (uint64_t)threads, fill_zero, out};
    jobs[t] = j;
    pthread_create(&tid[t], NULL, digest_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  free(tid);
  free(jobs);
}

/* ChecksumInfo::combine element-wise (Common.h:179-198, typed values): acc = combine(~acc,
 * crc2, len2) for len2 > 0 -- the CPU baseline of hf3fs_crc_combine_batch. */
typedef struct {
  uint32_t *acc;
  const uint32_t *crc2;
  const uint64_t *len2;
  size_t n, first, step;
  uint32_t poly;
} combine_job;

static void *combine_worker(void *arg) {
  combine_job *j = (combine_job *)arg;
  for (size_t i = j->first; i < j->n; i += j->step)
    if (j->len2[i]) j->acc[i] = orc_shift(~j->acc[i], j->len2[i], j->poly) ^ j->crc2[i];
  return NULL;
}

void orc_combine_batch(uint32_t *acc, const uint32_t *crc2, const uint64_t *len2, size_t n, uint32_t poly,
                       int threads) {
  ensure_init();
  if (threads < 1) threads = 1;
  pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  combine_job *jobs = (combine_job *)calloc((size_t)threads, sizeof(combine_job));
  for (int t = 0; t < threads; ++t) {
    combine_job j = {acc, crc2, len2, n, (size_t)t, (size_t)threads, poly};
    jobs[t] = j;
    pthread_create(&tid[t], NULL, combine_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  free(tid);
  free(jobs);
}

void orc_fill_synth(uint8_t *dst, size_t n, uint64_t seed, uint64_t chunk_id, uint64_t byte_off) {
  uint64_t key = seed ^ (chunk_id << 32);
  size_t i = 0;
  while (i < n) {
    uint64_t pos = byte_off + i;
    uint64_t w = splitmix64(key ^ (pos >> 3));
    size_t sub = (size_t)(pos & 7);
    size_t take = 8 - sub;
    if (take > n - i) take = n - i;
    for (size_t k = 0; k < take; ++k) dst[i + k] = (uint8_t)(w >> (8 * (sub + k)));
    i += take;
  }
}
