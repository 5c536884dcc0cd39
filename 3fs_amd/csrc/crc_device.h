// crc_device.h -- device building blocks of the CRC kernels,
// shared by crc_kernels.hip (create/verify, request service) and
// update_kernels.hip (fused verify + write + delta hash):
//   * 16 B granule loads/stores in the global address space (optionally
//     non-temporal), unaligned 16 B loads from two aligned ones;
//   * the 4-streams-per-lane stride-1024 CRC update through the lane's private
//     LDS table replica, and the fold of a wave's 256 stream registers;
//   * signed powers of x, computed lane-parallel;
//   * whole-workgroup hashing of one range, and write-while-hashing of the
//     old bytes a write overwrites.
#pragma once
#include "crc_kernels.h"

namespace hf3fs_crc {

#ifndef HF3FS_HASH_PREFETCH
#define HF3FS_HASH_PREFETCH 4
#endif
constexpr int kHashPrefetch = HF3FS_HASH_PREFETCH;  // 1 KiB blocks in flight per wave while hashing

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_cu32x4;
typedef __attribute__((address_space(1))) u32x4 g_u32x4;

// global_load_dwordx4 (address space 1, not flat: flat loads would also count
// on lgkmcnt and serialise against the LDS table reads).
__device__ __forceinline__ uint4 gload16(uint64_t addr) {
  const u32x4 v = *reinterpret_cast<g_cu32x4*>(addr);
  return make_uint4(v.x, v.y, v.z, v.w);
}
// The streamed body of a range: optionally non-temporal (read-once data).
template <bool NT>
__device__ __forceinline__ uint4 gload16s(uint64_t addr) {
  if (NT) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<g_cu32x4*>(addr));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return gload16(addr);
}

// Bytes [lo, hi) of dword `d` (byte positions 4d..4d+3 of a granule) kept.
__device__ __forceinline__ uint32_t dword_mask(int s, int e, int d) {
  int lo = s - 4 * d, hi = e - 4 * d;
  lo = lo < 0 ? 0 : lo;
  hi = hi > 4 ? 4 : hi;
  if (hi <= lo) return 0u;
  uint32_t m = hi == 4 ? 0xffffffffu : ((1u << (8 * hi)) - 1u);
  return m & ~((1u << (8 * lo)) - 1u);
}

// 16-byte granule at g (16-aligned) with only bytes inside [lo, hi) kept.
// The aligned granule never crosses a page, so touching it is safe whenever
// at least one of its bytes belongs to the buffer; fully outside -> no load.
__device__ __forceinline__ uint4 gload16_masked(uint64_t g, uint64_t lo, uint64_t hi) {
  uint64_t a = lo > g ? lo : g;
  uint64_t b = hi < g + 16 ? hi : g + 16;
  if (a >= b) return make_uint4(0, 0, 0, 0);
  uint4 w = gload16(g);
  int s = (int)(a - g), e = (int)(b - g);
  w.x &= dword_mask(s, e, 0);
  w.y &= dword_mask(s, e, 1);
  w.z &= dword_mask(s, e, 2);
  w.w &= dword_mask(s, e, 3);
  return w;
}

// The step tables in LDS: table k (byte k of the stream word), entry e, replica c at byte
//   (k >> 1) * 65536 + e * 256 + (k & 1) * 128 + c * 4,
// lane l reading replica l % 32 (bank l % 32: every lookup conflict-free whatever the data).
// With this layout ONE v_perm_b32 forms a lookup address: byte k of the word lands in address
// byte 1, and the lane's replica offset, the table's half and its 64 KiB pair come from one
// per-lane constant (two VALU ops per lookup before: the byte extract, then the lane offset).
struct StepLds {
  const uint8_t* base;  // the LDS image (uniform)
  uint32_t c;           // bytes: [l % 32 * 4, l % 32 * 4 + 128, 0, 1]
};
__device__ __forceinline__ StepLds step_lds(const uint32_t* lds, int lane) {
  const uint32_t o = (uint32_t)(lane & 31) * 4;
  return StepLds{reinterpret_cast<const uint8_t*>(lds), o | ((o | 128u) << 8) | (1u << 24)};
}
// perm selectors: address byte 0 <- constant byte (k & 1), byte 1 <- word byte k,
// byte 2 <- constant byte 2 + (k >> 1), byte 3 <- 0
__device__ __forceinline__ uint32_t step_lookup(uint32_t x, const StepLds& L, uint32_t sel) {
  return *reinterpret_cast<const uint32_t*>(L.base + __builtin_amdgcn_perm(x, L.c, sel));
}
// One stream update: x * x^8192 via the lane's private LDS table copy, as the two halves
// of the four lookups' xor: p = T0 ^ T1 ^ T2 (one v_bitop3), t = T3.
__device__ __forceinline__ void stride_step2(uint32_t x, const StepLds& lj, uint32_t& p, uint32_t& t) {
  p = __builtin_amdgcn_bitop3_b32(step_lookup(x, lj, 0x0C020400u), step_lookup(x, lj, 0x0C020501u),
                                  step_lookup(x, lj, 0x0C030600u), 0x96);
  t = step_lookup(x, lj, 0x0C030701u);
}
__device__ __forceinline__ uint32_t stride_step(uint32_t x, const StepLds& lj) {
  uint32_t p, t;
  stride_step2(x, lj, p, t);
  return p ^ t;
}
// LDS byte offset of step[k][e], replica c (fill_lds)
__host__ __device__ constexpr uint32_t step_lds_offset(int k, int e, int c) {
  return (uint32_t)(k >> 1) * 65536u + (uint32_t)e * 256u + (uint32_t)(k & 1) * 128u + (uint32_t)c * 4u;
}

// The 256 CRC streams of a wave: lane l, dword d of its granule.  Stream d's register is
// p_d ^ t_d (s_d() below), kept as the two halves of its last update so that the next update
// xors them with the data word in ONE v_bitop3: 6 VALU ops per stream and block (4 address
// perms, 2 xor3) instead of 8.
struct Streams {
  uint32_t p0 = 0, p1 = 0, p2 = 0, p3 = 0, t0 = 0, t1 = 0, t2 = 0, t3 = 0;
  __device__ __forceinline__ void step(const uint4& w, const StepLds& lj) {
    stride_step2(__builtin_amdgcn_bitop3_b32(p0, t0, w.x, 0x96), lj, p0, t0);
    stride_step2(__builtin_amdgcn_bitop3_b32(p1, t1, w.y, 0x96), lj, p1, t1);
    stride_step2(__builtin_amdgcn_bitop3_b32(p2, t2, w.z, 0x96), lj, p2, t2);
    stride_step2(__builtin_amdgcn_bitop3_b32(p3, t3, w.w, 0x96), lj, p3, t3);
  }
  __device__ __forceinline__ uint32_t s0() const { return p0 ^ t0; }
  __device__ __forceinline__ uint32_t s1() const { return p1 ^ t1; }
  __device__ __forceinline__ uint32_t s2() const { return p2 ^ t2; }
  __device__ __forceinline__ uint32_t s3() const { return p3 ^ t3; }
};

// LDS image: [0, kLdsWords) the 4 x 256 step table, 32 replicas per entry (StepLds
// layout above), so the hot loop is bank-conflict free.  [kLdsWords, +kMulcWords) the seven
// constant-multiply tables of the fold (read rarely; not replicated).
__device__ __forceinline__ void fill_step_tables(uint32_t* lds, const PolyTables* T) {
  const uint32_t* step = &T->step[0][0];
  for (int e = threadIdx.x; e < 1024; e += blockDim.x) {
    const uint32_t v = step[e];
    const uint4 v4 = make_uint4(v, v, v, v);
    uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(lds) + step_lds_offset(e >> 8, e & 255, 0));
#pragma unroll
    for (int c = 0; c < kCopies / 4; ++c) dst[c] = v4;
  }
}
__device__ __forceinline__ void fill_lds(uint32_t* lds, const PolyTables* T) {
  fill_step_tables(lds, T);
  const uint4* msrc = reinterpret_cast<const uint4*>(&T->mulc[0][0][0]);
  uint4* mdst = reinterpret_cast<uint4*>(lds + kLdsWords);
  for (int e = threadIdx.x; e < kMulcWords / 4; e += blockDim.x) mdst[e] = msrc[e];
  __syncthreads();
}

// a * C_k with the byte tables of constant C_k (lc = LDS base of table k).
__device__ __forceinline__ uint32_t mulc(uint32_t a, const uint32_t* lc) {
  return lc[a & 0xffu] ^ lc[256 + ((a >> 8) & 0xffu)] ^ lc[512 + ((a >> 16) & 0xffu)] ^ lc[768 + (a >> 24)];
}

// ---- the lane-weight fold (FoldTables, crc_kernels.h) ----------------------
// Lane l's Horner value over its 4 streams (byte tables of x^-32) is weighted by
// x^(-128 (l % 32)) from its own column of the nibble weight tables (conflict-free), the
// wave is xor-reduced by DPP (no multiplies in the tree) and the upper half shifted by
// x^-4096 once (byte tables; the value is wave-uniform there).  Every lookup address is one
// VALU op or none.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {  // lanes without a source read 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, true);
}
constexpr int kRowShl = 0x100, kRowShr = 0x110, kRowBcast15 = 0x142, kRowBcast31 = 0x143;
struct FoldLds {
  const uint32_t* wl;  // w + lane % 32
  const uint32_t* c0;  // byte tables of x^-32
  const uint32_t* ch;  // byte tables of x^-4096
};
// the LDS image of FoldTables at fb (after the step tables)
__device__ __forceinline__ FoldLds fold_lds(const uint32_t* fb) {
  return FoldLds{fb + (threadIdx.x & 31), fb + 8 * 16 * 32, fb + 8 * 16 * 32 + 4 * 256};
}
// a * C through the byte tables of C (4 x 256 words)
__device__ __forceinline__ uint32_t mulc_b(uint32_t a, const uint32_t* tab) {
  return tab[a & 0xffu] ^ tab[256 + ((a >> 8) & 0xffu)] ^ tab[512 + ((a >> 16) & 0xffu)] ^ tab[768 + (a >> 24)];
}
// a * x^(-128 (lane % 32)): the lane's column of the weight table
__device__ __forceinline__ uint32_t mulc_w(uint32_t a, const uint32_t* wl) {
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r ^= wl[(16 * j + ((a >> (4 * j)) & 15u)) * 32];
  return r;
}
__device__ __forceinline__ uint32_t weighted_lw(const Streams& s, const FoldLds& f) {  // x^(-128 l') sum_d s_d x^(-32 d)
  uint32_t u = mulc_b(s.s3(), f.c0) ^ s.s2();
  u = mulc_b(u, f.c0) ^ s.s1();
  return mulc_w(mulc_b(u, f.c0) ^ s.s0(), f.wl);
}
// inclusive xor-prefix of v within each 32-lane half
__device__ __forceinline__ uint32_t half_scan(uint32_t v) {
  v ^= dpp<kRowShr + 1>(v);
  v ^= dpp<kRowShr + 2>(v);
  v ^= dpp<kRowShr + 4>(v);
  v ^= dpp<kRowShr + 8>(v);
  return v ^ dpp<kRowBcast15, 0xa>(v);
}
// sum_{l,d} s_{l,d} x^(-32 (4l + d)), wave-uniform
__device__ __forceinline__ uint32_t fold_lw(const Streams& st, const FoldLds& f) {
  const uint32_t v = half_scan(weighted_lw(st, f));
  const uint32_t a = __builtin_amdgcn_readlane(v, 31), b = __builtin_amdgcn_readlane(v, 63);
  return a ^ mulc_b(b, f.ch);
}

// The step tables and, after them, the fold's constant tables: FoldTables
// (HF3FS_CRC_FOLD_LW, default) or the seven byte tables of PolyTables::mulc.
#ifndef HF3FS_CRC_FOLD_LW
#define HF3FS_CRC_FOLD_LW 1
#endif
constexpr int kFoldLdsWords = HF3FS_CRC_FOLD_LW ? kFoldWords : kMulcWords;
// FoldTables of the polynomial of T (kernels get T = &DeviceTables::poly[k], k = 1 for CRC32)
template <uint32_t POLY>
__device__ __forceinline__ const FoldTables* fold_tables_of(const PolyTables* T) {
  constexpr int k = POLY == kPolyCrc32 ? 1 : 0;
  return &reinterpret_cast<const DeviceTables*>(T - k)->fold[k];
}
// step tables + FoldTables F (whatever HF3FS_CRC_FOLD_LW says; the serde-frame kernel)
__device__ __forceinline__ void fill_lds_foldtables(uint32_t* lds, const PolyTables* T, const FoldTables* F) {
  fill_step_tables(lds, T);
  const uint4* fsrc = reinterpret_cast<const uint4*>(F);
  uint4* fdst = reinterpret_cast<uint4*>(lds + kLdsWords);
  for (int e = threadIdx.x; e < kFoldWords / 4; e += blockDim.x) fdst[e] = fsrc[e];
  __syncthreads();
}
template <uint32_t POLY>
__device__ __forceinline__ void fill_lds_fold(uint32_t* lds, const PolyTables* T) {
#if HF3FS_CRC_FOLD_LW
  fill_lds_foldtables(lds, T, fold_tables_of<POLY>(T));
#else
  fill_lds(lds, T);
#endif
}
// Fold the 256 stream registers of a wave into one value (in lane 0; every
// lane with the lane-weight fold):
//   R = sum_{l,d} s_{l,d} * x^(-32 (4l + d))
// Stream (l,d) carries an extra x^(32(4l+d)) relative to the block grid's end,
// so R = lin(grid bytes) exactly.  Byte-table form: in-lane Horner with
// C_0 = x^-32, then a shuffle tree with C_{k+1} = x^(-128*2^k) applied to the
// LATER lane of each pair.
__device__ __forceinline__ uint32_t fold_streams(const Streams& st, const uint32_t* lc, int lane) {
#if HF3FS_CRC_FOLD_LW
  (void)lane;
  return fold_lw(st, fold_lds(lc));
#else
  uint32_t u = mulc(st.s3(), lc) ^ st.s2();
  u = mulc(u, lc) ^ st.s1();
  u = mulc(u, lc) ^ st.s0();
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const uint32_t o = __shfl_down(u, 1 << k, 64);
    // only the lanes that keep a partial sum look up (fewer LDS bank conflicts)
    if ((lane & ((2 << k) - 1)) == 0) u ^= mulc(o, lc + (k + 1) * 1024);
  }
  return u;
#endif
}

// Stream nb 1 KiB blocks starting at vs (16-aligned) through the lane
// registers; bytes outside [a0, a1) read as zero (an aligned 16 B granule never
// crosses a page, and fully-outside granules are not loaded).  Block 0 holds a0.
// INIT: xor `start` into data bytes a0..a0+3 (raw(D, s) = lin(D with its first
// 4 bytes ^ s) for |D| >= 4), which replaces the start * x^(8 len) term.
// `st` continues the streams of the blocks in front of vs (the update is linear).
// QTAIL: queue the leftover blocks behind the last full group (below); off in
// the update kernels, where the extra registers spill.
template <bool INIT, bool NT, int U = kHashPrefetch, bool QTAIL = true>
__device__ __forceinline__ Streams hash_grid(uint64_t vs, uint64_t nb, uint64_t a0, uint64_t a1, uint32_t start,
                                             const StepLds& lj, int lane, Streams st = Streams()) {
  const uint64_t lane_off = (uint64_t)lane * 16;
  const uint64_t lb = (a1 - vs) / kBlockBytes;  // blocks ending at or before a1
  uint64_t b = 0;
  const bool head_full = vs >= a0 && lb >= 1;
  // INIT with a full head block (vs == a0: the start lands in lane 0's first dword) of a range
  // of <= 64 blocks: block 0 goes out with the first group of loads and takes the start when
  // it is stepped.  (Loaded and stepped alone, it cost every whole-buffer task one exposed
  // load latency: a 4 KiB KV block paid two; all-4 KiB d5 -10 % in one process.)
  bool init_late = INIT && head_full && nb <= 64;  // (long ranges: one latency per range is noise)
  auto late_xor = [&](uint4 w) -> uint4 {
    if (init_late) {  // wave-uniform
      w.x ^= lane == 0 ? start : 0u;
      init_late = false;
    }
    return w;
  };
  if (!head_full || (INIT && !init_late)) {
    uint4 w = head_full ? gload16s<NT>(vs + lane_off) : gload16_masked(vs + lane_off, a0, a1);
    if (INIT) {
      const int o = (int)(a0 - vs) - 16 * lane;  // start's byte offset within this lane's granule
#define HF3FS_INIT_XOR(F, D)                                           \
  {                                                                    \
    const int sh = o - 4 * (D);                                        \
    if (sh > -4 && sh < 4) w.F ^= sh >= 0 ? start << (8 * sh) : start >> (-8 * sh); \
  }
      HF3FS_INIT_XOR(x, 0)
      HF3FS_INIT_XOR(y, 1)
      HF3FS_INIT_XOR(z, 2)
      HF3FS_INIT_XOR(w, 3)
#undef HF3FS_INIT_XOR
    }
    st.step(w, lj);
    b = 1;
  }
  const uint64_t nfull = lb > b ? lb - b : 0;
  const uint64_t gbase = vs + b * kBlockBytes + lane_off;
  // full blocks go U at a time with the next U in flight; the leftover full
  // blocks (< U) and the masked last block are issued together before the last
  // full group is hashed, so a range pays one exposed load latency at its end
  // instead of one per leftover block (wave-uniform predicates throughout)
  const bool tail = lb < nb && lb >= b;
  uint64_t g = 0;
  uint4 c[U];
  if (nfull >= U) {
#pragma unroll
    for (int k = 0; k < U; ++k) c[k] = gload16s<NT>(gbase + k * kBlockBytes);
    g = U;
    if (init_late && g + U <= nfull) {  // the first group takes the start: peeled, so the loop stays xor-free
      uint4 nx[U];
#pragma unroll
      for (int k = 0; k < U; ++k) nx[k] = gload16s<NT>(gbase + g * kBlockBytes + k * kBlockBytes);
      st.step(late_xor(c[0]), lj);
#pragma unroll
      for (int k = 1; k < U; ++k) st.step(c[k], lj);
#pragma unroll
      for (int k = 0; k < U; ++k) c[k] = nx[k];
      g += U;
    }
    for (; g + U <= nfull; g += U) {
      const uint64_t q = gbase + g * kBlockBytes;
      uint4 nx[U];
#pragma unroll
      for (int k = 0; k < U; ++k) nx[k] = gload16s<NT>(q + k * kBlockBytes);
#pragma unroll
      for (int k = 0; k < U; ++k) st.step(c[k], lj);
#pragma unroll
      for (int k = 0; k < U; ++k) c[k] = nx[k];
    }
  }
  if (!QTAIL) {
    if (nfull >= U) {
      st.step(late_xor(c[0]), lj);
#pragma unroll
      for (int k = 1; k < U; ++k) st.step(c[k], lj);
    }
    for (; g < nfull; ++g) st.step(late_xor(gload16s<NT>(gbase + g * kBlockBytes)), lj);
    if (tail) st.step(gload16_masked(gbase + nfull * kBlockBytes, a0, a1), lj);
    return st;
  }
  const uint64_t rem = nfull - g;  // < U
  uint4 r[U - 1];
#pragma unroll
  for (int k = 0; k < U - 1; ++k)
    r[k] = (uint64_t)k < rem ? gload16s<NT>(gbase + (g + k) * kBlockBytes) : make_uint4(0, 0, 0, 0);
  const uint4 m = tail ? gload16_masked(gbase + nfull * kBlockBytes, a0, a1) : make_uint4(0, 0, 0, 0);
  if (nfull >= U) {
    st.step(late_xor(c[0]), lj);
#pragma unroll
    for (int k = 1; k < U; ++k) st.step(c[k], lj);
  }
#pragma unroll
  for (int k = 0; k < U - 1; ++k)
    if ((uint64_t)k < rem) st.step(late_xor(r[k]), lj);
  if (tail) st.step(m, lj);
  return st;
}

// x^(e) for a signed bit count e; every lane of each 32-lane half computes the
// same exponent (lanes 0-31: eA, lanes 32-63: eB) in 5 butterfly rounds.
template <uint32_t POLY>
__device__ __forceinline__ uint32_t xpow_pair(int64_t eA, int64_t eB, int lane, const PolyTables* T) {
  const int64_t e = lane < 32 ? eA : eB;
  const int k = lane & 31;
  const uint64_t m = e < 0 ? (uint64_t)(-e) : (uint64_t)e;
  const uint32_t* tab = e < 0 ? T->xinv : T->xpow;
  uint32_t f = ((m >> k) & 1u) ? tab[k] : kOne;
  if (m >> 32) {
    const uint32_t h = ((m >> (k + 32)) & 1u) ? tab[k + 32] : kOne;
    f = gf_mul(f, h, POLY);
  }
#pragma unroll
  for (int d = 1; d < 32; d <<= 1) f = gf_mul(f, __shfl_xor(f, d, 64), POLY);
  return f;
}


template <bool NT = false>
__device__ __forceinline__ u32x4 ld16(uint64_t a) {
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<g_cu32x4*>(a));
  return *reinterpret_cast<g_cu32x4*>(a);
}
template <bool NT = false>
__device__ __forceinline__ void st16(uint64_t a, u32x4 v) {
  if (NT)
    __builtin_nontemporal_store(v, reinterpret_cast<g_u32x4*>(a));
  else
    *reinterpret_cast<g_u32x4*>(a) = v;
}

// 16 bytes starting at arbitrary address S, all of which are valid.
template <bool NT = false>
__device__ __forceinline__ u32x4 ld16_unaligned(uint64_t S) {
  const uint64_t Sg = S & ~uint64_t(15);
  const uint32_t sh = (uint32_t)(S & 15);
  const u32x4 A = ld16<NT>(Sg);
  if (sh == 0) return A;
  const u32x4 B = ld16<NT>(Sg + 16);
  uint32_t w[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
  const uint32_t q = sh >> 2, r = sh & 3;
  uint32_t t[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) t[k] = q == 0 ? w[k] : q == 1 ? w[k + 1] : q == 2 ? w[k + 2] : w[k + 3];
  u32x4 o;
  o.x = __builtin_amdgcn_alignbyte(t[1], t[0], r);
  o.y = __builtin_amdgcn_alignbyte(t[2], t[1], r);
  o.z = __builtin_amdgcn_alignbyte(t[3], t[2], r);
  o.w = __builtin_amdgcn_alignbyte(t[4], t[3], r);
  return o;
}


// XOR of one value per wave (lane 0's) across the workgroup, in every thread.
// s_part: kWaves words of LDS.  Ends with a barrier so s_part can be reused.
__device__ __forceinline__ uint32_t wg_xor(uint32_t val, uint32_t* s_part) {
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = val;
  __syncthreads();
  uint32_t r = 0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) r ^= s_part[w];
  __syncthreads();
  return r;
}

// raw(bytes [base, base + len), start) hashed by all 16 waves of the
// workgroup: wave w takes the w-th 1 KiB-aligned slice (start-aligned grid),
// shifts its linear CRC to the end of the range by x^(8 e), wave 0 adds
// start * x^(8 len).  Every thread of the workgroup calls it (barriers
// inside) and gets the value.
template <uint32_t POLY>
__device__ __forceinline__ uint32_t wg_hash(uint64_t base, uint64_t len, uint32_t start, const StepLds& lj,
                                            const uint32_t* lc, const PolyTables* T, uint32_t* s_part) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const uint64_t seg = ((len + kWaves - 1) / kWaves + kBlockBytes - 1) / kBlockBytes * kBlockBytes;
  const uint64_t tb = (uint64_t)wave * seg;
  uint32_t val = (wave == 0 && len == 0) ? start : 0u;  // create(type, buf, 0, start) == start
  if (tb < len) {  // wave-uniform: the butterfly in xpow_pair needs every lane
    const uint64_t te = len < tb + seg ? len : tb + seg;
    const uint64_t a0 = base + tb, a1 = base + te;
    const uint64_t vs = a0 & ~uint64_t(15);
    const uint64_t nb = (a1 - vs + kBlockBytes - 1) / kBlockBytes;
    const uint64_t vend = vs + nb * kBlockBytes;
    const Streams st = hash_grid<false, false, kHashPrefetch, false>(vs, nb, a0, a1, 0u, lj, lane);
    const uint32_t v = fold_streams(st, lc, lane);  // lin(slice) * x^(8 (vend - a1))
    const uint32_t f = xpow_pair<POLY>(8 * (int64_t)(base + len - vend), 8 * (int64_t)len, lane, T);
    val = gf_mul(__builtin_amdgcn_readfirstlane(v), __builtin_amdgcn_readlane(f, 0), POLY);
    if (wave == 0) val ^= gf_mul(start, __builtin_amdgcn_readlane(f, 32), POLY);
  }
  return wg_xor(val, s_part);
}

// Write P = src[0, len) over dst[0, len) (any alignments; src and dst do not
// overlap) and return lin(O) = raw(O, 0) of the OLD bytes dst[0, olen),
// olen <= len.  The block grid is aligned to dst and wave w takes the w-th run
// of 1 KiB blocks; each lane loads its old granule before it stores the new
// one over it (same lane, same address: the load sees the old bytes), so the
// old bytes are read once, by the write itself.  Every thread calls it.
template <uint32_t POLY>
__device__ __forceinline__ uint32_t wg_write_hash_old(uint64_t dst, uint64_t src, uint64_t len, uint64_t olen,
                                                      const StepLds& lj, const uint32_t* lc, const PolyTables* T,
                                                      uint32_t* s_part) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const uint64_t d1 = dst + len, o1 = dst + olen;
  const uint64_t vs = dst & ~uint64_t(15);
  const uint64_t nb = (d1 - vs + kBlockBytes - 1) / kBlockBytes;
  const uint64_t bpw = (nb + kWaves - 1) / kWaves;
  const uint64_t b0 = (uint64_t)wave * bpw;
  const uint64_t b1 = b0 + bpw < nb ? b0 + bpw : nb;
  uint32_t val = 0;
  if (b0 < b1) {  // wave-uniform
    constexpr int U = 4;
    Streams st;
    for (uint64_t b = b0; b < b1; b += U) {
      uint4 o[U];
      u32x4 p[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {  // the loads of U blocks first: U KiB per wave in flight
        const uint64_t g = vs + (b + k) * kBlockBytes + 16 * (uint64_t)lane;
        const bool live = b + k < b1;
        o[k] = live ? gload16_masked(g, dst, o1) : make_uint4(0, 0, 0, 0);
        p[k] = live && g >= dst && g + 16 <= d1 ? ld16_unaligned(src + (g - dst)) : u32x4{0, 0, 0, 0};
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if (b + k >= b1) break;  // wave-uniform
        const uint64_t g = vs + (b + k) * kBlockBytes + 16 * (uint64_t)lane;
        st.step(o[k], lj);
        if (g >= dst && g + 16 <= d1) {
          st16(g, p[k]);
        } else if (g < d1 && g + 16 > dst) {  // the partial first / last granule of the write
          const uint64_t lo = g > dst ? g : dst, hi = g + 16 < d1 ? g + 16 : d1;
          for (uint64_t q = lo; q < hi; ++q)
            *reinterpret_cast<uint8_t*>(q) = *reinterpret_cast<const uint8_t*>(src + (q - dst));
        }
      }
    }
    const uint32_t v = fold_streams(st, lc, lane);  // lin(old bytes of this run) at the run's end
    const uint64_t vend = vs + b1 * kBlockBytes;
    const uint32_t f = xpow_pair<POLY>(8 * ((int64_t)o1 - (int64_t)vend), 0, lane, T);
    val = gf_mul(__builtin_amdgcn_readfirstlane(v), __builtin_amdgcn_readlane(f, 0), POLY);
  }
  return wg_xor(val, s_part);
}

}  // namespace hf3fs_crc
