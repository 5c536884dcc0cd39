// crc_kernels.hip -- CDNA4 kernels of the chunk-integrity engine (see crc_kernels.h).
#include "crc_kernels.h"

namespace hf3fs_crc {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;

// global_load_dwordx4 (address space 1, not flat: flat loads would also count
// on lgkmcnt and serialise against the LDS table reads).
__device__ __forceinline__ uint4 gload16(uint64_t addr) {
  const u32x4 v = *reinterpret_cast<g_u32x4*>(addr);
  return make_uint4(v.x, v.y, v.z, v.w);
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

// One stream update: (s ^ w) * x^8192 via the lane's private LDS table copy.
__device__ __forceinline__ uint32_t stride_step(uint32_t x, const uint32_t* lj) {
  return lj[(x & 0xffu) << 5] ^ lj[8192 + (((x >> 8) & 0xffu) << 5)] ^ lj[16384 + (((x >> 16) & 0xffu) << 5)] ^
         lj[24576 + ((x >> 24) << 5)];
}

struct Streams {
  uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  __device__ __forceinline__ void step(const uint4& w, const uint32_t* lj) {
    s0 = stride_step(s0 ^ w.x, lj);
    s1 = stride_step(s1 ^ w.y, lj);
    s2 = stride_step(s2 ^ w.z, lj);
    s3 = stride_step(s3 ^ w.w, lj);
  }
};

// Copy the 4 x 256 step table into LDS, 32 replicas per entry (entry e at
// words [32e, 32e+32)): lane l later reads replica l % 32 -> bank l % 32.
__device__ __forceinline__ void fill_lds(uint32_t* lds, const uint32_t* step) {
  for (int e = threadIdx.x; e < 1024; e += blockDim.x) {
    const uint32_t v = step[e];
    const uint4 v4 = make_uint4(v, v, v, v);
    uint4* dst = reinterpret_cast<uint4*>(lds + e * kCopies);
#pragma unroll
    for (int c = 0; c < kCopies / 4; ++c) dst[c] = v4;
  }
  __syncthreads();
}

// Hash bytes [a0, a1) (a1 > a0) with the wave; returns the streams folded to
// V = sum_{l,d} s_{l,d} * x^(8160 - 32(4l+d)) in lane 0, and the virtual end
// vend = (a0 & ~15) + nb * 1024 so that  lin([a0,a1)) * x^(8(vend-a1)) = V * x^-8160.
template <uint32_t POLY>
__device__ __forceinline__ uint32_t hash_range(uint64_t a0, uint64_t a1, const uint32_t* lj, int lane,
                                               uint64_t& vend) {
  constexpr int U = 4;
  const uint64_t vs = a0 & ~uint64_t(15);
  const uint64_t span = a1 - vs;
  const uint64_t nb = (span + kBlockBytes - 1) / kBlockBytes;
  const uint64_t lb = span / kBlockBytes;  // complete blocks counted from vs
  const uint64_t lane_off = (uint64_t)lane * 16;
  Streams st;
  uint64_t b = 0;
  if (a0 != vs) {  // unaligned head: block 0 masked
    st.step(gload16_masked(vs + lane_off, a0, a1), lj);
    b = 1;
  }
  const uint64_t nfull = lb > b ? lb - b : 0;
  const uint64_t gbase = vs + b * kBlockBytes + lane_off;
  uint64_t g = 0;
  if (nfull >= U) {
    uint4 c0 = gload16(gbase), c1 = gload16(gbase + 1024), c2 = gload16(gbase + 2048), c3 = gload16(gbase + 3072);
    for (g = U; g + U <= nfull; g += U) {
      const uint64_t q = gbase + g * kBlockBytes;
      uint4 n0 = gload16(q), n1 = gload16(q + 1024), n2 = gload16(q + 2048), n3 = gload16(q + 3072);
      st.step(c0, lj);
      st.step(c1, lj);
      st.step(c2, lj);
      st.step(c3, lj);
      c0 = n0;
      c1 = n1;
      c2 = n2;
      c3 = n3;
    }
    st.step(c0, lj);
    st.step(c1, lj);
    st.step(c2, lj);
    st.step(c3, lj);
  }
  for (; g < nfull; ++g) st.step(gload16(gbase + g * kBlockBytes), lj);
  if (lb < nb && lb >= b) st.step(gload16_masked(vs + lb * kBlockBytes + lane_off, a0, a1), lj);
  vend = vs + nb * kBlockBytes;

  // fold: U_l = ((s0 x^32 ^ s1) x^32 ^ s2) x^32 ^ s3, then a shuffle tree
  constexpr uint32_t X32 = xpow_bits(32, POLY);
  uint32_t u = gf_mul(st.s0, X32, POLY) ^ st.s1;
  u = gf_mul(u, X32, POLY) ^ st.s2;
  u = gf_mul(u, X32, POLY) ^ st.s3;
#define HF3FS_TREE_LEVEL(K)                                          \
  {                                                                  \
    constexpr uint32_t XL = xpow_bits(128ull << (K), POLY);          \
    const uint32_t o = __shfl_down(u, 1 << (K), 64);                 \
    if ((lane & ((2 << (K)) - 1)) == 0) u = gf_mul(u, XL, POLY) ^ o; \
  }
  HF3FS_TREE_LEVEL(0)
  HF3FS_TREE_LEVEL(1)
  HF3FS_TREE_LEVEL(2)
  HF3FS_TREE_LEVEL(3)
  HF3FS_TREE_LEVEL(4)
  HF3FS_TREE_LEVEL(5)
#undef HF3FS_TREE_LEVEL
  return u;
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

// Persistent kernel: wave w takes tasks w, w + W, ... of the (range, segment)
// grid.  A task hashes segment `seg` of range i and xors
//   lin(segment) * x^(8 * bytes after it)  [ ^ start * x^(8 len) for seg 0 ]
// into out[i]  (raw(buf, start) = start * x^(8 len) ^ lin(buf)).
template <uint32_t POLY, bool DIRECT, class Src>
__global__ __launch_bounds__(kThreads) void k_crc_ranges(Src src, uint64_t segs, uint64_t seg_bytes,
                                                         uint32_t* __restrict__ out,
                                                         const PolyTables* __restrict__ T) {
  __shared__ uint32_t lds[kLdsWords];
  fill_lds(lds, &T->step[0][0]);
  const int lane = threadIdx.x & 63;
  const uint32_t* lj = lds + (lane & 31);
  const uint64_t ntasks = src.n * segs;
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
  const uint64_t wave = (uint64_t)blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (uint64_t t = wave; t < ntasks; t += nwaves) {
    const uint64_t i = segs == 1 ? t : t / segs;
    const uint64_t seg = t - i * segs;
    const uint64_t len = src.length(i);
    const uint64_t tb = seg * seg_bytes;
    if (seg != 0 && tb >= len) continue;
    if (len == 0) {  // create(type, buf, 0, start) == {type, start}
      if (lane == 0) {
        if (DIRECT)
          out[i] = src.start_of(i);
        else
          atomicXor(out + i, src.start_of(i));
      }
      continue;
    }
    const uint64_t te = len < tb + seg_bytes ? len : tb + seg_bytes;
    const uint64_t base = src.addr(i);
    uint32_t v = 0;
    int64_t ebits = 0;
    if (te > tb) {
      uint64_t vend;
      v = hash_range<POLY>(base + tb, base + te, lj, lane, vend);
      ebits = 8 * (int64_t)(base + len - vend) - 8160;
    }
    const uint32_t f = xpow_pair<POLY>(ebits, 8 * (int64_t)len, lane, T);
    const uint32_t pa = __builtin_amdgcn_readlane(f, 0);
    const uint32_t pb = __builtin_amdgcn_readlane(f, 32);
    const uint32_t vv = __builtin_amdgcn_readfirstlane(v);
    uint32_t val = gf_mul(vv, pa, POLY);
    if (seg == 0) val ^= gf_mul(src.start_of(i), pb, POLY);
    if (lane == 0) {
      if (DIRECT)
        out[i] = val;
      else
        atomicXor(out + i, val);
    }
  }
}

template <class Src>
hipError_t launch_ranges(uint8_t type, const Src& src, const Plan& p, uint32_t* out, const DeviceTables* tabs,
                         hipStream_t s) {
  const bool direct = p.segs == 1;
  if (type == kTypeCrc32) {
    const PolyTables* T = &tabs->poly[1];
    if (direct)
      hipLaunchKernelGGL((k_crc_ranges<kPolyCrc32, true, Src>), dim3(p.grid), dim3(kThreads), 0, s, src, p.segs,
                         p.seg_bytes, out, T);
    else
      hipLaunchKernelGGL((k_crc_ranges<kPolyCrc32, false, Src>), dim3(p.grid), dim3(kThreads), 0, s, src, p.segs,
                         p.seg_bytes, out, T);
  } else {
    const PolyTables* T = &tabs->poly[0];
    if (direct)
      hipLaunchKernelGGL((k_crc_ranges<kPolyCrc32c, true, Src>), dim3(p.grid), dim3(kThreads), 0, s, src, p.segs,
                         p.seg_bytes, out, T);
    else
      hipLaunchKernelGGL((k_crc_ranges<kPolyCrc32c, false, Src>), dim3(p.grid), dim3(kThreads), 0, s, src, p.segs,
                         p.seg_bytes, out, T);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
__global__ void k_compare(const uint32_t* __restrict__ computed, const uint32_t* __restrict__ expected,
                          uint8_t* __restrict__ mismatch, uint32_t* __restrict__ count, uint64_t n) {
  uint32_t local = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t bad = computed[i] != expected[i];
    mismatch[i] = bad;
    local += bad;
  }
  // wave-aggregate then one atomic per wave
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) local += __shfl_xor(local, d, 64);
  if ((threadIdx.x & 63) == 0 && local) atomicAdd(count, local);
}

// ChecksumInfo::combine element-wise: acc = (~acc) * x^(8 len2) ^ crc2.
template <uint32_t POLY>
__global__ void k_combine(uint32_t* __restrict__ acc, const uint32_t* __restrict__ crc2,
                          const uint64_t* __restrict__ len2, uint64_t n, const PolyTables* __restrict__ T) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t l = len2[i];
    if (l == 0) continue;
    uint64_t m = 8 * l;
    uint32_t x = kOne;
    for (int k = 0; m; ++k, m >>= 1)
      if (m & 1) x = gf_mul(x, T->xpow[k], POLY);
    acc[i] = gf_mul(~acc[i], x, POLY) ^ crc2[i];
  }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_fill_synth(uint8_t* __restrict__ dst, uint64_t stride, uint64_t chunk_len, uint64_t n_chunks,
                             uint64_t seed, uint64_t first_chunk_id) {
  const uint64_t wpc = (chunk_len + 7) / 8;
  const uint64_t total = wpc * n_chunks;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t c = t / wpc, w = t - c * wpc;
    const uint64_t v = splitmix64(seed ^ ((first_chunk_id + c) << 32) ^ w);
    uint8_t* p = dst + c * stride + w * 8;
    if (w * 8 + 8 <= chunk_len) {
      *reinterpret_cast<uint64_t*>(p) = v;
    } else {
      for (uint64_t k = 0; w * 8 + k < chunk_len; ++k) p[k] = (uint8_t)(v >> (8 * k));
    }
  }
}

}  // namespace

hipError_t launch_ranges_strided(uint8_t type, const StridedSource& src, const Plan& p, uint32_t* out,
                                 const DeviceTables* tabs, hipStream_t s) {
  return launch_ranges(type, src, p, out, tabs, s);
}
hipError_t launch_ranges_list(uint8_t type, const ListSource& src, const Plan& p, uint32_t* out,
                              const DeviceTables* tabs, hipStream_t s) {
  return launch_ranges(type, src, p, out, tabs, s);
}
hipError_t launch_ranges_arena(uint8_t type, const ArenaSource& src, const Plan& p, uint32_t* out,
                               const DeviceTables* tabs, hipStream_t s) {
  return launch_ranges(type, src, p, out, tabs, s);
}

hipError_t launch_compare(const uint32_t* computed, const uint32_t* expected, uint8_t* mismatch, uint32_t* count,
                          uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t want = (n + 255) / 256;
  const unsigned grid = (unsigned)(want < 4096 ? want : 4096);
  hipLaunchKernelGGL(k_compare, dim3(grid), dim3(256), 0, s, computed, expected, mismatch, count, n);
  return hipGetLastError();
}

hipError_t launch_combine(uint8_t type, uint32_t* acc, const uint32_t* crc2, const uint64_t* len2, uint64_t n,
                          const DeviceTables* tabs, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t want = (n + 255) / 256;
  const unsigned grid = (unsigned)(want < 8192 ? want : 8192);
  if (type == kTypeCrc32)
    hipLaunchKernelGGL(k_combine<kPolyCrc32>, dim3(grid), dim3(256), 0, s, acc, crc2, len2, n, &tabs->poly[1]);
  else
    hipLaunchKernelGGL(k_combine<kPolyCrc32c>, dim3(grid), dim3(256), 0, s, acc, crc2, len2, n, &tabs->poly[0]);
  return hipGetLastError();
}

hipError_t launch_fill_synth(uint8_t* dst, uint64_t stride, uint64_t chunk_len, uint64_t n_chunks, uint64_t seed,
                             uint64_t first_chunk_id, hipStream_t s) {
  const uint64_t total = (chunk_len + 7) / 8 * n_chunks;
  if (total == 0) return hipSuccess;
  const uint64_t want = (total + 255) / 256;
  const unsigned grid = (unsigned)(want < 16384 ? want : 16384);
  hipLaunchKernelGGL(k_fill_synth, dim3(grid), dim3(256), 0, s, dst, stride, chunk_len, n_chunks, seed,
                     first_chunk_id);
  return hipGetLastError();
}

}  // namespace hf3fs_crc
