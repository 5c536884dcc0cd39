// scripts/probe_copy_ceiling.hip -- the part's store / copy / read ceilings at d3's byte
// count (probe, not product code; VERDICT r05 "next" item 1).
//
// MI355X_MICROARCH.md:36 quotes 6.29 TB/s for a float4 copy and :332 6.0-6.2 TB/s for
// plain stores; the d3 apply (k_update_apply) moves its 4.58 GB at ~5.0 TB/s read +
// write.  This probe times, interleaved in one process on one pair of 2.25 GiB
// buffers, contiguous copies / stores / reads in several shapes:
//   flat<U,W>   persistent grid-stride copy, W waves per CU, U x 16 B loads in flight
//               per lane before the U stores
//   oneshot     the textbook float4 copy: one thread per 16-B granule, no loop
//   tile<U,W>   persistent, each workgroup copies a contiguous 64 KiB tile at a time
//   store<U,W>  16-B stores only;  read<U,W>  16-B loads only (xor-reduced)
//   memcpy      hipMemcpyAsync device to device
// each with cached or non-temporal loads / stores.  Rates are bytes moved (read +
// write for copies) / median event time of 9 launches.  Every copy leg is checked.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probe_copy_ceiling.hip -o build/probe_copy_ceiling
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                        \
    }                                                                                 \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_flat(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t ng) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; g + (U - 1) * stride < ng; g += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = ld<NTL>(s + g + k * stride);
#pragma unroll
    for (int k = 0; k < U; ++k) st<NTS>(d + g + k * stride, v[k]);
  }
  for (; g < ng; g += stride) st<NTS>(d + g, ld<NTL>(s + g));
}

template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_oneshot(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t ng) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g < ng) st<NTS>(d + g, ld<NTL>(s + g));
}

// contiguous tiles of 4096 granules (64 KiB) per workgroup, static order
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_tile(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t ng) {
  constexpr uint64_t kTile = 4096;
  const uint64_t ntiles = ng / kTile;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const u32x4* ss = s + t * kTile;
    u32x4* dd = d + t * kTile;
    for (uint32_t g = threadIdx.x; g < kTile; g += U * 256) {
      u32x4 v[U];
#pragma unroll
      for (int k = 0; k < U; ++k) v[k] = ld<NTL>(ss + g + k * 256);
#pragma unroll
      for (int k = 0; k < U; ++k) st<NTS>(dd + g + k * 256, v[k]);
    }
  }
}

template <int U, bool NTS>
__global__ __launch_bounds__(256) void k_store(u32x4* __restrict__ d, uint64_t ng, uint32_t seed) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const u32x4 v = {seed, seed ^ 1u, seed ^ 2u, (uint32_t)g};
  for (; g + (U - 1) * stride < ng; g += U * stride) {
#pragma unroll
    for (int k = 0; k < U; ++k) st<NTS>(d + g + k * stride, v);
  }
  for (; g < ng; g += stride) st<NTS>(d + g, v);
}

template <int U, bool NTL>
__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ s, uint64_t ng, uint32_t* sink) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (; g + (U - 1) * stride < ng; g += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = ld<NTL>(s + g + k * stride);
#pragma unroll
    for (int k = 0; k < U; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  for (; g < ng; g += stride) {
    const u32x4 v = ld<NTL>(s + g);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;
}

// one-shot with U granules per thread: each workgroup copies 256*U contiguous granules, then exits
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_oneshot_u(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t ng) {
  const uint64_t g0 = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int k = 0; k < U; ++k)
    if (g0 + k * 256 < ng) v[k] = ld<NTL>(s + g0 + k * 256);
#pragma unroll
  for (int k = 0; k < U; ++k)
    if (g0 + k * 256 < ng) st<NTS>(d + g0 + k * 256, v[k]);
}
template <bool NTS>
__global__ __launch_bounds__(256) void k_store_oneshot(u32x4* __restrict__ d, uint64_t ng, uint32_t seed) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g < ng) st<NTS>(d + g, u32x4{seed, seed ^ 1u, seed ^ 2u, (uint32_t)g});
}
template <bool NTL>
__global__ __launch_bounds__(256) void k_read_oneshot(const u32x4* __restrict__ s, uint64_t ng, uint32_t* sink) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g < ng) {
    const u32x4 v = ld<NTL>(s + g);
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9e3779b9u) sink[threadIdx.x] = 1;
  }
}
// persistent, tickets over contiguous pieces of PG granules in stream order (tight front)
template <int PG, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_ticket(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t ng,
                                                uint32_t* q) {
  __shared__ uint32_t t;
  uint64_t p = blockIdx.x;
  const uint64_t np = ng / PG;
  while (p < np) {
    constexpr int U = PG / 256;
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = ld<NTL>(s + p * PG + threadIdx.x + k * 256);
#pragma unroll
    for (int k = 0; k < U; ++k) st<NTS>(d + p * PG + threadIdx.x + k * 256, v[k]);
    __syncthreads();
    if (threadIdx.x == 0) t = atomicAdd(q, 1u);
    __syncthreads();
    p = gridDim.x + (uint64_t)t;
  }
}

// ---- ragged (d3-shaped) copies: 4096 ranges of U[64 KiB, 1 MiB] from 1 MiB-strided payloads to
// byte offsets of 4 MiB chunks ----
struct Range {
  uint64_t dst, src, len;
};
typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(1)));
template <bool NT>
__device__ __forceinline__ u32x4 ldu(uint64_t a) {
  typedef __attribute__((address_space(1))) const u32x4u gq;
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<gq*>(a));
  return *reinterpret_cast<gq*>(a);
}
template <bool NT>
__device__ __forceinline__ void sta(uint64_t a, u32x4 v) {
  st<NT>(reinterpret_cast<u32x4*>(a), v);
}
// bytes [a, e) of range R (dst addresses), 256 threads, granules strided by 256
template <bool NTL, bool NTS>
__device__ __forceinline__ void copy_piece(const Range& R, uint64_t a, uint64_t e) {
  const uint32_t tid = threadIdx.x;
  const uint64_t ga = (a + 15) & ~uint64_t(15), ge = e & ~uint64_t(15);
  const int64_t so = (int64_t)R.src - (int64_t)R.dst;
  if (ga >= ge) {  // tiny piece: bytes
    if (tid < e - a) *reinterpret_cast<uint8_t*>(a + tid) = *reinterpret_cast<const uint8_t*>(a + tid + so);
    return;
  }
  const uint64_t nh = ga - a, nt = e - ge;
  if (tid < nh + nt) {
    const uint64_t b = tid < nh ? a + tid : ge + (tid - nh);
    *reinterpret_cast<uint8_t*>(b) = *reinterpret_cast<const uint8_t*>(b + so);
  }
  const uint64_t ng = (ge - ga) / 16;
  for (uint64_t g = tid; g < ng; g += 256) sta<NTS>(ga + g * 16, ldu<NTL>(ga + g * 16 + so));
}
// one workgroup per P-aligned destination piece, one-shot grid
template <uint32_t P, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_ragged_oneshot(const Range* __restrict__ rs, const uint32_t* __restrict__ ptab,
                                                        const uint32_t* __restrict__ first) {
  const uint32_t r = ptab[blockIdx.x];
  const Range R = rs[r];
  const uint64_t k = blockIdx.x - first[r];
  const uint64_t base = (R.dst & ~uint64_t(P - 1)) + k * P;
  const uint64_t a = base > R.dst ? base : R.dst, e = base + P < R.dst + R.len ? base + P : R.dst + R.len;
  copy_piece<NTL, NTS>(R, a, e);
}
// the library's current shape: 8 pieces of >= 64 KiB per range, tickets, 2048 workgroups,
// U = 4 granules per thread per step
template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_ragged_tasks(const Range* __restrict__ tasks, uint64_t n, uint32_t* q) {
  __shared__ uint32_t t;
  uint64_t i = blockIdx.x;
  while (i < n) {
    const Range R = tasks[i];
    const uint64_t a = R.dst, e = R.dst + R.len;
    const uint64_t ga = (a + 15) & ~uint64_t(15), ge = e & ~uint64_t(15);
    const int64_t so = (int64_t)R.src - (int64_t)R.dst;
    const uint64_t nh = ga - a, nt = e - ge;
    if (threadIdx.x < nh + nt) {
      const uint64_t b = threadIdx.x < nh ? a + threadIdx.x : ge + (threadIdx.x - nh);
      *reinterpret_cast<uint8_t*>(b) = *reinterpret_cast<const uint8_t*>(b + so);
    }
    const uint64_t ng = (ge - ga) / 16;
    uint64_t g = threadIdx.x;
    for (; g + 768 < ng; g += 1024) {
      u32x4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = ldu<NTL>(ga + (g + k * 256) * 16 + so);
#pragma unroll
      for (int k = 0; k < 4; ++k) sta<NTS>(ga + (g + k * 256) * 16, v[k]);
    }
    for (; g < ng; g += 256) sta<NTS>(ga + g * 16, ldu<NTL>(ga + g * 16 + so));
    __syncthreads();
    if (threadIdx.x == 0) t = atomicAdd(q, 1u);
    __syncthreads();
    i = gridDim.x + (uint64_t)t;
  }
}

// one-shot u1 with LDS_KB of LDS per workgroup (caps resident workgroups per CU)
template <int LDS_KB, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_oneshot_lds(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t ng) {
  __shared__ uint32_t pad[LDS_KB * 256];
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g < ng) {
    u32x4 v = ld<NTL>(s + g);
    if (v.x == 0x12345678u && v.y == 0x9abcdef0u) pad[threadIdx.x] = v.z;  // keeps the LDS allocation
    st<NTS>(d + g, v);
  }
}
// ragged tasks with U granules per thread, loads of a step before its stores
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_ragged_tasks_u(const Range* __restrict__ tasks, uint64_t n, uint32_t* q) {
  __shared__ uint32_t t;
  uint64_t i = blockIdx.x;
  while (i < n) {
    const Range R = tasks[i];
    const uint64_t a = R.dst, e = R.dst + R.len;
    const uint64_t ga = (a + 15) & ~uint64_t(15), ge = e & ~uint64_t(15);
    const int64_t so = (int64_t)R.src - (int64_t)R.dst;
    const uint64_t nh = ga - a, nt = e - ge;
    if (threadIdx.x < nh + nt) {
      const uint64_t b = threadIdx.x < nh ? a + threadIdx.x : ge + (threadIdx.x - nh);
      *reinterpret_cast<uint8_t*>(b) = *reinterpret_cast<const uint8_t*>(b + so);
    }
    const uint64_t ng = (ge - ga) / 16;
    uint64_t g = threadIdx.x;
    for (; g + (U - 1) * 256 < ng; g += U * 256) {
      u32x4 v[U];
#pragma unroll
      for (int k = 0; k < U; ++k) v[k] = ldu<NTL>(ga + (g + k * 256) * 16 + so);
#pragma unroll
      for (int k = 0; k < U; ++k) sta<NTS>(ga + (g + k * 256) * 16, v[k]);
    }
    for (; g < ng; g += 256) sta<NTS>(ga + g * 16, ldu<NTL>(ga + g * 16 + so));
    __syncthreads();
    if (threadIdx.x == 0) t = atomicAdd(q, 1u);
    __syncthreads();
    i = gridDim.x + (uint64_t)t;
  }
}
// ragged, static: workgroup w takes tasks w, w + G, ...
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_ragged_static_u(const Range* __restrict__ tasks, uint64_t n) {
  for (uint64_t i = blockIdx.x; i < n; i += gridDim.x) {
    const Range R = tasks[i];
    const uint64_t a = R.dst, e = R.dst + R.len;
    const uint64_t ga = (a + 15) & ~uint64_t(15), ge = e & ~uint64_t(15);
    const int64_t so = (int64_t)R.src - (int64_t)R.dst;
    const uint64_t nh = ga - a, nt = e - ge;
    if (threadIdx.x < nh + nt) {
      const uint64_t b = threadIdx.x < nh ? a + threadIdx.x : ge + (threadIdx.x - nh);
      *reinterpret_cast<uint8_t*>(b) = *reinterpret_cast<const uint8_t*>(b + so);
    }
    const uint64_t ng = (ge - ga) / 16;
    uint64_t g = threadIdx.x;
    for (; g + (U - 1) * 256 < ng; g += U * 256) {
      u32x4 v[U];
#pragma unroll
      for (int k = 0; k < U; ++k) v[k] = ldu<NTL>(ga + (g + k * 256) * 16 + so);
#pragma unroll
      for (int k = 0; k < U; ++k) sta<NTS>(ga + (g + k * 256) * 16, v[k]);
    }
    for (; g < ng; g += 256) sta<NTS>(ga + g * 16, ldu<NTL>(ga + g * 16 + so));
  }
}
// one-shot with a 16-byte piece descriptor {dst_begin | (len << 48), src - dst}
template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_ragged_desc(const ulonglong2* __restrict__ desc, uint32_t np) {
  if (blockIdx.x >= np) return;
  const ulonglong2 D = desc[blockIdx.x];
  const uint64_t a = D.x & ((1ull << 48) - 1), e = a + (D.x >> 48);
  Range R{0, D.y, 0};  // copy_piece uses src - dst only
  R.src = D.y;
  R.dst = 0;
  copy_piece<NTL, NTS>(R, a, e);
}
__global__ void k_empty(uint32_t* sink) {
  if (blockIdx.x == 0xffffffffu) sink[0] = 1;
}
// every range's source bytes and the destination bytes it overwrites, nt loads
__global__ __launch_bounds__(256) void k_preread(const Range* __restrict__ rs, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t j = blockIdx.x; j < 2 * n; j += gridDim.x) {
    const Range R = rs[j >> 1];
    const uint64_t b = (j & 1) ? R.dst : R.src;
    const uint64_t a0 = b & ~uint64_t(15), a1 = (b + R.len + 15) & ~uint64_t(15);
    for (uint64_t g = a0 + threadIdx.x * 16; g < a1; g += 256 * 16) {
      const u32x4 v = ld<true>(reinterpret_cast<const u32x4*>(g));
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;
}


// The library's one-shot apply body (update_kernels.hip k_update_apply_one_shot) with its
// features switchable, to find what separates it from k_ragged_oneshot:
//   VERD: a verdict word per range loaded beside the data (pre_out), stores only if it matches
//   CNT:  the piece count loaded from memory (prep's atomic counter), not the launch size
//   LOOP: the grid-stride loop (the next entry loaded before the count is checked)
struct ARec {  // ApplyTask: dst, src, len, io, wval, first | verify << 31
  uint64_t dst, src;
  uint32_t len, io, wval, first_v;
};
template <bool VERD, bool CNT, bool LOOP>
__global__ __launch_bounds__(256) void k_libshape(const ARec* __restrict__ recs, const uint32_t* __restrict__ ptab,
                                                  const uint32_t* __restrict__ verdict, const uint64_t* cnt,
                                                  uint64_t np_host, uint64_t cap, uint64_t nrec) {
  constexpr uint64_t P = 8192;
  const uint32_t tid = threadIdx.x;
  const uint64_t npieces = CNT ? *cnt : np_host;
  for (uint64_t b = blockIdx.x; b < cap; b += gridDim.x) {
    const uint32_t r = ptab[b];
    if (b >= npieces) break;
    const ARec R = recs[r < nrec ? r : 0];
    const uint32_t first = R.first_v & 0x7fffffffu;
    const uint32_t got = VERD ? verdict[R.io] : R.wval;
    const uint64_t cut = (R.dst & ~(P - 1)) + ((b - first) << 13);
    const uint64_t a = cut > R.dst ? cut : R.dst, e = cut + P < R.dst + R.len ? cut + P : R.dst + R.len;
    const int64_t so = (int64_t)(R.src - R.dst);
    const uint64_t ga = (a + 15) & ~uint64_t(15), ge = e & ~uint64_t(15);
    uint64_t bb = 0;
    bool byte = false;
    if (ga >= ge) {
      byte = tid < e - a;
      bb = a + tid;
    } else {
      const uint64_t nh = ga - a, nt = e - ge;
      byte = tid < nh + nt;
      bb = tid < nh ? a + tid : ge + (tid - nh);
    }
    const uint8_t x = byte && R.src ? *reinterpret_cast<const uint8_t*>(bb + so) : 0;
    const uint64_t ng = ge > ga ? (ge - ga) >> 4 : 0;
    u32x4 v = tid < ng && R.src ? ldu<false>(ga + tid * 16 + so) : u32x4{0, 0, 0, 0};
    if (got != R.wval) continue;
    if (byte) *reinterpret_cast<uint8_t*>(bb) = x;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint64_t g = tid + k * 256;
      if (k) v = g < ng && R.src ? ldu<false>(ga + g * 16 + so) : u32x4{0, 0, 0, 0};
      if (g < ng) sta<true>(ga + g * 16, v);
    }
    if (!LOOP) break;
  }
}
__global__ void k_count(uint64_t* c, uint64_t v) {  // the count, written by an atomic as prep does
  if (threadIdx.x == 0 && blockIdx.x == 0) atomicAdd((unsigned long long*)c, (unsigned long long)v);
}
__global__ void k_check_ranges(const Range* __restrict__ rs, uint64_t n, unsigned long long* bad) {
  for (uint64_t r = blockIdx.x; r < n; r += gridDim.x) {
    const Range R = rs[r];
    unsigned long long b = 0;
    for (uint64_t x = threadIdx.x; x < R.len; x += blockDim.x)
      b += reinterpret_cast<const uint8_t*>(R.dst)[x] != reinterpret_cast<const uint8_t*>(R.src)[x];
    if (b) atomicAdd(bad, b);
  }
}

__global__ void k_fill(uint64_t* p, uint64_t n, uint64_t seed) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + i * 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    p[i] = z ^ (z >> 31);
  }
}

__global__ void k_cmp(const uint64_t* a, const uint64_t* b, uint64_t n, unsigned long long* bad) {
  unsigned long long c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    c += a[i] != b[i];
  if (c) atomicAdd(bad, c);
}

struct Leg {
  std::string name;
  int kind;  // 0 copy, 1 store, 2 read, 3 ragged copy, 4 empty
  std::function<void()> run;
};

static void time_legs(std::vector<Leg>& legs, int reps, double bytes, std::function<void()> before = nullptr,
                      const char* tag = "") {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 20; ++i) legs[0].run();  // warm
  CK(hipDeviceSynchronize());
  std::vector<std::vector<float>> ms(legs.size());
  for (int r = 0; r < reps; ++r)
    for (size_t i = 0; i < legs.size(); ++i) {
      if (before) before();
      CK(hipEventRecord(e0, 0));
      legs[i].run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[i].push_back(t);
    }
  static const char* kinds[] = {"copy", "store", "read", "ragged copy", "empty"};
  for (size_t i = 0; i < legs.size(); ++i) {
    std::vector<float> x = ms[i];
    std::sort(x.begin(), x.end());
    const double m = x[x.size() / 2];
    const double moved = legs[i].kind == 0 || legs[i].kind == 3 ? 2.0 * bytes : legs[i].kind == 4 ? 0.0 : bytes;
    printf("{\"leg\":\"%s%s\",\"kind\":\"%s\",\"bytes\":%.0f,\"ms\":%.4f,\"tbs\":%.3f,\"best_tbs\":%.3f}\n",
           legs[i].name.c_str(), tag, kinds[legs[i].kind], bytes, m, moved / m / 1e9, moved / x[0] / 1e9);
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 9;
  const std::string sec = argc > 2 ? argv[2] : "flat,ragged";
  auto want = [&](const char* x) { return sec.find(x) != std::string::npos; };
  const uint64_t bytes = 2304ull << 20;
  const uint64_t ng = bytes / 16;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const uint32_t cus = prop.multiProcessorCount;
  u32x4 *src, *dst;
  uint32_t *sink, *q;
  unsigned long long* bad;
  CK(hipMalloc(&src, bytes));
  CK(hipMalloc(&dst, bytes));
  CK(hipMalloc(&sink, 4096));
  CK(hipMalloc(&bad, 8));
  CK(hipMalloc(&q, 64));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)src, bytes / 8, 7ull);
  CK(hipDeviceSynchronize());
  printf("{\"probe\":\"copy_ceiling\",\"cus\":%u,\"bytes\":%llu,\"reps\":%d,\"sections\":\"%s\"}\n", cus,
         (unsigned long long)bytes, reps, sec.c_str());
  auto grid_w = [&](int waves) { return dim3(cus * waves / 4 ? cus * waves / 4 : 1); };
  auto check_flat = [&](std::vector<Leg>& legs) {
    for (const Leg& l : legs) {
      if (l.kind != 0) continue;
      CK(hipMemsetAsync(dst, 0, bytes, 0));
      l.run();
      CK(hipMemsetAsync(bad, 0, 8, 0));
      hipLaunchKernelGGL(k_cmp, dim3(4096), dim3(256), 0, 0, (const uint64_t*)src, (const uint64_t*)dst,
                         (ng / 4096) * 4096 * 2, bad);
      unsigned long long b = 0;
      CK(hipMemcpy(&b, bad, 8, hipMemcpyDeviceToHost));
      if (b) {
        printf("{\"check\":\"%s\",\"bad_words\":%llu}\n", l.name.c_str(), b);
        exit(1);
      }
    }
    printf("{\"check\":\"copy legs\",\"bad_words\":0}\n");
  };
#define FLAT(U, W, L, S)                                                                                      \
  legs.push_back({"flat_u" #U "_w" #W "_l" #L "_s" #S, 0, [&, g = grid_w(W)] {                                \
                    hipLaunchKernelGGL((k_flat<U, (bool)L, (bool)S>), g, dim3(256), 0, 0, src, dst, ng);    \
                  }})
#define ONESHOT_LDS(K)                                                                                        \
  legs.push_back({"oneshot_lds" #K "k_l1_s1", 0, [&] {                                                        \
                    hipLaunchKernelGGL((k_oneshot_lds<K, true, true>), dim3((ng + 255) / 256), dim3(256), 0, 0, \
                                       src, dst, ng);                                                         \
                  }})
  if (want("flat")) {
    std::vector<Leg> legs;
    legs.push_back({"oneshot_l1_s1", 0, [&] {
                      hipLaunchKernelGGL((k_oneshot<true, true>), dim3((ng + 255) / 256), dim3(256), 0, 0, src, dst, ng);
                    }});
    legs.push_back({"oneshot_l0_s0", 0, [&] {
                      hipLaunchKernelGGL((k_oneshot<false, false>), dim3((ng + 255) / 256), dim3(256), 0, 0, src, dst, ng);
                    }});
    ONESHOT_LDS(1);
    ONESHOT_LDS(20);
    ONESHOT_LDS(40);
    ONESHOT_LDS(80);
    FLAT(1, 4, 1, 1);
    FLAT(2, 4, 1, 1);
    FLAT(4, 4, 1, 1);
    FLAT(1, 8, 1, 1);
    FLAT(2, 8, 1, 1);
    FLAT(4, 8, 1, 1);
    FLAT(1, 16, 1, 1);
    FLAT(2, 16, 1, 1);
    FLAT(1, 4, 0, 0);
    FLAT(2, 4, 0, 0);
    FLAT(1, 8, 0, 0);
    FLAT(4, 8, 0, 0);
    legs.push_back({"store_oneshot_s0", 1, [&] {
                      hipLaunchKernelGGL((k_store_oneshot<false>), dim3((ng + 255) / 256), dim3(256), 0, 0, dst, ng, 3u);
                    }});
    legs.push_back({"read_oneshot_l1", 2, [&] {
                      hipLaunchKernelGGL((k_read_oneshot<true>), dim3((ng + 255) / 256), dim3(256), 0, 0, src, ng, sink);
                    }});
    legs.push_back({"empty_1M_wg", 4, [&] { hipLaunchKernelGGL(k_empty, dim3(1u << 20), dim3(256), 0, 0, sink); }});
    legs.push_back({"empty_4M_wg", 4, [&] { hipLaunchKernelGGL(k_empty, dim3(4u << 20), dim3(256), 0, 0, sink); }});
    check_flat(legs);
    time_legs(legs, reps, (double)bytes);
  }

  if (want("ragged")) {
    const uint64_t n = 4096, chunk = 4ull << 20, pay = 1ull << 20;
    uint8_t *chunks, *payload;
    CK(hipMalloc(&chunks, n * chunk));
    CK(hipMalloc(&payload, n * pay));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)payload, n * pay / 8, 11ull);
    std::mt19937_64 rng(3);
    std::vector<Range> rs(n);
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i) {
      const uint64_t len = (64 << 10) + rng() % ((1 << 20) - (64 << 10) + 1);
      const uint64_t off = rng() % (chunk - len + 1);
      rs[i] = {(uint64_t)chunks + i * chunk + off, (uint64_t)payload + i * pay, len};
      total += len;
    }
    // the library's task cut: 8 pieces of >= 64 KiB, 16-aligned on the destination
    std::vector<Range> tasks;
    for (const Range& x : rs) {
      const uint64_t even = ((x.len + 7) / 8 + 15) & ~uint64_t(15);
      const uint64_t ps = std::max<uint64_t>(even, 64 << 10), h = x.dst & 15;
      for (uint64_t j = 0;; ++j) {
        const uint64_t a = j ? j * ps - h : 0, b = std::min(x.len, (j + 1) * ps - h);
        if (a >= x.len) break;
        if (a < b) tasks.push_back({x.dst + a, x.src + a, b - a});
      }
    }
    Range *d_rs, *d_tasks;
    CK(hipMalloc(&d_rs, n * sizeof(Range)));
    CK(hipMalloc(&d_tasks, tasks.size() * sizeof(Range)));
    CK(hipMemcpy(d_rs, rs.data(), n * sizeof(Range), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_tasks, tasks.data(), tasks.size() * sizeof(Range), hipMemcpyHostToDevice));
    struct PT {
      uint32_t P;
      uint32_t *ptab, *first;
      ulonglong2* desc;
      uint32_t np;
    };
    std::vector<PT> pts;
    for (uint32_t P : {4096u, 8192u, 16384u}) {
      std::vector<uint32_t> ptab, first(n);
      std::vector<ulonglong2> desc;
      for (uint64_t r = 0; r < n; ++r) {
        first[r] = (uint32_t)ptab.size();
        const uint64_t a0 = rs[r].dst & ~uint64_t(P - 1), e = rs[r].dst + rs[r].len;
        for (uint64_t b = a0; b < e; b += P) {
          ptab.push_back((uint32_t)r);
          const uint64_t a = std::max(b, rs[r].dst), z = std::min(b + P, e);
          desc.push_back({a | ((z - a) << 48), rs[r].src - rs[r].dst});
        }
      }
      PT pt{P, nullptr, nullptr, nullptr, (uint32_t)ptab.size()};
      CK(hipMalloc(&pt.ptab, ptab.size() * 4));
      CK(hipMalloc(&pt.first, n * 4));
      CK(hipMalloc(&pt.desc, desc.size() * 16));
      CK(hipMemcpy(pt.ptab, ptab.data(), ptab.size() * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(pt.first, first.data(), n * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(pt.desc, desc.data(), desc.size() * 16, hipMemcpyHostToDevice));
      pts.push_back(pt);
    }
    printf("{\"ragged\":{\"ranges\":%llu,\"bytes\":%llu,\"tasks\":%zu,\"pieces_4k\":%u,\"pieces_8k\":%u}}\n",
           (unsigned long long)n, (unsigned long long)total, tasks.size(), pts[0].np, pts[1].np);
    std::vector<Leg> rl;
#define RTASK(U, WG, L, S)                                                                                     \
  rl.push_back({"tasks8_u" #U "_wg" #WG "_l" #L "_s" #S, 3, [&] {                                              \
                  CK(hipMemsetAsync(q, 0, 4, 0));                                                              \
                  hipLaunchKernelGGL((k_ragged_tasks_u<U, (bool)L, (bool)S>), dim3(cus * WG), dim3(256), 0, 0, \
                                     d_tasks, (uint64_t)tasks.size(), q);                                      \
                }})
#define RSTAT(U, WG, L, S)                                                                                      \
  rl.push_back({"static8_u" #U "_wg" #WG "_l" #L "_s" #S, 3, [&] {                                              \
                  hipLaunchKernelGGL((k_ragged_static_u<U, (bool)L, (bool)S>), dim3(cus * WG), dim3(256), 0, 0, \
                                     d_tasks, (uint64_t)tasks.size());                                          \
                }})
#define RDESC(I, P, OVER)                                                                                        \
  rl.push_back({"desc_p" #P "_over" #OVER "_l1_s1", 3, [&, ii = I] {                                            \
                  hipLaunchKernelGGL((k_ragged_desc<true, true>), dim3(pts[ii].np * OVER), dim3(256), 0, 0,       \
                                     pts[ii].desc, pts[ii].np);                                                  \
                }})
#define ROS(I, P, L, S)                                                                                       \
  rl.push_back({"table_p" #P "_l" #L "_s" #S, 3, [&, ii = I] {                                                \
                  hipLaunchKernelGGL((k_ragged_oneshot<P, (bool)L, (bool)S>), dim3(pts[ii].np), dim3(256), 0, 0, \
                                     d_rs, pts[ii].ptab, pts[ii].first);                                      \
                }})
    RTASK(4, 8, 1, 1);  // the library's shape (apply: copy_range_hw U = 4, nt stores)
    RTASK(4, 8, 0, 1);
    RTASK(1, 8, 1, 1);
    RTASK(2, 8, 1, 1);
    RTASK(1, 4, 1, 1);
    RTASK(2, 4, 1, 1);
    RTASK(4, 4, 1, 1);
    RTASK(1, 2, 1, 1);
    RTASK(2, 2, 1, 1);
    RTASK(4, 2, 1, 1);
    RSTAT(1, 4, 1, 1);
    RSTAT(2, 4, 1, 1);
    RSTAT(1, 8, 1, 1);
    ROS(1, 8192, 1, 1);
    // library-shaped one-shot (k_libshape): records, verdicts, the count in memory
    std::vector<ARec> arec(n);
    for (uint64_t r = 0; r < n; ++r)
      arec[r] = ARec{rs[r].dst, rs[r].src, (uint32_t)rs[r].len, (uint32_t)r, 0x1234u + (uint32_t)r, 0};
    {
      std::vector<uint32_t> first(n);
      CK(hipMemcpy(first.data(), pts[1].first, n * 4, hipMemcpyDeviceToHost));
      for (uint64_t r = 0; r < n; ++r) arec[r].first_v = first[r] | (1u << 31);
    }
    ARec* d_arec;
    uint32_t* d_verd;
    uint64_t* d_cnt;
    CK(hipMalloc(&d_arec, n * sizeof(ARec)));
    CK(hipMalloc(&d_verd, n * 4));
    CK(hipMalloc(&d_cnt, 8));
    CK(hipMemcpy(d_arec, arec.data(), n * sizeof(ARec), hipMemcpyHostToDevice));
    {
      std::vector<uint32_t> vv(n);
      for (uint64_t r = 0; r < n; ++r) vv[r] = 0x1234u + (uint32_t)r;
      CK(hipMemcpy(d_verd, vv.data(), n * 4, hipMemcpyHostToDevice));
    }
    const uint64_t np8 = pts[1].np, cap8 = np8 + np8 / 16;
    uint32_t* ptab8;  // the 8 KiB table with spare capacity (the library's ptab_cap)
    CK(hipMalloc(&ptab8, cap8 * 4));
    CK(hipMemset(ptab8, 0xff, cap8 * 4));
    CK(hipMemcpy(ptab8, pts[1].ptab, np8 * 4, hipMemcpyDeviceToDevice));
#define LIB(V, C, LP, OVER)                                                                                   \
  rl.push_back({"lib_v" #V "_c" #C "_loop" #LP "_over" #OVER, 3, [&] {                                         \
                  if (C) {                                                                                     \
                    CK(hipMemsetAsync(d_cnt, 0, 8, 0));                                                        \
                    hipLaunchKernelGGL(k_count, dim3(1), dim3(64), 0, 0, d_cnt, np8);                          \
                  }                                                                                            \
                  hipLaunchKernelGGL((k_libshape<(bool)V, (bool)C, (bool)LP>), dim3(np8 + np8 * OVER / 100), dim3(256), \
                                     0, 0, d_arec, ptab8, d_verd, d_cnt, np8, cap8, n);                        \
                }})
    // the same table with the ranges' 64-IO groups in a shuffled order (prep's waves reserve
    // their pieces in arrival order), records and first pieces rebuilt for it
    uint32_t* ptab8p;
    ARec* d_arecp;
    {
      std::vector<uint32_t> order(n / 64);
      for (uint32_t g = 0; g < n / 64; ++g) order[g] = g;
      std::shuffle(order.begin(), order.end(), std::mt19937_64(11));
      std::vector<uint32_t> pt;
      std::vector<ARec> ar = arec;
      for (uint32_t g : order)
        for (uint32_t r = g * 64; r < g * 64 + 64; ++r) {
          ar[r].first_v = (uint32_t)pt.size() | (1u << 31);
          const uint64_t a0 = rs[r].dst & ~uint64_t(8191), e = rs[r].dst + rs[r].len;
          for (uint64_t b = a0; b < e; b += 8192) pt.push_back(r);
        }
      CK(hipMalloc(&ptab8p, cap8 * 4));
      CK(hipMemset(ptab8p, 0xff, cap8 * 4));
      CK(hipMemcpy(ptab8p, pt.data(), pt.size() * 4, hipMemcpyHostToDevice));
      CK(hipMalloc(&d_arecp, n * sizeof(ARec)));
      CK(hipMemcpy(d_arecp, ar.data(), n * sizeof(ARec), hipMemcpyHostToDevice));
    }
    rl.push_back({"lib_shuffled_groups", 3, [&] {
                    hipLaunchKernelGGL((k_libshape<true, false, true>), dim3(np8), dim3(256), 0, 0, d_arecp, ptab8p,
                                       d_verd, d_cnt, np8, cap8, n);
                  }});
    LIB(0, 0, 0, 0);
    LIB(1, 0, 0, 0);
    LIB(0, 1, 0, 0);
    LIB(0, 0, 1, 0);
    LIB(0, 0, 0, 3);
    LIB(1, 1, 1, 3);
    RDESC(0, 4096, 1);
    RDESC(1, 8192, 1);
    RDESC(1, 8192, 4);
    RDESC(2, 16384, 1);
    for (const Leg& l : rl) {
      hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)chunks, n * chunk / 8, 99ull);
      l.run();
      CK(hipMemsetAsync(bad, 0, 8, 0));
      hipLaunchKernelGGL(k_check_ranges, dim3(4096), dim3(256), 0, 0, d_rs, n, bad);
      unsigned long long b = 0;
      CK(hipMemcpy(&b, bad, 8, hipMemcpyDeviceToHost));
      if (b) {
        printf("{\"check\":\"%s\",\"bad_bytes\":%llu}\n", l.name.c_str(), b);
        return 1;
      }
    }
    printf("{\"check\":\"ragged legs\",\"bad_bytes\":0}\n");
    time_legs(rl, reps, (double)total);
    // the same legs, each right after a pass that reads every payload and the old bytes under
    // every write (the update pipeline's pre hash, non-temporal loads), untimed
    time_legs(rl, reps, (double)total, [&] {
      hipLaunchKernelGGL(k_preread, dim3(cus * 4), dim3(256), 0, 0, d_rs, n, sink);
    }, "+preread");
  }
  return 0;
}
