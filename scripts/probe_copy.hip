// scripts/probe_copy.hip -- what limits the d3 apply copy?  (probe, not product code)
//
// The d3 DELTA batch copies 4096 payloads of U[64 KiB, 1 MiB] bytes (1 MiB-aligned
// sources) to byte-granular offsets of 4 MiB chunks (ChunkReplica.cc:281-292 on
// HBM).  The library's k_update_apply moves them at ~4.8 TB/s (read + write).
// This probe times, in one process on one set of buffers, the same task list
// (8 pieces of >= 64 KiB per range, ticketed to 2048 256-thread workgroups)
// with several copy bodies, a flat aligned copy as the ceiling, and the
// Infinity-Cache reuse of a payload that was just read (the sub-batched
// pre-hash -> apply idea).  Every task-list variant is checked byte-exact.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include scripts/probe_copy.hip -o build/probe_copy
#include "../3fs_amd/csrc/update_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

using namespace hf3fs_crc;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                        \
    }                                                                                 \
  } while (0)

struct Task {
  uint64_t dst, src, len;
};

typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) const u32x4u g_cu32x4u;

template <bool NT = false>
__device__ __forceinline__ u32x4 ldu(uint64_t a) {  // 16 bytes at any byte address: one dwordx4
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<g_cu32x4u*>(a));
  return *reinterpret_cast<g_cu32x4u*>(a);
}

// Body "hw": unaligned source loads straight from the hardware (one dwordx4 per
// granule), aligned 16-byte stores, rows starting at a 1 KiB destination boundary.
// PIPE: the next row's loads are issued before this row's stores.
template <int U, bool NTS, bool PIPE, bool NTL = false>
__device__ void copy_hw(uint64_t dst, uint64_t src, uint64_t len, uint32_t tid, uint32_t nthreads) {
  const uint64_t d0 = dst, d1 = dst + len;
  const uint64_t gfirst = (d0 + 15) & ~uint64_t(15);
  const uint64_t glast = d1 & ~uint64_t(15);
  {
    const uint64_t hend = gfirst < d1 ? gfirst : d1;
    const uint64_t tstart = glast >= gfirst ? glast : d1;
    const uint64_t nh = hend - d0, nt = d1 - tstart;
    if (tid < nh + nt) {
      const uint64_t b = tid < nh ? d0 + tid : tstart + (tid - nh);
      *reinterpret_cast<uint8_t*>(b) = *reinterpret_cast<const uint8_t*>(src + (b - d0));
    }
  }
  if (glast <= gfirst) return;
  const uint64_t ga0 = (gfirst + 1023) & ~uint64_t(1023);
  const uint64_t ga = ga0 < glast ? ga0 : glast;
  if (tid < (ga - gfirst) / 16) {
    const uint64_t gd = gfirst + 16 * (uint64_t)tid;
    st16<NTS>(gd, ldu<NTL>(src + (gd - d0)));
  }
  if (glast <= ga) return;
  const uint64_t ng = (glast - ga) / 16;
  const uint64_t s0 = src + (ga - d0);
  const uint64_t stride = nthreads;
  // whole steps of U granules for every lane of this wave: a wave-uniform count,
  // so the loop is a scalar loop and the waits are counted, not vmcnt(0) at a join
  const uint64_t wlast = tid | 63;  // this wave's last thread
  const uint64_t span = wlast + (U - 1) * stride;  // highest granule of step 0 in the wave
  const uint64_t steps = ng > span ? (ng - 1 - span) / (U * stride) + 1 : 0;
  const uint32_t nsteps = __builtin_amdgcn_readfirstlane((uint32_t)steps);
  uint64_t g = tid;
  if (PIPE && nsteps) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = ldu<NTL>(s0 + (g + k * stride) * 16);
    for (uint32_t i = 1; i < nsteps; ++i) {
      u32x4 w[U];
      const uint64_t gn = g + U * stride;
#pragma unroll
      for (int k = 0; k < U; ++k) w[k] = ldu<NTL>(s0 + (gn + k * stride) * 16);
#pragma unroll
      for (int k = 0; k < U; ++k) st16<NTS>(ga + (g + k * stride) * 16, v[k]);
#pragma unroll
      for (int k = 0; k < U; ++k) v[k] = w[k];
      g = gn;
    }
#pragma unroll
    for (int k = 0; k < U; ++k) st16<NTS>(ga + (g + k * stride) * 16, v[k]);
    g += U * stride;
  } else {
    for (uint32_t i = 0; i < nsteps; ++i, g += U * stride) {
      u32x4 v[U];
#pragma unroll
      for (int k = 0; k < U; ++k) v[k] = ldu<NTL>(s0 + (g + k * stride) * 16);
#pragma unroll
      for (int k = 0; k < U; ++k) st16<NTS>(ga + (g + k * stride) * 16, v[k]);
    }
  }
  for (; g < ng; g += stride) st16<NTS>(ga + g * 16, ldu<NTL>(s0 + g * 16));
}


// Body "dma": LDS-DMA staging with split roles, so no wave ever waits for its
// own stores.  Waves 0-1 issue global_load_lds_dwordx4 (per-lane unaligned
// source address; LDS destination base + 16 lane) into ring slot k % 2 and wait
// only for their own loads of the previous step (counted vmcnt); waves 2-3 read
// the previous slot (ds_read_b128) and store it.  One s_barrier per step.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
template <int U, bool NTL>
__device__ void copy_dma(uint64_t dst, uint64_t src, uint64_t len, uint32_t tid, lds_u32* ring) {
  const uint64_t d0 = dst, d1 = dst + len;
  const uint64_t gfirst = (d0 + 15) & ~uint64_t(15);
  const uint64_t glast = d1 & ~uint64_t(15);
  {
    const uint64_t hend = gfirst < d1 ? gfirst : d1;
    const uint64_t tstart = glast >= gfirst ? glast : d1;
    const uint64_t nh = hend - d0, nt = d1 - tstart;
    if (tid < nh + nt) {
      const uint64_t b = tid < nh ? d0 + tid : tstart + (tid - nh);
      *reinterpret_cast<uint8_t*>(b) = *reinterpret_cast<const uint8_t*>(src + (b - d0));
    }
  }
  if (glast <= gfirst) return;
  const uint64_t ng = (glast - gfirst) / 16;
  const uint64_t s0 = src + (gfirst - d0);
  constexpr uint32_t kStep = 2 * U * 64;  // granules per step
  const uint32_t nsteps = (uint32_t)((ng + kStep - 1) / kStep);
  const uint32_t wave = tid >> 6, lane = tid & 63;
  const bool loader = wave < 2;
  const uint32_t w = wave & 1;
  for (uint32_t k = 0; k <= nsteps; ++k) {
    if (loader) {
      if (k < nsteps) {
        lds_u32* slot = ring + (k & 1) * (kStep * 4);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t gi = (u * 2 + w) * 64;  // wave-uniform granule offset in the step
          const uint64_t g = (uint64_t)k * kStep + gi + lane;
          const uint64_t gc = g < ng ? g : ng - 1;  // clamp: every lane issues (the slot image stays lane-linear)
          __builtin_amdgcn_global_load_lds(reinterpret_cast<__attribute__((address_space(1))) void*>(s0 + gc * 16),
                                           slot + gi * 4, 16, 0, NTL ? 2 : 0);
        }
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    asm volatile("s_barrier" ::: "memory");
    if (!loader && k > 0) {
      const uint32_t kk = k - 1;
      const lds_u32* slot = ring + (kk & 1) * (kStep * 4);
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u] = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(slot + ((u * 2 + w) * 64 + lane) * 4);
      if ((uint64_t)k * kStep <= ng) {  // whole step (wave-uniform)
#pragma unroll
        for (int u = 0; u < U; ++u) st16<false>(gfirst + ((uint64_t)kk * kStep + (u * 2 + w) * 64 + lane) * 16, v[u]);
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint64_t g = (uint64_t)kk * kStep + (u * 2 + w) * 64 + lane;
          if (g < ng) st16<false>(gfirst + g * 16, v[u]);
        }
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // the ring is reused by the next task
}

enum Body { kLib = 0, kHw = 1, kHwPipe = 2, kHw8 = 3, kHwNt = 4, kHw2 = 5, kHwNtl = 6, kHwNtlNts = 7, kDma = 8, kDmaNt = 9 };

template <int BODY, bool STATIC>
__global__ __launch_bounds__(256) void k_tasks(const Task* __restrict__ tasks, uint64_t n, uint32_t* queue) {
  __shared__ uint32_t ticket;
  __shared__ __attribute__((aligned(16))) uint32_t ring[(BODY == kDma || BODY == kDmaNt) ? 2 * 2 * 4 * 64 * 4 : 4];
  uint64_t t = blockIdx.x;
  while (t < n) {
    const Task tk = tasks[t];
    if (BODY == kLib) copy_range<4, false, true, 1024>(tk.dst, tk.src, tk.len, threadIdx.x, blockDim.x);
    if (BODY == kHw) copy_hw<4, false, false>(tk.dst, tk.src, tk.len, threadIdx.x, blockDim.x);
    if (BODY == kHwPipe) copy_hw<4, false, true>(tk.dst, tk.src, tk.len, threadIdx.x, blockDim.x);
    if (BODY == kHw8) copy_hw<8, false, false>(tk.dst, tk.src, tk.len, threadIdx.x, blockDim.x);
    if (BODY == kHwNt) copy_hw<4, true, false>(tk.dst, tk.src, tk.len, threadIdx.x, blockDim.x);
    if (BODY == kHw2) copy_hw<2, false, true>(tk.dst, tk.src, tk.len, threadIdx.x, blockDim.x);
    if (BODY == kHwNtl) copy_hw<4, false, false, true>(tk.dst, tk.src, tk.len, threadIdx.x, blockDim.x);
    if (BODY == kHwNtlNts) copy_hw<4, true, false, true>(tk.dst, tk.src, tk.len, threadIdx.x, blockDim.x);
    if (BODY == kDma) copy_dma<4, false>(tk.dst, tk.src, tk.len, threadIdx.x, (lds_u32*)ring);
    if (BODY == kDmaNt) copy_dma<4, true>(tk.dst, tk.src, tk.len, threadIdx.x, (lds_u32*)ring);
    if (STATIC) {
      t += gridDim.x;
    } else {
      __syncthreads();
      if (threadIdx.x == 0) ticket = atomicAdd(queue, 1u);
      __syncthreads();
      t = gridDim.x + (uint64_t)ticket;
    }
  }
}

// flat aligned copy (the float4-copy ceiling), U granules per thread per step
__global__ __launch_bounds__(256) void k_flat(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t ng) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; g + 3 * stride < ng; g += 4 * stride) {
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = s[g + k * stride];
#pragma unroll
    for (int k = 0; k < 4; ++k) d[g + k * stride] = v[k];
  }
  for (; g < ng; g += stride) d[g] = s[g];
}

// read-only pass over task sources (cached loads), one word out per thread
template <bool NT>
__global__ __launch_bounds__(256) void k_read_tasks(const Task* __restrict__ tasks, uint64_t n, uint32_t* queue,
                                                    uint32_t* sink) {
  __shared__ uint32_t ticket;
  uint64_t t = blockIdx.x;
  uint32_t acc = 0;
  while (t < n) {
    const Task tk = tasks[t];
    const uint64_t a0 = tk.src & ~uint64_t(15), a1 = (tk.src + tk.len + 15) & ~uint64_t(15);
    const uint64_t ng = (a1 - a0) / 16;
    uint64_t g = threadIdx.x;
    for (; g + 3 * 256 < ng; g += 4 * 256) {
      u32x4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = ld16<NT>(a0 + (g + k * 256) * 16);
#pragma unroll
      for (int k = 0; k < 4; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    for (; g < ng; g += 256) {
      const u32x4 v = ld16<NT>(a0 + g * 16);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    __syncthreads();
    if (threadIdx.x == 0) ticket = atomicAdd(queue, 1u);
    __syncthreads();
    t = gridDim.x + (uint64_t)ticket;
  }
  if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;  // keeps the loads
}

// mismatching bytes of every task (dst vs src)
__global__ void k_check(const Task* __restrict__ tasks, uint64_t n, unsigned long long* bad) {
  for (uint64_t t = blockIdx.x; t < n; t += gridDim.x) {
    const Task tk = tasks[t];
    unsigned long long b = 0;
    for (uint64_t x = threadIdx.x; x < tk.len; x += blockDim.x)
      b += reinterpret_cast<const uint8_t*>(tk.dst)[x] != reinterpret_cast<const uint8_t*>(tk.src)[x];
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

static std::vector<Task> cut_pieces(const std::vector<Task>& r, uint32_t pieces, uint64_t piece_min) {
  std::vector<Task> out;
  for (const Task& x : r) {
    const uint64_t even = ((x.len + pieces - 1) / pieces + 15) & ~uint64_t(15);
    const uint64_t ps = std::max(even, piece_min), h = x.dst & 15;
    for (uint64_t j = 0;; ++j) {
      const uint64_t a = j ? j * ps - h : 0, b = std::min(x.len, (j + 1) * ps - h);
      if (a >= x.len) break;
      if (a < b) out.push_back({x.dst + a, x.src + a, b - a});
    }
  }
  return out;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  const std::string sec = argc > 2 ? argv[2] : "bodies,mall,sub";
  auto want = [&](const char* x) { return sec.find(x) != std::string::npos; };
  const uint64_t n = 4096, chunk = 4ull << 20, pay = 1ull << 20;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const uint32_t cus = prop.multiProcessorCount;
  uint8_t *chunks, *payload, *flat_dst;
  CK(hipMalloc(&chunks, n * chunk));
  CK(hipMalloc(&payload, n * pay));
  CK(hipMalloc(&flat_dst, n * pay));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)payload, n * pay / 8, 7ull);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)chunks, n * chunk / 8, 9ull);
  std::mt19937_64 rng(3);
  std::vector<Task> ranges(n);
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t len = (64 << 10) + rng() % ((1 << 20) - (64 << 10) + 1);
    const uint64_t off = rng() % (chunk - len + 1);
    ranges[i] = {(uint64_t)chunks + i * chunk + off, (uint64_t)payload + i * pay, len};
    total += len;
  }
  const std::vector<Task> tasks = cut_pieces(ranges, 8, 64 << 10);
  Task* d_tasks;
  Task* d_ranges;
  CK(hipMalloc(&d_tasks, tasks.size() * sizeof(Task)));
  CK(hipMalloc(&d_ranges, n * sizeof(Task)));
  CK(hipMemcpy(d_tasks, tasks.data(), tasks.size() * sizeof(Task), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ranges, ranges.data(), n * sizeof(Task), hipMemcpyHostToDevice));
  uint32_t* q;
  unsigned long long* bad;
  uint32_t* sink;
  CK(hipMalloc(&q, 4096 * 4));
  CK(hipMalloc(&bad, 8));
  CK(hipMalloc(&sink, 4096));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const uint32_t grid = cus * 8;
  printf("{\"probe\":\"copy\",\"cus\":%u,\"ranges\":%llu,\"tasks\":%zu,\"bytes\":%llu}\n", cus,
         (unsigned long long)n, tasks.size(), (unsigned long long)total);

  struct V {
    const char* name;
    void (*fn)(const Task*, uint64_t, uint32_t*, uint32_t);
  };
#define TV(NAME, B, S)                                                                          \
  V {                                                                                           \
    NAME, [](const Task* t, uint64_t nt, uint32_t* qq, uint32_t g) {                            \
      (void)hipMemsetAsync(qq, 0, 4, 0);                                                        \
      hipLaunchKernelGGL((k_tasks<B, S>), dim3(g), dim3(256), 0, 0, t, nt, qq);                 \
    }                                                                                           \
  }
  const V vars[] = {TV("lib", kLib, false),       TV("hw", kHw, false),      TV("hw_pipe", kHwPipe, false),
                    TV("hw_u8", kHw8, false),     TV("hw_ntstore", kHwNt, false), TV("hw_u2pipe", kHw2, false),
                    TV("hw_static", kHw, true),   TV("lib_static", kLib, true),
                    TV("hw_ntload", kHwNtl, false), TV("hw_ntload_ntstore", kHwNtlNts, false),
                    TV("dma_split", kDma, false), TV("dma_split_nt", kDmaNt, false)};
  const int nv = sizeof(vars) / sizeof(vars[0]);
  // correctness: scramble the chunks, run once, compare every task's bytes
  for (int v = 0; v < nv; ++v) {
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)chunks, n * chunk / 8, 100ull + v);
    vars[v].fn(d_tasks, tasks.size(), q, grid);
    CK(hipMemsetAsync(bad, 0, 8, 0));
    hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, 0, d_ranges, n, bad);
    unsigned long long b = 0;
    CK(hipMemcpy(&b, bad, 8, hipMemcpyDeviceToHost));
    printf("{\"check\":\"%s\",\"bad_bytes\":%llu}\n", vars[v].name, b);
    if (b) return 1;
  }
  std::vector<std::vector<float>> ms(nv + 3);
  for (int r = 0; r < (want("bodies") ? reps : 0); ++r) {
    for (int v = 0; v < nv; ++v) {
      CK(hipEventRecord(e0, 0));
      vars[v].fn(d_tasks, tasks.size(), q, grid);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t);
    }
    // flat copy of the same byte count, aligned
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_flat, dim3(grid), dim3(256), 0, 0, (const u32x4*)payload, (u32x4*)flat_dst, total / 16);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    ms[nv].push_back(t);
    // read-only pass over the task sources
    CK(hipMemsetAsync(q, 0, 4, 0));
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_read_tasks<false>, dim3(grid), dim3(256), 0, 0, d_tasks, (uint64_t)tasks.size(), q, sink);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&t, e0, e1));
    ms[nv + 1].push_back(t);
    CK(hipMemsetAsync(q, 0, 4, 0));
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_read_tasks<true>, dim3(grid), dim3(256), 0, 0, d_tasks, (uint64_t)tasks.size(), q, sink);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&t, e0, e1));
    ms[nv + 2].push_back(t);
  }
  auto med = [](std::vector<float> x) {
    std::sort(x.begin(), x.end());
    return x[x.size() / 2];
  };
  for (int v = 0; v < (want("bodies") ? nv + 3 : 0); ++v) {
    const char* nm = v < nv ? vars[v].name : v == nv ? "flat_aligned" : v == nv + 1 ? "read_only" : "read_only_nt";
    const double m = med(ms[v]);
    const double moved = v > nv ? (double)total : 2.0 * total;
    printf("{\"variant\":\"%s\",\"ms\":%.4f,\"tbs_moved\":%.3f}\n", nm, m, moved / m / 1e9);
  }

  // Infinity-Cache reuse: copy a window of W bytes cold (after a 2 GiB sweep
  // elsewhere) vs right after a read of the same window.
  if (want("mall")) for (uint64_t W : {32ull << 20, 64ull << 20, 128ull << 20, 192ull << 20, 256ull << 20, 512ull << 20}) {
    std::vector<float> cold, warm;
    std::vector<Task> one{{(uint64_t)flat_dst, (uint64_t)payload + (1ull << 30), W}};
    Task* d_one;
    CK(hipMalloc(&d_one, sizeof(Task)));
    CK(hipMemcpy(d_one, one.data(), sizeof(Task), hipMemcpyHostToDevice));
    for (int r = 0; r < reps; ++r) {
      for (int w = 0; w < 2; ++w) {
        hipLaunchKernelGGL(k_flat, dim3(grid), dim3(256), 0, 0, (const u32x4*)chunks, (u32x4*)(chunks + (4ull << 30)),
                           (2ull << 30) / 16);  // evict
        if (w) {  // read the window (cached loads): 1 task spread by the read kernel's static grid
          std::vector<Task> parts;
          for (uint64_t o = 0; o < W; o += 256 << 10) parts.push_back({0, (uint64_t)payload + (1ull << 30) + o, 256 << 10});
          static Task* d_parts = nullptr;
          static size_t cap = 0;
          if (parts.size() > cap) {
            if (d_parts) CK(hipFree(d_parts));
            CK(hipMalloc(&d_parts, parts.size() * sizeof(Task)));
            cap = parts.size();
          }
          CK(hipMemcpy(d_parts, parts.data(), parts.size() * sizeof(Task), hipMemcpyHostToDevice));
          CK(hipMemsetAsync(q, 0, 4, 0));
          hipLaunchKernelGGL(k_read_tasks<false>, dim3(grid), dim3(256), 0, 0, d_parts, (uint64_t)parts.size(), q, sink);
        }
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k_flat, dim3(grid), dim3(256), 0, 0, (const u32x4*)(payload + (1ull << 30)),
                           (u32x4*)flat_dst, W / 16);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        (w ? warm : cold).push_back(t);
      }
    }
    printf("{\"mall\":\"copy after read\",\"window_mib\":%llu,\"cold_ms\":%.4f,\"warm_ms\":%.4f,\"cold_tbs\":%.3f,"
           "\"warm_tbs\":%.3f}\n",
           (unsigned long long)(W >> 20), med(cold), med(warm), 2.0 * W / med(cold) / 1e9,
           2.0 * W / med(warm) / 1e9);
    CK(hipFree(d_one));
  }

  // Sub-batched read -> copy of the d3 ranges (the read stands in for the pre hash: payload + old
  // bytes, cached loads) vs read-all then copy-all.
  {
    std::vector<Task> rd;  // per range: payload and the old bytes under the write
    for (const Task& x : ranges) {
      rd.push_back({0, x.src, x.len});
      rd.push_back({0, x.dst, x.len});
    }
    Task* d_rd;
    CK(hipMalloc(&d_rd, rd.size() * sizeof(Task)));
    CK(hipMemcpy(d_rd, rd.data(), rd.size() * sizeof(Task), hipMemcpyHostToDevice));
    for (uint64_t B : {4096ull, 1024ull, 512ull, 256ull, 128ull}) {
      if (!want("sub")) break;
      // task index ranges per sub-batch
      std::vector<uint64_t> tfirst;
      {
        uint64_t ti = 0;
        for (uint64_t i = 0; i < n; ++i) {
          if (i % B == 0) tfirst.push_back(ti);
          while (ti < tasks.size() && tasks[ti].src < (uint64_t)payload + (i + 1) * pay) ++ti;
        }
        tfirst.push_back(tasks.size());
      }
      std::vector<float> tt;
      for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(k_flat, dim3(grid), dim3(256), 0, 0, (const u32x4*)chunks, (u32x4*)(chunks + (4ull << 30)),
                           (2ull << 30) / 16);
        CK(hipEventRecord(e0, 0));
        for (uint64_t b = 0; b * B < n; ++b) {
          CK(hipMemsetAsync(q + 2 * b, 0, 8, 0));
          hipLaunchKernelGGL(k_read_tasks<false>, dim3(grid), dim3(256), 0, 0, d_rd + 2 * b * B, 2 * std::min(B, n - b * B),
                             q + 2 * b, sink);
          hipLaunchKernelGGL((k_tasks<kHw, false>), dim3(grid), dim3(256), 0, 0, d_tasks + tfirst[b],
                             tfirst[b + 1] - tfirst[b], q + 2 * b + 1);
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        tt.push_back(t);
      }
      printf("{\"subbatch\":%llu,\"ms\":%.4f,\"note\":\"read(payload+old) then hw copy per sub-batch\"}\n",
             (unsigned long long)B, med(tt));
    }
  }

  // piece-size sweep of the task copy (hw body, tickets)
  if (want("pieces")) {
    struct PC { uint32_t pieces; uint64_t pmin; };
    for (PC pc : {PC{8, 64 << 10}, PC{16, 32 << 10}, PC{4, 128 << 10}, PC{1, 1 << 20}, PC{64, 16 << 10}, PC{32, 32 << 10}}) {
      const std::vector<Task> tk = cut_pieces(ranges, pc.pieces, pc.pmin);
      Task* d_tk;
      CK(hipMalloc(&d_tk, tk.size() * sizeof(Task)));
      CK(hipMemcpy(d_tk, tk.data(), tk.size() * sizeof(Task), hipMemcpyHostToDevice));
      std::vector<float> tt;
      for (int r = 0; r < reps; ++r) {
        CK(hipMemsetAsync(q, 0, 4, 0));
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((k_tasks<kHw2, false>), dim3(grid), dim3(256), 0, 0, d_tk, (uint64_t)tk.size(), q);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        tt.push_back(t);
      }
      printf("{\"pieces\":%u,\"piece_min_kib\":%llu,\"tasks\":%zu,\"ms\":%.4f}\n", pc.pieces,
             (unsigned long long)(pc.pmin >> 10), tk.size(), med(tt));
      CK(hipFree(d_tk));
    }
  }
  // two-stream overlap: reads of sub-batch j+1 (stand-in for the pre hash) beside the copy of sub-batch j
  if (want("overlap")) {
    std::vector<Task> rd;
    for (const Task& x : ranges) {
      rd.push_back({0, x.src, x.len});
      rd.push_back({0, x.dst, x.len});
    }
    Task* d_rd;
    CK(hipMalloc(&d_rd, rd.size() * sizeof(Task)));
    CK(hipMemcpy(d_rd, rd.data(), rd.size() * sizeof(Task), hipMemcpyHostToDevice));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(64);
    for (auto& x : ev) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
    for (uint64_t K : {1ull, 2ull, 4ull, 8ull}) {
      const uint64_t B = n / K;
      std::vector<uint64_t> tfirst;
      {
        uint64_t ti = 0;
        for (uint64_t i = 0; i < n; ++i) {
          if (i % B == 0) tfirst.push_back(ti);
          while (ti < tasks.size() && tasks[ti].src < (uint64_t)payload + (i + 1) * pay) ++ti;
        }
        tfirst.push_back(tasks.size());
      }
      std::vector<float> tt;
      for (int r = 0; r < reps; ++r) {
        CK(hipMemsetAsync(q, 0, 4 * 4 * K, s1));
        CK(hipStreamSynchronize(s1));
        CK(hipEventRecord(e0, s1));
        CK(hipStreamWaitEvent(s2, e0, 0));
        for (uint64_t b = 0; b < K; ++b) {
          hipLaunchKernelGGL(k_read_tasks<true>, dim3(grid), dim3(256), 0, s1, d_rd + 2 * b * B, 2 * B, q + 2 * b, sink);
          CK(hipEventRecord(ev[b], s1));
          CK(hipStreamWaitEvent(s2, ev[b], 0));
          hipLaunchKernelGGL((k_tasks<kHw2, false>), dim3(grid), dim3(256), 0, s2, d_tasks + tfirst[b],
                             tfirst[b + 1] - tfirst[b], q + 2 * b + 1);
        }
        CK(hipEventRecord(e1, s2));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        tt.push_back(t);
      }
      printf("{\"overlap_parts\":%llu,\"ms\":%.4f,\"note\":\"nt read(payload+old) on s1, copy on s2 after its part\"}\n",
             (unsigned long long)K, med(tt));
    }
  }
  return 0;
}
