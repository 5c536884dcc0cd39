// scripts/probe_gather.hip -- d5 gather-only probe (probe, not product code).
//
// Question: do 4 KiB KV blocks hash at 3.7 TB/s (64 KiB blocks: 6.0-6.5) because random
// 4 KiB-aligned reads are slow in DRAM, or because of the kernel's per-task structure?
// Same geometry as tests/bench_suite.py d5 / scripts/d5_size_probe.py: ~25 GB of blocks at
// random 4 KiB-aligned offsets of a 32 GiB arena, 16 waves per CU, one workgroup per CU,
// byte-balanced contiguous runs of blocks per wave (as the library's k_bal_assign).  No hash:
// each lane xors the 16 B granules it loads and lane 0 stores one word per block.
//   plain  : per block, load the descriptor, then the block's granules (4 KiB in flight per
//            wave at a time), reduce, store -- the library's per-task shape without the CRC
//   pipe   : the next block's descriptor and first 4 KiB are loaded before this block is
//            reduced (cross-task prefetch)
//   seq    : the same bytes read as one contiguous stream per wave (no gather)
// Usage: probe_gather [reps]   prints one JSON line per (variant, block mix).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define HIP_ASSERT(x)                                                                \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));            \
      std::exit(2);                                                                  \
    }                                                                                \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_cu32x4;

__device__ __forceinline__ u32x4 ldnt(uint64_t a) {
  return __builtin_nontemporal_load(reinterpret_cast<g_cu32x4*>(a));
}

constexpr int kWaves = 16;

__global__ void k_fill(uint32_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 17);
}

// one block: its granules (len multiple of 1 KiB), 4 KiB of loads in flight
__device__ __forceinline__ uint32_t gather_block(uint64_t a, uint32_t len, int lane) {
  u32x4 acc = {0, 0, 0, 0};
  const uint32_t nb = len >> 10;
  const uint64_t g = a + 16 * (uint64_t)lane;
  for (uint32_t b = 0; b < nb; b += 4) {
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = b + k < nb ? ldnt(g + (uint64_t)(b + k) * 1024) : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; ++k) acc ^= v[k];
  }
  return acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int MODE>
__global__ __launch_bounds__(1024) void k_gather(const uint8_t* arena, const uint64_t* __restrict__ offs,
                                                 const uint32_t* __restrict__ lens, const uint32_t* __restrict__ bal,
                                                 uint32_t* __restrict__ out, const uint64_t* __restrict__ seqoff) {
  const int lane = threadIdx.x & 63;
  const uint32_t w = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t t0 = __builtin_amdgcn_readfirstlane(bal[w]), t1 = __builtin_amdgcn_readfirstlane(bal[w + 1]);
  const uint64_t base = (uint64_t)arena;
  if (MODE == 0) {
    for (uint32_t t = t0; t < t1; ++t) {
      const uint64_t a = base + offs[t];
      const uint32_t r = gather_block(a, lens[t], lane);
      if (lane == 0) out[t] = r;
    }
  } else if (MODE == 1) {
    if (t0 >= t1) return;
    uint64_t a = base + offs[t0];
    uint32_t len = lens[t0];
    u32x4 pre[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      pre[k] = (uint32_t)k < (len >> 10) ? ldnt(a + 16 * (uint64_t)lane + k * 1024) : u32x4{0, 0, 0, 0};
    for (uint32_t t = t0; t < t1; ++t) {
      uint64_t na = 0;
      uint32_t nlen = 0;
      if (t + 1 < t1) {
        na = base + offs[t + 1];
        nlen = lens[t + 1];
      }
      u32x4 acc = pre[0] ^ pre[1] ^ pre[2] ^ pre[3];
      const uint32_t nb = len >> 10;
      if (nb > 4) {
        const uint32_t r = gather_block(a + 4096, len - 4096, lane);
        acc.x ^= r;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
        pre[k] = (uint32_t)k < (nlen >> 10) ? ldnt(na + 16 * (uint64_t)lane + k * 1024) : u32x4{0, 0, 0, 0};
      if (lane == 0) out[t] = acc.x ^ acc.y ^ acc.z ^ acc.w;
      a = na;
      len = nlen;
    }
  } else {  // contiguous: the wave's bytes as one run
    const uint64_t s = seqoff[w], e = seqoff[w + 1];
    const uint32_t r = gather_block(base + s, (uint32_t)(e - s), lane);
    if (lane == 0) out[w] = r;
  }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  hipDeviceProp_t prop;
  HIP_ASSERT(hipGetDeviceProperties(&prop, 0));
  const uint32_t cus = prop.multiProcessorCount, nw = cus * kWaves;
  const uint64_t arena_bytes = 32ull << 30;
  uint8_t* arena = nullptr;
  HIP_ASSERT(hipMalloc(&arena, arena_bytes));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t*)arena, arena_bytes / 4);
  HIP_ASSERT(hipDeviceSynchronize());
  const double total_target = 1e6 * 24.8 * 1024;
  struct Mix { const char* name; int kib; };
  const Mix mixes[] = {{"mixed", 0}, {"u4", 4}, {"u16", 16}, {"u64", 64}};
  std::mt19937_64 rng(5);
  for (const Mix& m : mixes) {
    std::vector<uint32_t> lens;
    if (m.kib == 0) {
      const int pool[5] = {4, 8, 16, 32, 64};
      for (int i = 0; i < 1000000; ++i) lens.push_back(pool[rng() % 5] * 1024u);
    } else {
      lens.assign((size_t)(total_target / (m.kib * 1024.0)), m.kib * 1024u);
    }
    const size_t n = lens.size();
    std::vector<uint64_t> offs(n);
    for (size_t i = 0; i < n; ++i) offs[i] = (rng() % ((arena_bytes - 65536) / 4096)) * 4096;
    // byte-balanced contiguous runs: wave w starts at the first block whose prefix >= w * T / nw
    std::vector<uint64_t> pre(n + 1, 0);
    for (size_t i = 0; i < n; ++i) pre[i + 1] = pre[i] + lens[i];
    const uint64_t T = pre[n];
    std::vector<uint32_t> bal(nw + 1);
    std::vector<uint64_t> seqoff(nw + 1);
    for (uint32_t w = 0; w <= nw; ++w) {
      const uint64_t target = (T * w + nw - 1) / nw;
      bal[w] = (uint32_t)(std::lower_bound(pre.begin(), pre.end(), target) - pre.begin());
      if (bal[w] > n) bal[w] = (uint32_t)n;
      seqoff[w] = (target / 1024) * 1024;
    }
    bal[nw] = (uint32_t)n;
    seqoff[nw] = (T / 1024) * 1024;
    uint64_t *dOffs, *dSeq;
    uint32_t *dLens, *dBal, *dOut;
    HIP_ASSERT(hipMalloc(&dOffs, n * 8));
    HIP_ASSERT(hipMalloc(&dLens, n * 4));
    HIP_ASSERT(hipMalloc(&dBal, (nw + 1) * 4));
    HIP_ASSERT(hipMalloc(&dSeq, (nw + 1) * 8));
    HIP_ASSERT(hipMalloc(&dOut, std::max<size_t>(n, nw) * 4));
    HIP_ASSERT(hipMemcpy(dOffs, offs.data(), n * 8, hipMemcpyHostToDevice));
    HIP_ASSERT(hipMemcpy(dLens, lens.data(), n * 4, hipMemcpyHostToDevice));
    HIP_ASSERT(hipMemcpy(dBal, bal.data(), (nw + 1) * 4, hipMemcpyHostToDevice));
    HIP_ASSERT(hipMemcpy(dSeq, seqoff.data(), (nw + 1) * 8, hipMemcpyHostToDevice));
    const char* vname[3] = {"plain", "pipe", "seq"};
    for (int v = 0; v < 3; ++v) {
      auto launch = [&] {
        if (v == 0)
          hipLaunchKernelGGL(k_gather<0>, dim3(cus), dim3(1024), 0, 0, arena, dOffs, dLens, dBal, dOut, dSeq);
        else if (v == 1)
          hipLaunchKernelGGL(k_gather<1>, dim3(cus), dim3(1024), 0, 0, arena, dOffs, dLens, dBal, dOut, dSeq);
        else
          hipLaunchKernelGGL(k_gather<2>, dim3(cus), dim3(1024), 0, 0, arena, dOffs, dLens, dBal, dOut, dSeq);
      };
      launch();
      HIP_ASSERT(hipDeviceSynchronize());
      hipEvent_t e0, e1;
      HIP_ASSERT(hipEventCreate(&e0));
      HIP_ASSERT(hipEventCreate(&e1));
      HIP_ASSERT(hipEventRecord(e0, 0));
      for (int r = 0; r < reps; ++r) launch();
      HIP_ASSERT(hipEventRecord(e1, 0));
      HIP_ASSERT(hipEventSynchronize(e1));
      float ms = 0;
      HIP_ASSERT(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      std::printf("{\"probe\":\"gather\",\"mix\":\"%s\",\"variant\":\"%s\",\"blocks\":%zu,\"bytes\":%llu,\"ms\":%.4f,\"tbs\":%.3f}\n",
                  m.name, vname[v], n, (unsigned long long)T, ms, T / (ms * 1e-3) / 1e12);
      std::fflush(stdout);
      HIP_ASSERT(hipEventDestroy(e0));
      HIP_ASSERT(hipEventDestroy(e1));
    }
    HIP_ASSERT(hipFree(dOffs));
    HIP_ASSERT(hipFree(dLens));
    HIP_ASSERT(hipFree(dBal));
    HIP_ASSERT(hipFree(dSeq));
    HIP_ASSERT(hipFree(dOut));
  }
  HIP_ASSERT(hipFree(arena));
  return 0;
}
