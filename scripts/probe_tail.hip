// Tail probe (not product code): how long does a pure streaming read of 4 / 16 GB take with
// a static equal split over the waves against a dynamic split (wave-claimed pieces), and
// how far apart do the waves finish?  Each wave records its first-load and last-load
// wall clock (wall_clock64) with a vector store.  Prints one JSON line per case.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/probe_tail scripts/probe_tail.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

typedef unsigned int u4v __attribute__((ext_vector_type(4)));
constexpr int kThreads = 256, kWaves = kThreads / 64, kUnroll = 8;
constexpr uint64_t kWaveStep = 64 * 16 * kUnroll;  // bytes one wave loads per iteration

__device__ __forceinline__ uint4 sweep(const uint4* p, uint64_t n16, uint32_t lane, uint4 acc) {
  // n16: 16 B words, a multiple of 64 * kUnroll
  for (uint64_t i = lane; i < n16; i += 64 * kUnroll) {
    u4v v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) v[u] = __builtin_nontemporal_load((const u4v*)(p + i + 64 * u));
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      acc.x ^= v[u].x;
      acc.y ^= v[u].y;
      acc.z ^= v[u].z;
      acc.w ^= v[u].w;
    }
  }
  return acc;
}

// piece == 0: static split (total / nwaves per wave); else waves claim pieces of `piece` bytes
__global__ void __launch_bounds__(kThreads) k_read(const uint4* buf, uint64_t total, uint64_t piece,
                                                   uint32_t* counter, uint64_t* times, uint32_t* sink) {
  const uint32_t lane = threadIdx.x & 63, w = blockIdx.x * kWaves + (threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  uint64_t t0 = wall_clock64();
  uint4 acc = make_uint4(0, 0, 0, 0);
  if (piece == 0) {
    const uint64_t share = total / nwaves / kWaveStep * kWaveStep;
    acc = sweep(buf + w * share / 16, share / 16, lane, acc);
  } else {
    const uint64_t npieces = total / piece;
    for (;;) {
      uint32_t t = 0;
      if (lane == 0) t = atomicAdd(counter, 1u);
      t = __builtin_amdgcn_readfirstlane(t);
      if (t >= npieces) break;
      acc = sweep(buf + (uint64_t)t * piece / 16, piece / 16, lane, acc);
    }
  }
  const uint64_t t1 = wall_clock64();
  if (lane == 0) {
    times[2 * w] = t0;
    times[2 * w + 1] = t1;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) sink[0] = w;
}

int main() {
  int cus = 0, khz = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  const uint64_t cap = 16ull << 30;
  uint4* buf;
  CK(hipMalloc(&buf, cap));
  CK(hipMemset(buf, 0x5A, cap));
  uint32_t *counter, *sink;
  CK(hipMalloc(&counter, 4));
  CK(hipMalloc(&sink, 4));
  const int wgs_per_cu[] = {4, 8};
  const uint32_t max_waves = cus * 8 * kWaves;
  uint64_t* times;
  CK(hipMalloc(&times, 16ull * max_waves));
  std::vector<uint64_t> h(2ull * max_waves);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const uint64_t sizes[] = {4ull << 30, 16ull << 30};
  const uint64_t pieces[] = {0, 64 << 10, 256 << 10, 1 << 20};
  for (int round = 0; round < 2; ++round)
    for (uint64_t total : sizes)
      for (int wpc : wgs_per_cu)
        for (uint64_t piece : pieces) {
          const uint32_t grid = cus * wpc, nwaves = grid * kWaves;
          float best = 1e9f, sum = 0;
          const int reps = 8;
          for (int r = 0; r < reps + 1; ++r) {
            CK(hipMemsetAsync(counter, 0, 4));
            CK(hipEventRecord(a));
            k_read<<<grid, kThreads>>>(buf, total, piece, counter, times, sink);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (r == 0) continue;  // warm-up
            best = std::min(best, ms);
            sum += ms;
          }
          CK(hipMemcpy(h.data(), times, 16ull * nwaves, hipMemcpyDeviceToHost));
          uint64_t s0 = ~0ull, s1 = 0, e0 = ~0ull, e1 = 0;
          std::vector<uint64_t> ends(nwaves);
          for (uint32_t w = 0; w < nwaves; ++w) {
            s0 = std::min(s0, h[2 * w]);
            s1 = std::max(s1, h[2 * w]);
            e0 = std::min(e0, h[2 * w + 1]);
            e1 = std::max(e1, h[2 * w + 1]);
            ends[w] = h[2 * w + 1];
          }
          std::sort(ends.begin(), ends.end());
          auto us = [&](uint64_t t) { return (double)(t - s0) * 1e3 / khz; };
          printf("{\"probe\": \"tail\", \"round\": %d, \"gb\": %.2f, \"wg_per_cu\": %d, \"piece_kib\": %llu, "
                 "\"ms_mean\": %.4f, \"ms_min\": %.4f, \"tbs_mean\": %.3f, \"last_start_us\": %.1f, "
                 "\"first_end_us\": %.1f, \"p50_end_us\": %.1f, \"p99_end_us\": %.1f, \"last_end_us\": %.1f}\n",
                 round, total / 1e9, wpc, (unsigned long long)(piece >> 10), sum / reps, best,
                 total / (sum / reps) / 1e9, us(s1), us(e0), us(ends[nwaves / 2]),
                 us(ends[(uint64_t)nwaves * 99 / 100]), us(e1));
          fflush(stdout);
        }
  return 0;
}
