// scripts/probe_pool_growth.hip -- do kernels see their own writes on memory the stream-ordered
// pool has just grown (or re-mapped after a trim)?  Library-free probe (not product code).
//
// The update wrong-checksum incident hit the first DELTA update of a process,
// i.e. the first call whose per-call hipMallocAsync scratch had to come from new pool memory.
// This probe replays the pipeline's write/read pattern on such memory without the library:
//   zero launch (every word) -> "prep" (plain stores of job words, atomicMax / 64-bit atomicAdd
//   on control words, plain zero stores of accumulators) -> "hash" (atomicXor into the
//   accumulators from many waves) -> check (every word against the host's expectation),
// on the null stream or a created stream, and counts iterations with any wrong word.
//   probe_pool_growth ITERS MODE STREAM [memcpy]
//     MODE   trim  : hipMemPoolTrimTo(pool, 0) before every allocation (fresh physical memory)
//            grow  : every allocation larger than any before (the pool grows every time)
//            reuse : same size every time (cached pool block; control)
//            malloc: hipMalloc / hipFree instead of the pool (control)
//     STREAM null | own
//     memcpy: a pageable hipMemcpy of a 56 B record before each iteration's kernels (the C++
//             drop-in test's staging), checked too
// Prints one JSON line.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define HIP_ASSERT(x)                                                                \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));            \
      std::exit(2);                                                                  \
    }                                                                                \
  } while (0)

__host__ __device__ inline uint32_t mix(uint32_t a, uint32_t b) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u + (a << 6) + (a >> 2));
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h | 1u;  // never zero
}

// layout (words): [0] max, [2..3] u64 count, [16, 16 + J) job words, [16 + J, 16 + 2J) accumulators,
// the rest only zeroed
constexpr uint32_t kHead = 16;
constexpr int kXorRounds = 8;

__global__ void k_zero(uint32_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = 0u;
}

__global__ void k_prep(uint32_t* p, uint32_t J, uint32_t iter) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < J; i += gridDim.x * blockDim.x) {
    const uint32_t v = mix(i, iter);
    p[kHead + i] = v;
    p[kHead + J + i] = 0u;
    atomicMax(p, v >> 8);
    atomicAdd(reinterpret_cast<unsigned long long*>(p + 2), 1ull);
  }
}

__global__ void k_hash(uint32_t* p, uint32_t J, uint32_t iter) {
  // every wave reads the control word first (as k_crc_ranges reads dyn_max), then xors
  const uint32_t m = __builtin_amdgcn_readfirstlane(p[0]);
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < J * kXorRounds; t += gridDim.x * blockDim.x) {
    const uint32_t i = t % J, r = t / J;
    atomicXor(p + kHead + J + i, mix(i ^ (r << 24), iter) ^ (m == 0 ? 0xDEADu : 0u));
  }
}

struct Bad {
  unsigned long long count;
  unsigned long long first;  // word index + 1
  uint32_t got, want;
  uint32_t rec_bad, pad;
};

__global__ void k_check(const uint32_t* p, uint64_t n, uint32_t J, uint32_t iter, uint32_t want_max,
                        const uint8_t* rec, const uint8_t* rec_want, Bad* bad) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t want;
    if (i == 0) {
      want = want_max;
    } else if (i == 2) {
      want = J;
    } else if (i >= kHead && i < kHead + J) {
      want = mix((uint32_t)(i - kHead), iter);
    } else if (i >= kHead + J && i < kHead + 2 * (uint64_t)J) {
      const uint32_t k = (uint32_t)(i - kHead - J);
      want = 0;
      for (int r = 0; r < kXorRounds; ++r) want ^= mix(k ^ ((uint32_t)r << 24), iter);
    } else {
      want = 0;
    }
    const uint32_t got = p[i];
    if (got != want) {
      if (atomicAdd(&bad->count, 1ull) == 0) {
        bad->first = i + 1;
        bad->got = got;
        bad->want = want;
      }
    }
  }
  if (rec && blockIdx.x == 0 && threadIdx.x < 56 && rec[threadIdx.x] != rec_want[threadIdx.x]) atomicAdd(&bad->rec_bad, 1u);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  const char* mode = argc > 2 ? argv[2] : "trim";
  const bool own = argc > 3 && !strcmp(argv[3], "own");
  const bool memcpy_rec = argc > 4 && !strcmp(argv[4], "memcpy");
  hipStream_t s = nullptr;
  if (own) HIP_ASSERT(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipMemPool_t pool;
  HIP_ASSERT(hipDeviceGetDefaultMemPool(&pool, 0));
  uint64_t keep = UINT64_MAX;  // as the library configured the pool
  HIP_ASSERT(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep));
  Bad* dbad = nullptr;
  uint8_t *drec = nullptr, *dwant = nullptr;
  HIP_ASSERT(hipMalloc(&dbad, sizeof(Bad)));
  HIP_ASSERT(hipMalloc(&drec, 64));
  HIP_ASSERT(hipMalloc(&dwant, 64));
  int bad_iters = 0, rec_bad_iters = 0;
  Bad first{};
  int first_iter = -1;
  uint64_t first_bytes = 0;
  for (int it = 0; it < iters; ++it) {
    uint64_t bytes;
    if (!strcmp(mode, "grow"))
      bytes = (64ull << 10) * (it + 1) + 4096 * (it % 7);
    else if (!strcmp(mode, "reuse"))
      bytes = 8ull << 20;
    else
      bytes = (64ull << 10) << (it % 9);  // trim / malloc: 64 KiB .. 16 MiB
    const uint64_t words = bytes / 4;
    const uint32_t J = (uint32_t)((words - kHead) / 4);
    uint32_t want_max = 0;
    for (uint32_t i = 0; i < J; ++i) want_max = std::max(want_max, mix(i, it) >> 8);
    if (!strcmp(mode, "trim")) {
      HIP_ASSERT(hipDeviceSynchronize());
      HIP_ASSERT(hipMemPoolTrimTo(pool, 0));
    }
    HIP_ASSERT(hipMemset(dbad, 0, sizeof(Bad)));
    uint8_t rec[64];
    for (int k = 0; k < 64; ++k) rec[k] = (uint8_t)(mix(k, it) >> 3);
    if (memcpy_rec) {
      HIP_ASSERT(hipMemcpy(dwant, rec, 64, hipMemcpyHostToDevice));
      HIP_ASSERT(hipDeviceSynchronize());
      HIP_ASSERT(hipMemcpy(drec, rec, 56, hipMemcpyHostToDevice));  // pageable, like the test's IO record
    }
    uint32_t* p = nullptr;
    if (!strcmp(mode, "malloc"))
      HIP_ASSERT(hipMalloc(&p, bytes));
    else
      HIP_ASSERT(hipMallocAsync((void**)&p, bytes, s));
    const unsigned gz = (unsigned)std::min<uint64_t>(4096, (words + 255) / 256);
    hipLaunchKernelGGL(k_zero, dim3(gz), dim3(256), 0, s, p, words);
    hipLaunchKernelGGL(k_prep, dim3(std::min<uint32_t>(4096, (J + 255) / 256)), dim3(256), 0, s, p, J, (uint32_t)it);
    hipLaunchKernelGGL(k_hash, dim3(256), dim3(1024), 0, s, p, J, (uint32_t)it);
    hipLaunchKernelGGL(k_check, dim3(gz), dim3(256), 0, s, p, words, J, (uint32_t)it, want_max,
                       memcpy_rec ? drec : nullptr, dwant, dbad);
    HIP_ASSERT(hipGetLastError());
    if (!strcmp(mode, "malloc")) {
      HIP_ASSERT(hipStreamSynchronize(s));
      HIP_ASSERT(hipFree(p));
    } else {
      HIP_ASSERT(hipFreeAsync(p, s));
    }
    HIP_ASSERT(hipStreamSynchronize(s));
    Bad b{};
    HIP_ASSERT(hipMemcpy(&b, dbad, sizeof(Bad), hipMemcpyDeviceToHost));
    if (b.count) {
      if (!bad_iters) {
        first = b;
        first_iter = it;
        first_bytes = bytes;
      }
      ++bad_iters;
    }
    rec_bad_iters += b.rec_bad != 0;
  }
  std::printf("{\"mode\":\"%s\",\"stream\":\"%s\",\"memcpy\":%d,\"iters\":%d,\"bad_iters\":%d,\"rec_bad_iters\":%d,"
              "\"first_iter\":%d,\"first_bytes\":%llu,\"first_bad_words\":%llu,\"first_word\":%lld,"
              "\"got\":\"%08x\",\"want\":\"%08x\"}\n",
              mode, own ? "own" : "null", (int)memcpy_rec, iters, bad_iters, rec_bad_iters, first_iter,
              (unsigned long long)first_bytes, (unsigned long long)first.count, (long long)first.first - 1, first.got,
              first.want);
  return 0;
}
