// scripts/probe_staging.cpp -- does a kernel see the bytes of a small pageable hipMemcpy
// issued right after an asynchronous hipMemset of ANOTHER buffer?  (probe, not product code)
//
// tests/cpp/test_checksuminfo.cpp failed once in 8 fresh processes in round 3 (and twice in
// round 1) on the first update of a write pattern: the pattern starts with
// hipMemset(dChunk, 0xAB, 512) on the null stream, then a pageable hipMemcpy of the payload
// (1..256 B) and of the 56 B IO record, then the update kernels -- which verified a wrong
// payload hash, while the staged bytes read back correct and a retry passed.  This probe runs
// that sequence without the library: a one-workgroup kernel sums the staged payload and record
// (position-weighted) and the host compares with the bytes it copied; a mismatch is classified
// as "payload stale" (matches the previous payload) or "record stale" or other.
//   probe_staging ROUNDS   variants, one JSON line each:
//     memset      the test's sequence: memset(A) -> memcpy(B) -> memcpy(C) -> kernel
//     nomemset    memcpy(B) -> memcpy(C) -> kernel
//     memset_sync memset(A) -> hipDeviceSynchronize -> memcpy(B) -> memcpy(C) -> kernel
//     copy_sync   memset(A) -> memcpy(B) -> memcpy(C) -> hipDeviceSynchronize -> kernel
//     pinned      memset(A) -> hipMemcpyAsync(B, C from pinned host, null stream) -> kernel
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
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

template <bool NT>
__global__ void k_sum(const uint8_t* __restrict__ b, uint32_t nb, const uint8_t* __restrict__ c, uint32_t nc,
                      unsigned long long* __restrict__ out) {
  __shared__ unsigned long long part[4];
  unsigned long long s = 0;
  for (uint32_t i = threadIdx.x; i < nb + nc; i += blockDim.x) {
    const uint8_t* p = i < nb ? b + i : c + (i - nb);
    const uint8_t v = NT ? __builtin_nontemporal_load(p) : *p;
    s += (unsigned long long)v * (i + 1);
  }
  for (int d = 32; d > 0; d >>= 1) s += __shfl_xor(s, d, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = part[0] + part[1] + part[2] + part[3];
}

static unsigned long long host_sum(const uint8_t* b, uint32_t nb, const uint8_t* c, uint32_t nc) {
  unsigned long long s = 0;
  for (uint32_t i = 0; i < nb + nc; ++i) s += (unsigned long long)(i < nb ? b[i] : c[i - nb]) * (i + 1);
  return s;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 20000;
  const char* names[] = {"memset", "nomemset", "memset_sync", "copy_sync", "pinned", "memset_nt"};
  uint8_t *dA, *dB, *dC;
  unsigned long long* dOut;
  HIP_ASSERT(hipMalloc(&dA, 512));
  HIP_ASSERT(hipMalloc(&dB, 512));
  HIP_ASSERT(hipMalloc(&dC, 64));
  HIP_ASSERT(hipMalloc(&dOut, 8));
  uint8_t *hB, *hC;
  HIP_ASSERT(hipHostMalloc(&hB, 512, 0));
  HIP_ASSERT(hipHostMalloc(&hC, 64, 0));
  std::mt19937_64 rng(12345);
  for (int v = 0; v < 6; ++v) {
    int bad = 0, stale_b = 0, stale_c = 0;
    std::vector<uint8_t> pb(256, 0), pc(56, 0), b(256), c(56);
    uint32_t pnb = 0;
    for (int r = 0; r < rounds; ++r) {
      const uint32_t nb = 1 + rng() % 256;
      for (uint32_t i = 0; i < nb; ++i) b[i] = (uint8_t)rng();
      for (auto& x : c) x = (uint8_t)rng();
      if (v != 1) HIP_ASSERT(hipMemset(dA, 0xAB, 512));
      if (v == 2) HIP_ASSERT(hipDeviceSynchronize());
      if (v == 4) {
        std::memcpy(hB, b.data(), nb);
        std::memcpy(hC, c.data(), 56);
        HIP_ASSERT(hipMemcpyAsync(dB, hB, nb, hipMemcpyHostToDevice, nullptr));
        HIP_ASSERT(hipMemcpyAsync(dC, hC, 56, hipMemcpyHostToDevice, nullptr));
      } else {
        HIP_ASSERT(hipMemcpy(dB, b.data(), nb, hipMemcpyHostToDevice));
        HIP_ASSERT(hipMemcpy(dC, c.data(), 56, hipMemcpyHostToDevice));
      }
      if (v == 3) HIP_ASSERT(hipDeviceSynchronize());
      if (v == 5)
        hipLaunchKernelGGL(k_sum<true>, dim3(1), dim3(256), 0, nullptr, dB, nb, dC, 56u, dOut);
      else
        hipLaunchKernelGGL(k_sum<false>, dim3(1), dim3(256), 0, nullptr, dB, nb, dC, 56u, dOut);
      unsigned long long got = 0;
      HIP_ASSERT(hipMemcpy(&got, dOut, 8, hipMemcpyDeviceToHost));
      const unsigned long long want = host_sum(b.data(), nb, c.data(), 56);
      if (got != want) {
        ++bad;
        // previous payload bytes where the new payload is longer: the buffer held pb[0..pnb) then older bytes
        std::vector<uint8_t> ob(b.begin(), b.begin() + nb);
        for (uint32_t i = 0; i < nb && i < pnb; ++i) ob[i] = pb[i];
        if (got == host_sum(ob.data(), nb, c.data(), 56)) ++stale_b;
        if (got == host_sum(b.data(), nb, pc.data(), 56)) ++stale_c;
        if (bad <= 5)
          std::fprintf(stderr, "%s round %d nb=%u got=%llu want=%llu\n", names[v], r, nb, got, want);
      }
      std::copy(b.begin(), b.begin() + nb, pb.begin());
      pnb = nb;
      pc = c;
    }
    std::printf("{\"probe\":\"staging\",\"variant\":\"%s\",\"rounds\":%d,\"bad\":%d,\"payload_stale\":%d,\"record_stale\":%d}\n",
                names[v], rounds, bad, stale_b, stale_c);
    std::fflush(stdout);
  }
  return 0;
}
