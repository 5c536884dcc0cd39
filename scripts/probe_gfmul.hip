// GF(2^32) multiply probe (not product code): the bit-serial gf_mul of gf2.h (~215 VALU)
// against a carry-less multiply built from 16 integer multiplies (bits split in four
// residue classes mod 4, so no carry reaches a bit of its own class) reduced by one
// x^32 dword step through LDS tables.  Checks both on the host and on the device over
// random operands, then times a dependent chain of each per thread.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I 3fs_amd/csrc -o scripts/probe_gfmul scripts/probe_gfmul.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#include "gf2.h"

using namespace hf3fs_crc;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__host__ __device__ inline uint64_t clmul32(uint32_t x, uint32_t y) {
  const uint32_t m0 = 0x11111111u, m1 = 0x22222222u, m2 = 0x44444444u, m3 = 0x88888888u;
  const uint32_t x0 = x & m0, x1 = x & m1, x2 = x & m2, x3 = x & m3;
  const uint32_t y0 = y & m0, y1 = y & m1, y2 = y & m2, y3 = y & m3;
  auto M = [](uint32_t a, uint32_t b) { return (uint64_t)a * b; };
  const uint64_t z0 = M(x0, y0) ^ M(x1, y3) ^ M(x2, y2) ^ M(x3, y1);
  const uint64_t z1 = M(x0, y1) ^ M(x1, y0) ^ M(x2, y3) ^ M(x3, y2);
  const uint64_t z2 = M(x0, y2) ^ M(x1, y1) ^ M(x2, y0) ^ M(x3, y3);
  const uint64_t z3 = M(x0, y3) ^ M(x1, y2) ^ M(x2, y1) ^ M(x3, y0);
  return (z0 & 0x1111111111111111ull) | (z1 & 0x2222222222222222ull) | (z2 & 0x4444444444444444ull) |
         (z3 & 0x8888888888888888ull);
}

// a * b mod P, reflected (bit 31 = x^0): clmul << 1 puts degrees 0..31 in the high word and
// degrees 32..63 in the low word as (reflected poly) * x^32, which the dword tables reduce.
__host__ __device__ inline uint32_t gf_mul_cl(uint32_t a, uint32_t b, const uint32_t* dw) {
  const uint64_t z = clmul32(a, b) << 1;
  const uint32_t h = (uint32_t)(z >> 32), l = (uint32_t)z;
  return h ^ dw[l & 0xffu] ^ dw[256 + ((l >> 8) & 0xffu)] ^ dw[512 + ((l >> 16) & 0xffu)] ^ dw[768 + (l >> 24)];
}

constexpr int kChain = 256;

__global__ void k_old(const uint32_t* in, uint32_t* out, uint32_t f) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t v = in[i];
  for (int k = 0; k < kChain; ++k) v = gf_mul(v, f ^ (uint32_t)k, kPolyCrc32c);
  out[i] = v;
}

__global__ void k_new(const uint32_t* in, uint32_t* out, uint32_t f, const uint32_t* dwg) {
  __shared__ uint32_t dw[1024];
  for (int k = threadIdx.x; k < 1024; k += blockDim.x) dw[k] = dwg[k];
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t v = in[i];
  for (int k = 0; k < kChain; ++k) v = gf_mul_cl(v, f ^ (uint32_t)k, dw);
  out[i] = v;
}

int main() {
  std::vector<uint32_t> dw(1024);
  const uint32_t x32 = xpow_bits(32, kPolyCrc32c);
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) dw[256 * k + b] = gf_mul(b << (8 * k), x32, kPolyCrc32c);
  std::mt19937_64 rng(7);
  for (int t = 0; t < 200000; ++t) {
    const uint32_t a = (uint32_t)rng(), b = (uint32_t)rng();
    if (gf_mul_cl(a, b, dw.data()) != gf_mul(a, b, kPolyCrc32c)) {
      printf("{\"probe\": \"gfmul\", \"host_check\": false, \"a\": %u, \"b\": %u}\n", a, b);
      return 1;
    }
  }
  const int n = 1 << 20;
  std::vector<uint32_t> h(n), o1(n), o2(n);
  for (auto& x : h) x = (uint32_t)rng();
  uint32_t *din, *d1, *d2, *ddw;
  CK(hipMalloc(&din, 4 * n));
  CK(hipMalloc(&d1, 4 * n));
  CK(hipMalloc(&d2, 4 * n));
  CK(hipMalloc(&ddw, 4096));
  CK(hipMemcpy(din, h.data(), 4 * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(ddw, dw.data(), 4096, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float t_old = 0, t_new = 0;
  for (int r = 0; r < 3; ++r) {
    float ms;
    CK(hipEventRecord(a));
    k_old<<<n / 256, 256>>>(din, d1, 0x9E3779B9u);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    if (r) t_old += ms / 2;
    CK(hipEventRecord(a));
    k_new<<<n / 256, 256>>>(din, d2, 0x9E3779B9u, ddw);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    if (r) t_new += ms / 2;
  }
  CK(hipMemcpy(o1.data(), d1, 4 * n, hipMemcpyDeviceToHost));
  CK(hipMemcpy(o2.data(), d2, 4 * n, hipMemcpyDeviceToHost));
  size_t diff = 0;
  for (int i = 0; i < n; ++i) diff += o1[i] != o2[i];
  const double muls = (double)n * kChain;
  printf("{\"probe\": \"gfmul\", \"host_check\": true, \"device_mismatches\": %zu, \"old_ms\": %.4f, \"new_ms\": %.4f, "
         "\"old_gmul_per_s\": %.1f, \"new_gmul_per_s\": %.1f}\n",
         diff, t_old, t_new, muls / t_old / 1e6, muls / t_new / 1e6);
  return diff ? 1 : 0;
}
