// scripts/probe_apply_inlib.hip -- the update pipeline's apply in the library vs the copy
// probe's library-shaped one-shot kernel, on the SAME buffers in one process (probe, not
// product code).  d3-shaped batch: 4096 writes of U[64 KiB, 1 MiB] at byte offsets of full
// 4 MiB chunks from 1 MiB-strided payloads; every call re-applies the same IOs (payload
// checksums stay valid, so every write verifies and copies).  Per variant: K calls of
// hf3fs_crc_update_batch (DELTA) timed with events, then (same buffers) the standalone
// one-shot copy of the same ranges.  Run under rocprofv3 --kernel-trace for per-kernel times.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include scripts/probe_apply_inlib.hip \
//         -L3fs_amd/lib -lhf3fs_crc -Wl,-rpath,$PWD/3fs_amd/lib -o /tmp/pai
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "hf3fs_crc.h"

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                        \
    }                                                                                 \
  } while (0)
#define RC(x)                                                              \
  do {                                                                     \
    int r_ = (x);                                                          \
    if (r_) {                                                              \
      fprintf(stderr, "%s:%d %s: rc=%d\n", __FILE__, __LINE__, #x, r_);    \
      exit(3);                                                             \
    }                                                                      \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(1)));

__global__ void k_fill(uint64_t* p, uint64_t n, uint64_t seed) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + i * 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    p[i] = z ^ (z >> 31);
  }
}

struct Range {
  uint64_t dst, src, len;
};
// the copy probe's table form (k_ragged_oneshot), 8 KiB destination pieces
__global__ __launch_bounds__(256) void k_oneshot8(const Range* __restrict__ rs, const uint32_t* __restrict__ ptab,
                                                  const uint32_t* __restrict__ first) {
  constexpr uint64_t P = 8192;
  const uint32_t r = ptab[blockIdx.x];
  const Range R = rs[r];
  const uint64_t k = blockIdx.x - first[r];
  const uint64_t base = (R.dst & ~(P - 1)) + k * P;
  const uint64_t a = base > R.dst ? base : R.dst, e = base + P < R.dst + R.len ? base + P : R.dst + R.len;
  const uint32_t tid = threadIdx.x;
  const uint64_t ga = (a + 15) & ~uint64_t(15), ge = e & ~uint64_t(15);
  const int64_t so = (int64_t)R.src - (int64_t)R.dst;
  if (ga >= ge) {
    if (tid < e - a) *reinterpret_cast<uint8_t*>(a + tid) = *reinterpret_cast<const uint8_t*>(a + tid + so);
    return;
  }
  const uint64_t nh = ga - a, nt = e - ge;
  if (tid < nh + nt) {
    const uint64_t b = tid < nh ? a + tid : ge + (tid - nh);
    *reinterpret_cast<uint8_t*>(b) = *reinterpret_cast<const uint8_t*>(b + so);
  }
  const uint64_t ng = (ge - ga) / 16;
  typedef __attribute__((address_space(1))) const u32x4u gq;
  for (uint64_t g = tid; g < ng; g += 256)
    __builtin_nontemporal_store(*reinterpret_cast<gq*>(ga + g * 16 + so), reinterpret_cast<u32x4*>(ga + g * 16));
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 8;
  const uint64_t n = 4096, chunk = 4ull << 20, pay = 1ull << 20;
  uint8_t *chunks, *payload;
  CK(hipMalloc(&chunks, n * chunk));
  CK(hipMalloc(&payload, n * pay));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)payload, n * pay / 8, 11ull);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)chunks, n * chunk / 8, 12ull);
  std::mt19937_64 rng(3);
  std::vector<Range> rs(n);
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t len = (64 << 10) + rng() % ((1 << 20) - (64 << 10) + 1);
    const uint64_t off = rng() % (chunk - len + 1);
    rs[i] = {(uint64_t)chunks + i * chunk + off, (uint64_t)payload + i * pay, len};
    total += len;
  }
  // payload and chunk checksums through the library
  std::vector<uint64_t> pa(n), pl(n), ca(n), cl(n);
  for (uint64_t i = 0; i < n; ++i) {
    pa[i] = rs[i].src, pl[i] = rs[i].len, ca[i] = (uint64_t)chunks + i * chunk, cl[i] = chunk;
  }
  uint64_t *d_pa, *d_pl, *d_ca, *d_cl;
  uint32_t *d_pck, *d_cck;
  CK(hipMalloc(&d_pa, n * 8));
  CK(hipMalloc(&d_pl, n * 8));
  CK(hipMalloc(&d_ca, n * 8));
  CK(hipMalloc(&d_cl, n * 8));
  CK(hipMalloc(&d_pck, n * 4));
  CK(hipMalloc(&d_cck, n * 4));
  CK(hipMemcpy(d_pa, pa.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_pl, pl.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ca, ca.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_cl, cl.data(), n * 8, hipMemcpyHostToDevice));
  RC(hf3fs_crc_create_batch(1, (const void* const*)d_pa, d_pl, nullptr, d_pck, n, pay, nullptr));
  RC(hf3fs_crc_create_batch(1, (const void* const*)d_ca, d_cl, nullptr, d_cck, n, chunk, nullptr));
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> pck(n), cck(n);
  CK(hipMemcpy(pck.data(), d_pck, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(cck.data(), d_cck, n * 4, hipMemcpyDeviceToHost));
  std::vector<hf3fs_crc_update_io> ios(n);
  for (uint64_t i = 0; i < n; ++i) {
    hf3fs_crc_update_io& u = ios[i];
    memset(&u, 0, sizeof(u));
    u.chunk = (uint64_t)chunks + i * chunk;
    u.payload = rs[i].src;
    u.offset = (uint32_t)(rs[i].dst - u.chunk);
    u.length = (uint32_t)rs[i].len;
    u.chunk_size = (uint32_t)chunk;
    u.update_type = HF3FS_UPDATE_WRITE;
    u.chunk_checksum_type = 1;
    u.chunk_checksum = cck[i];
    u.write_checksum_type = 1;
    u.write_checksum = pck[i];
  }
  hf3fs_crc_update_io* d_ios;
  CK(hipMalloc(&d_ios, n * sizeof(hf3fs_crc_update_io)));
  // the standalone one-shot copy's table
  std::vector<uint32_t> ptab, first(n);
  for (uint64_t r = 0; r < n; ++r) {
    first[r] = (uint32_t)ptab.size();
    for (uint64_t b = rs[r].dst & ~uint64_t(8191); b < rs[r].dst + rs[r].len; b += 8192) ptab.push_back((uint32_t)r);
  }
  Range* d_rs;
  uint32_t *d_ptab, *d_first;
  CK(hipMalloc(&d_rs, n * sizeof(Range)));
  CK(hipMalloc(&d_ptab, ptab.size() * 4));
  CK(hipMalloc(&d_first, n * 4));
  CK(hipMemcpy(d_rs, rs.data(), n * sizeof(Range), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ptab, ptab.data(), ptab.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_first, first.data(), n * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("{\"probe\":\"apply_inlib\",\"ios\":%llu,\"bytes\":%llu,\"pieces8k\":%zu}\n", (unsigned long long)n,
         (unsigned long long)total, ptab.size());
  const char* variants[][2] = {{"0", "tickets"}, {"-1", "one_shot"}, {"0", "tickets"}, {"-1", "one_shot"}};
  for (auto& v : variants) {
    RC(hf3fs_crc_set_option("apply_grid", v[0]));
    std::vector<float> ms;
    for (int k = 0; k < K + 2; ++k) {
      CK(hipMemcpy(d_ios, ios.data(), n * sizeof(hf3fs_crc_update_io), hipMemcpyHostToDevice));
      CK(hipEventRecord(e0, 0));
      RC(hf3fs_crc_update_batch(1, d_ios, n, (uint32_t)chunk, HF3FS_UPDATE_MODE_DELTA, nullptr));
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (k >= 2) ms.push_back(t);
    }
    std::vector<hf3fs_crc_update_io> out(n);
    CK(hipMemcpy(out.data(), d_ios, n * sizeof(hf3fs_crc_update_io), hipMemcpyDeviceToHost));
    int bad = 0;
    for (auto& u : out) bad += u.status != 0;
    std::sort(ms.begin(), ms.end());
    // the standalone one-shot copy of the same ranges, right after a pipeline call
    std::vector<float> cs;
    for (int k = 0; k < K; ++k) {
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(k_oneshot8, dim3((unsigned)ptab.size()), dim3(256), 0, 0, d_rs, d_ptab, d_first);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      cs.push_back(t);
    }
    std::sort(cs.begin(), cs.end());
    printf("{\"variant\":\"%s\",\"batch_ms\":%.4f,\"bad_status\":%d,\"standalone_oneshot_ms\":%.4f,"
           "\"standalone_tbs\":%.3f}\n",
           v[1], ms[ms.size() / 2], bad, cs[cs.size() / 2], 2.0 * total / cs[cs.size() / 2] / 1e9);
  }
  return 0;
}
