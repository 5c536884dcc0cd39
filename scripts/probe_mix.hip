// probe_mix.hip -- HBM read/write mix probe for the d3 DELTA schedule.
// Is reading the old bytes inside the apply (read payload + read old + write, 1.7:1) faster
// than reading them in the pre-hash pass (pure reads) with a 1:1 copy after it?
// Kernels over uint4 granules, grid-stride, U granules in flight per thread:
//   k_read   sum of A[0, na)                         (pure reads)
//   k_copy   C[i] = A[i]                             (1:1)
//   k_copy_r C[i] = A[i], plus B[0, nb) read and summed along (reads B in step with A)
// Built by the probe script: hipcc --offload-arch=gfx950 -O3 -shared -fPIC.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NTS>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if (NTS)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ a, uint64_t n, uint32_t* __restrict__ sink) {
  u32x4 acc = {0, 0, 0, 0};
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const u32x4 v0 = a[i], v1 = a[i + stride], v2 = a[i + 2 * stride], v3 = a[i + 3 * stride];
    acc ^= v0 ^ v1 ^ v2 ^ v3;
  }
  for (; i < n; i += stride) acc ^= a[i];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

template <bool NTS>
__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ c, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const u32x4 v0 = a[i], v1 = a[i + stride], v2 = a[i + 2 * stride], v3 = a[i + 3 * stride];
    st<NTS>(c + i, v0);
    st<NTS>(c + i + stride, v1);
    st<NTS>(c + i + 2 * stride, v2);
    st<NTS>(c + i + 3 * stride, v3);
  }
  for (; i < n; i += stride) st<NTS>(c + i, a[i]);
}

// copy A -> C (n granules) and read B (nb granules, nb <= n) at the same index
template <bool NTS>
__global__ __launch_bounds__(256) void k_copy_r(const u32x4* __restrict__ a, u32x4* __restrict__ c, uint64_t n,
                                                const u32x4* __restrict__ b, uint64_t nb, uint32_t* __restrict__ sink) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  for (; i + 3 * stride < n; i += 4 * stride) {
    u32x4 o0 = {0, 0, 0, 0}, o1 = o0, o2 = o0, o3 = o0;
    if (i < nb) o0 = b[i];
    if (i + stride < nb) o1 = b[i + stride];
    if (i + 2 * stride < nb) o2 = b[i + 2 * stride];
    if (i + 3 * stride < nb) o3 = b[i + 3 * stride];
    const u32x4 v0 = a[i], v1 = a[i + stride], v2 = a[i + 2 * stride], v3 = a[i + 3 * stride];
    acc ^= o0 ^ o1 ^ o2 ^ o3;
    st<NTS>(c + i, v0);
    st<NTS>(c + i + stride, v1);
    st<NTS>(c + i + 2 * stride, v2);
    st<NTS>(c + i + 3 * stride, v3);
  }
  for (; i < n; i += stride) {
    if (i < nb) acc ^= b[i];
    st<NTS>(c + i, a[i]);
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

extern "C" {
int probe_read(const void* a, uint64_t bytes, uint32_t* sink, uint32_t grid, void* s) {
  hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, (hipStream_t)s, (const u32x4*)a, bytes / 16, sink);
  return (int)hipGetLastError();
}
int probe_copy(const void* a, void* c, uint64_t bytes, uint32_t grid, int nts, void* s) {
  if (nts)
    hipLaunchKernelGGL(k_copy<true>, dim3(grid), dim3(256), 0, (hipStream_t)s, (const u32x4*)a, (u32x4*)c, bytes / 16);
  else
    hipLaunchKernelGGL(k_copy<false>, dim3(grid), dim3(256), 0, (hipStream_t)s, (const u32x4*)a, (u32x4*)c, bytes / 16);
  return (int)hipGetLastError();
}
int probe_copy_r(const void* a, void* c, uint64_t bytes, const void* b, uint64_t bbytes, uint32_t* sink, uint32_t grid,
                 int nts, void* s) {
  if (nts)
    hipLaunchKernelGGL(k_copy_r<true>, dim3(grid), dim3(256), 0, (hipStream_t)s, (const u32x4*)a, (u32x4*)c,
                       bytes / 16, (const u32x4*)b, bbytes / 16, sink);
  else
    hipLaunchKernelGGL(k_copy_r<false>, dim3(grid), dim3(256), 0, (hipStream_t)s, (const u32x4*)a, (u32x4*)c,
                       bytes / 16, (const u32x4*)b, bbytes / 16, sink);
  return (int)hipGetLastError();
}
}
