// aux_kernels.hip -- see aux_kernels.h.  The bytes are hashed by k_crc_ranges
// between prep and finalize; these kernels only move 24-32 B records.
#include "aux_kernels.h"
#include "gf2.h"

namespace hf3fs_crc {
namespace {

unsigned grid_of(uint64_t n) {
  const uint64_t want = (n + 255) / 256;
  return (unsigned)(want < 4096 ? (want ? want : 1) : 4096);
}

// Wave-aggregated mismatch count: one atomic per wave.
__device__ __forceinline__ void count_bad(uint32_t bad, uint32_t* count) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) bad += __shfl_xor(bad, d, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(count, bad);
}

__global__ void k_scrub_prep(hf3fs_crc_scrub_io* __restrict__ ios, uint64_t n, uint8_t type, uint32_t max_len,
                             uint64_t* __restrict__ addr, uint64_t* __restrict__ len, uint32_t* __restrict__ maxl) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    hf3fs_crc_scrub_io io = ios[i];
    const bool typed = io.checksum_type != kTypeNone;
    const bool ok = (!typed || io.checksum_type == type) && io.length <= max_len && (io.data || !io.length) &&
                    io.fin <= 1;
    const bool need = ok && typed;
    addr[i] = need ? io.data : 0;
    len[i] = need ? io.length : 0;
    io.status = ok ? HF3FS_CRC_OK : HF3FS_CRC_INVALID_ARG;
    io.computed = 0;
    ios[i] = io;
    if (need && io.length) atomicMax(maxl, io.length);
  }
}

// ChunkMetadata::checksum() (Common.h:676) is {checksumType, checksumValue}
// in the raw convention; the chunk engine's ChunkMeta.checksum
// (chunk_engine/src/types/chunk_meta.rs:13) is finalized (ChunkEngine.cc:42,66).
__global__ void k_scrub_finalize(hf3fs_crc_scrub_io* __restrict__ ios, uint64_t n, const uint32_t* __restrict__ v,
                                 uint32_t* __restrict__ count) {
  uint32_t bad = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    hf3fs_crc_scrub_io io = ios[i];
    if (io.status != HF3FS_CRC_OK) {
      ++bad;
      continue;
    }
    if (io.checksum_type == kTypeNone) continue;  // nothing persisted to check against
    io.computed = v[i];
    const uint32_t stored = io.fin ? ~io.checksum : io.checksum;
    if (io.computed != stored) {
      io.status = HF3FS_CRC_CHECKSUM_MISMATCH;
      ++bad;
    }
    ios[i] = io;
  }
  count_bad(bad, count);
}

// One thread per record: {0x05, type, value LE} (hf3fs_checksum_serialize).
__global__ void k_serialize(uint8_t type, const uint32_t* __restrict__ values, uint64_t n, uint8_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t v = values[i];
    uint8_t* o = out + 6 * i;
    o[0] = 5;
    o[1] = type;
    o[2] = (uint8_t)v;
    o[3] = (uint8_t)(v >> 8);
    o[4] = (uint8_t)(v >> 16);
    o[5] = (uint8_t)(v >> 24);
  }
}

__global__ void k_finalize_values(uint32_t* __restrict__ values, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    values[i] = ~values[i];
}

}  // namespace

hipError_t launch_serialize(uint8_t type, const uint32_t* values, uint64_t n, uint8_t* out, hipStream_t st) {
  hipLaunchKernelGGL(k_serialize, dim3(grid_of(n)), dim3(256), 0, st, type, values, n, out);
  return hipGetLastError();
}
hipError_t launch_finalize_values(uint32_t* values, uint64_t n, hipStream_t st) {
  hipLaunchKernelGGL(k_finalize_values, dim3(grid_of(n)), dim3(256), 0, st, values, n);
  return hipGetLastError();
}

hipError_t launch_scrub_prep(hf3fs_crc_scrub_io* ios, uint64_t n, uint8_t type, uint32_t max_len, uint64_t* addr,
                             uint64_t* len, uint32_t* maxl, hipStream_t st) {
  hipLaunchKernelGGL(k_scrub_prep, dim3(grid_of(n)), dim3(256), 0, st, ios, n, type, max_len, addr, len, maxl);
  return hipGetLastError();
}
hipError_t launch_scrub_finalize(hf3fs_crc_scrub_io* ios, uint64_t n, const uint32_t* v, uint32_t* count,
                                 hipStream_t st) {
  hipLaunchKernelGGL(k_scrub_finalize, dim3(grid_of(n)), dim3(256), 0, st, ios, n, v, count);
  return hipGetLastError();
}

}  // namespace hf3fs_crc
