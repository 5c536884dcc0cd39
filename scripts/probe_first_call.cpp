// scripts/probe_first_call.cpp -- does the FIRST library call of a process verify a correct
// payload?  (probe, not product code; the C++ drop-in test's first update_batch reported
// kChecksumMismatch on correct bytes in rounds 1 and 3, and a retry passed.)
//
//   probe_first_call MODE [warm|grow|refN]
//     MODE 0/1 = REFERENCE/DELTA; warm = a create_batch before the update (context built);
//     grow = a 256 MiB stream-ordered allocation freed before the update (pool grown);
//     refN = N REFERENCE updates of the same IO before (the C++ drop-in test's order)
// Prints one JSON line: status of the first update, its retry, the device create of the
// staged payload, and the oracle's value.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../include/hf3fs_crc.h"
extern "C" {
#include "../oracle/crc_oracle.h"
}

#define HIP_ASSERT(x)                                                                \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));            \
      std::exit(2);                                                                  \
    }                                                                                \
  } while (0)

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 1;
  // options, comma separated: warm, grow, refN, sync (device sync before the probed update),
  // trim (the pool's free blocks returned to the driver before it)
  const char* opt = argc > 2 ? argv[2] : "";
  auto has = [&](const char* o) { return strstr(opt, o) != nullptr; };
  const bool warm = has("warm"), grow = has("grow"), sync = has("sync"), trim = has("trim");
  const char* rp = strstr(opt, "ref");
  const int refs = rp ? atoi(rp + 3) : 0;
  const uint32_t chunk = 512, len = 232;
  std::mt19937_64 rng(512 + mode);
  std::vector<uint8_t> data(len);
  for (auto& x : data) x = (uint8_t)rng();
  const uint32_t want = orc_crc32c_hw(~0u, data.data(), len);
  uint8_t *dChunk = nullptr, *dPayload = nullptr;
  hf3fs_crc_update_io* dIo = nullptr;
  HIP_ASSERT(hipMalloc(&dChunk, chunk));
  HIP_ASSERT(hipMalloc(&dPayload, chunk));
  HIP_ASSERT(hipMalloc(&dIo, sizeof(hf3fs_crc_update_io)));
  uint64_t* dDesc = nullptr;
  uint32_t* dOut = nullptr;
  HIP_ASSERT(hipMalloc(&dDesc, 16));
  HIP_ASSERT(hipMalloc(&dOut, 4));
  HIP_ASSERT(hipMemcpy(dPayload, data.data(), len, hipMemcpyHostToDevice));
  uint64_t desc[2] = {(uint64_t)dPayload, len};
  HIP_ASSERT(hipMemcpy(dDesc, desc, 16, hipMemcpyHostToDevice));
  if (warm) (void)hf3fs_crc_create_batch(1, (const void* const*)dDesc, dDesc + 1, nullptr, dOut, 1, len, nullptr);
  if (grow) {
    void* big = nullptr;
    HIP_ASSERT(hipMallocAsync(&big, 256ull << 20, nullptr));
    HIP_ASSERT(hipFreeAsync(big, nullptr));
    HIP_ASSERT(hipDeviceSynchronize());
  }
  int ref_bad = 0;
  for (int r = 0; r < refs; ++r) {
    hf3fs_crc_update_io io{};
    io.chunk = (uint64_t)dChunk;
    io.payload = (uint64_t)dPayload;
    io.length = len;
    io.update_type = HF3FS_UPDATE_WRITE;
    io.write_checksum_type = 1;
    io.write_checksum = want;
    HIP_ASSERT(hipMemcpy(dIo, &io, sizeof(io), hipMemcpyHostToDevice));
    (void)hf3fs_crc_update_batch(1, dIo, 1, chunk, HF3FS_UPDATE_MODE_REFERENCE, nullptr);
    HIP_ASSERT(hipMemcpy(&io, dIo, sizeof(io), hipMemcpyDeviceToHost));
    ref_bad += io.status != 0;
  }
  if (sync) HIP_ASSERT(hipDeviceSynchronize());
  if (trim) {
    hipMemPool_t pool;
    HIP_ASSERT(hipDeviceGetDefaultMemPool(&pool, 0));
    HIP_ASSERT(hipDeviceSynchronize());
    HIP_ASSERT(hipMemPoolTrimTo(pool, 0));
  }
  int st[2] = {-1, -1};
  uint32_t out[2] = {0, 0};
  for (int k = 0; k < 2; ++k) {
    hf3fs_crc_update_io io{};
    io.chunk = (uint64_t)dChunk;
    io.payload = (uint64_t)dPayload;
    io.offset = 0;
    io.length = len;
    io.chunk_size = 0;
    io.update_type = HF3FS_UPDATE_WRITE;
    io.write_checksum_type = 1;
    io.write_checksum = want;
    HIP_ASSERT(hipMemcpy(dIo, &io, sizeof(io), hipMemcpyHostToDevice));
    const int rc = hf3fs_crc_update_batch(1, dIo, 1, chunk, mode, nullptr);
    HIP_ASSERT(hipMemcpy(&io, dIo, sizeof(io), hipMemcpyDeviceToHost));
    st[k] = rc ? -rc : io.status;
    out[k] = io.out_checksum;
  }
  (void)hf3fs_crc_create_batch(1, (const void* const*)dDesc, dDesc + 1, nullptr, dOut, 1, len, nullptr);
  uint32_t dev = 0;
  HIP_ASSERT(hipMemcpy(&dev, dOut, 4, hipMemcpyDeviceToHost));
  std::printf("{\"opt\":\"%s\",\"mode\":%d,\"warm\":%d,\"grow\":%d,\"refs\":%d,\"ref_bad\":%d,\"first_status\":%d,\"first_out\":\"%08x\",\"retry_status\":%d,"
              "\"retry_out\":\"%08x\",\"device_create\":\"%08x\",\"oracle\":\"%08x\"}\n",
              opt, mode, (int)warm, (int)grow, refs, ref_bad, st[0], out[0], st[1], out[1], dev, want);
  return 0;
}
