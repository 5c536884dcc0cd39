// Payload staging through a pageable hipMemcpy, then hf3fs_crc_update_batch on
// the null stream (VERDICT r01 "next" #1; reference contract ChunkReplica.cc:193-207:
// the payload checksum is recomputed from the bytes the update reads).
//
//   test_staging                 the deterministic pattern: ONE reused device payload
//                                buffer, a pageable hipMemcpy of distinct bytes per IO,
//                                update_batch on the null stream, 100 IOs per (mode,
//                                pipeline, chunk size), every status / checksum / chunk
//                                byte checked against the CPU oracle.
//   test_staging --stress N      the same pattern N IOs per cell over staging variants
//                                (pageable / pageable + device sync / pinned async /
//                                cached loads) plus a library-free probe kernel that
//                                sums the staged bytes with non-temporal and with cached
//                                loads; prints the failure count of every cell and the
//                                diagnostics of each failure (which bytes the device saw).
// Built with hipcc (the probe kernel) by 3fs_amd/build.py; run by tests/test_cpp_dropin.py.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/hf3fs_crc.h"
extern "C" {
#include "../../oracle/crc_oracle.h"
}

#define HIP_ASSERT(x)                                                                \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));            \
      std::exit(2);                                                                  \
    }                                                                                \
  } while (0)

// ---- library-free probe: position-weighted sum of the staged dwords ----
template <bool NT>
__global__ void k_probe(const uint32_t* __restrict__ p, uint64_t words, unsigned long long* out) {
  unsigned long long acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t w = NT ? __builtin_nontemporal_load(p + i) : p[i];
    acc += (unsigned long long)w * (2 * i + 1);
  }
  atomicAdd(out, acc);
}
static unsigned long long probe_host(const uint8_t* b, uint64_t words) {
  unsigned long long acc = 0;
  for (uint64_t i = 0; i < words; ++i) {
    uint32_t w;
    std::memcpy(&w, b + 4 * i, 4);
    acc += (unsigned long long)w * (2 * i + 1);
  }
  return acc;
}

enum Staging { kPageable = 0, kPageableSync, kPinned, kPageableCached, kNumStaging };
static const char* kStagingName[] = {"pageable", "pageable+devsync", "pinned-async", "pageable+cached-loads"};

struct Cell {
  int fails = 0, ios = 0, stale_prev = 0, staged_bad = 0, create_bad = 0;
};

// One cell: n IOs of the RANDWRITE/SEQWRITE mix on one chunk, payload staged per `how`.
static Cell run_cell(uint32_t chunkSize, int mode, bool unfused, Staging how, int n, uint64_t seed, bool verbose) {
  setenv("HF3FS_CRC_UPDATE_PIPELINE", unfused ? "unfused" : "fused", 1);
  if (how == kPageableCached) setenv("HF3FS_CRC_NT", "0", 1); else unsetenv("HF3FS_CRC_NT");
  std::mt19937_64 rng(seed);
  Cell cell;
  uint8_t *dChunk = nullptr, *dPayload = nullptr, *hPinned = nullptr;
  hf3fs_crc_update_io* dIo = nullptr;
  HIP_ASSERT(hipMalloc(&dChunk, chunkSize));
  HIP_ASSERT(hipMalloc(&dPayload, chunkSize));
  HIP_ASSERT(hipMalloc(&dIo, sizeof(hf3fs_crc_update_io)));
  HIP_ASSERT(hipHostMalloc((void**)&hPinned, chunkSize, hipHostMallocDefault));
  HIP_ASSERT(hipMemset(dChunk, 0xAB, chunkSize));
  HIP_ASSERT(hipMemset(dPayload, 0, chunkSize));
  std::vector<uint8_t> chunk, shadow(chunkSize, 0);  // shadow = what dPayload holds if every copy landed
  uint32_t size = 0;
  orc_checksum meta{ORC_NONE, 0};
  size_t offset = 0, length = 0;
  for (int w = 0; w < n; ++w) {
    if (rng() % 2) offset = rng() % chunkSize;  // RANDWRITE
    else offset = (offset + length) % chunkSize;  // SEQWRITE (wraps)
    if (offset + 1 >= chunkSize) offset = 0;
    length = 1 + rng() % ((chunkSize - offset) / 2 + 1);
    std::vector<uint8_t> data(length);
    for (auto& x : data) x = (uint8_t)rng();
    const uint32_t client = orc_crc32c_hw(~0u, data.data(), length);
    std::vector<uint8_t> prev(shadow.begin(), shadow.begin() + length);
    switch (how) {
      case kPageable:
      case kPageableCached:
        HIP_ASSERT(hipMemcpy(dPayload, data.data(), length, hipMemcpyHostToDevice));
        break;
      case kPageableSync:
        HIP_ASSERT(hipMemcpy(dPayload, data.data(), length, hipMemcpyHostToDevice));
        HIP_ASSERT(hipDeviceSynchronize());
        break;
      default:
        std::memcpy(hPinned, data.data(), length);
        HIP_ASSERT(hipMemcpyAsync(dPayload, hPinned, length, hipMemcpyHostToDevice, nullptr));
        HIP_ASSERT(hipStreamSynchronize(nullptr));
    }
    std::memcpy(shadow.data(), data.data(), length);
    hf3fs_crc_update_io io{};
    io.chunk = (uint64_t)dChunk;
    io.payload = (uint64_t)dPayload;
    io.offset = (uint32_t)offset;
    io.length = (uint32_t)length;
    io.chunk_size = size;
    io.update_type = HF3FS_UPDATE_WRITE;
    io.chunk_checksum_type = meta.type;
    io.chunk_checksum = meta.value;
    io.write_checksum_type = ORC_CRC32C;
    io.write_checksum = client;
    HIP_ASSERT(hipMemcpy(dIo, &io, sizeof(io), hipMemcpyHostToDevice));
    const int rc = hf3fs_crc_update_batch(HF3FS_CHECKSUM_CRC32C, dIo, 1, chunkSize, mode, nullptr);
    HIP_ASSERT(hipMemcpy(&io, dIo, sizeof(io), hipMemcpyDeviceToHost));
    ++cell.ios;
    // oracle: the write applied to the host model (gap zero-filled), checksum of the bytes
    std::vector<uint8_t> next = chunk;
    if (offset + length > next.size()) next.resize(offset + length, 0);
    std::memcpy(&next[offset], data.data(), length);
    const uint32_t want = orc_crc32c_hw(~0u, next.data(), next.size());
    std::vector<uint8_t> back(next.size());
    HIP_ASSERT(hipMemcpy(back.data(), dChunk, back.size(), hipMemcpyDeviceToHost));
    const bool ok = rc == 0 && io.status == 0 && io.out_size == next.size() && io.out_checksum == want &&
                    io.out_checksum_type == ORC_CRC32C && back == next;
    if (!ok) {
      ++cell.fails;
      std::vector<uint8_t> staged(length);
      HIP_ASSERT(hipMemcpy(staged.data(), dPayload, length, hipMemcpyDeviceToHost));
      const bool staged_ok = staged == data;
      cell.staged_bad += !staged_ok;
      // what a hash of the PREVIOUS contents of the payload buffer would have been
      const uint32_t prev_crc = orc_crc32c_hw(~0u, prev.data(), length);
      uint64_t* dDesc = nullptr;
      uint32_t* dOut = nullptr;
      HIP_ASSERT(hipMalloc(&dDesc, 16));
      HIP_ASSERT(hipMalloc(&dOut, 4));
      const uint64_t desc[2] = {(uint64_t)dPayload, length};
      HIP_ASSERT(hipMemcpy(dDesc, desc, 16, hipMemcpyHostToDevice));
      const int crc_rc = hf3fs_crc_create_batch(1, (const void* const*)dDesc, dDesc + 1, nullptr, dOut, 1, length, nullptr);
      uint32_t dev = 0;
      HIP_ASSERT(hipMemcpy(&dev, dOut, 4, hipMemcpyDeviceToHost));
      cell.create_bad += dev != client;
      HIP_ASSERT(hipFree(dDesc));
      HIP_ASSERT(hipFree(dOut));
      size_t first_bad = 0;
      while (first_bad < back.size() && back[first_bad] == next[first_bad]) ++first_bad;
      if (verbose || cell.fails <= 5)
        std::fprintf(stderr,
                     "FAIL %s chunk=%u mode=%d unfused=%d io=%d off=%zu len=%zu size=%u rc=%d status=%d "
                     "out=%08x want=%08x client=%08x prev_contents_crc=%08x staged_ok=%d recreate=%08x(rc=%d) "
                     "first_bad_chunk_byte=%zu/%zu\n",
                     kStagingName[how], chunkSize, mode, (int)unfused, w, offset, length, size, rc, io.status,
                     io.out_checksum, want, client, prev_crc, (int)staged_ok, dev, crc_rc, first_bad, back.size());
      // resynchronise the model with the device so later IOs stay meaningful
      if (io.status == 0) {
        chunk = back;
        size = io.out_size;
        meta = orc_checksum{io.out_checksum_type, io.out_checksum};
        if (orc_crc32c_hw(~0u, chunk.data(), chunk.size()) != meta.value) {
          // device bytes and checksum disagree: restart the chunk
          chunk.clear();
          size = 0;
          meta = orc_checksum{ORC_NONE, 0};
        }
      }
      continue;
    }
    chunk.swap(next);
    size = io.out_size;
    meta = orc_checksum{io.out_checksum_type, io.out_checksum};
  }
  HIP_ASSERT(hipFree(dChunk));
  HIP_ASSERT(hipFree(dPayload));
  HIP_ASSERT(hipFree(dIo));
  HIP_ASSERT(hipHostFree(hPinned));
  unsetenv("HF3FS_CRC_UPDATE_PIPELINE");
  unsetenv("HF3FS_CRC_NT");
  return cell;
}

// Library-free probe: pageable copy of fresh bytes into ONE reused buffer, then
// one kernel reads them (non-temporal or cached loads); n rounds.
static int run_probe(bool nt, int n, uint64_t seed) {
  std::mt19937_64 rng(seed);
  const uint64_t cap = 256 << 10;
  uint32_t* dBuf = nullptr;
  unsigned long long* dSum = nullptr;
  HIP_ASSERT(hipMalloc(&dBuf, cap));
  HIP_ASSERT(hipMalloc(&dSum, 8));
  int fails = 0;
  for (int r = 0; r < n; ++r) {
    const uint64_t words = 1 + rng() % (cap / 4);
    std::vector<uint8_t> h(4 * words);
    for (auto& x : h) x = (uint8_t)rng();
    HIP_ASSERT(hipMemcpy(dBuf, h.data(), h.size(), hipMemcpyHostToDevice));
    HIP_ASSERT(hipMemsetAsync(dSum, 0, 8, nullptr));
    const unsigned grid = (unsigned)((words + 255) / 256 < 1024 ? (words + 255) / 256 : 1024);
    if (nt) hipLaunchKernelGGL(k_probe<true>, dim3(grid), dim3(256), 0, nullptr, dBuf, words, dSum);
    else hipLaunchKernelGGL(k_probe<false>, dim3(grid), dim3(256), 0, nullptr, dBuf, words, dSum);
    HIP_ASSERT(hipGetLastError());
    unsigned long long got = 0;
    HIP_ASSERT(hipMemcpy(&got, dSum, 8, hipMemcpyDeviceToHost));
    if (got != probe_host(h.data(), words)) {
      if (++fails <= 5) std::fprintf(stderr, "PROBE FAIL nt=%d round=%d words=%llu\n", (int)nt, r, (unsigned long long)words);
    }
  }
  HIP_ASSERT(hipFree(dBuf));
  HIP_ASSERT(hipFree(dSum));
  return fails;
}

int main(int argc, char** argv) {
  int stress = 0;
  if (argc > 2 && std::string(argv[1]) == "--stress") stress = std::atoi(argv[2]);
  int total_fail = 0;
  if (!stress) {
    // the deterministic pattern: 100 IOs per (chunk size, mode, pipeline), every result vs the oracle
    for (uint32_t cs : {512u, 128u << 10})
      for (int mode : {HF3FS_UPDATE_MODE_REFERENCE, HF3FS_UPDATE_MODE_DELTA})
        for (bool unfused : {false, true}) {
          Cell c = run_cell(cs, mode, unfused, kPageable, 100, cs * 7 + mode * 3 + unfused, true);
          std::printf("pageable chunk=%u mode=%d unfused=%d ios=%d fails=%d\n", cs, mode, (int)unfused, c.ios,
                      c.fails);
          total_fail += c.fails;
        }
  } else {
    for (int how = 0; how < kNumStaging; ++how)
      for (uint32_t cs : {512u, 128u << 10, 4u << 20})
        for (int mode : {HF3FS_UPDATE_MODE_REFERENCE, HF3FS_UPDATE_MODE_DELTA})
          for (bool unfused : {false, true}) {
            Cell c = run_cell(cs, mode, unfused, (Staging)how, stress, 1000 + how * 100 + cs + mode * 3 + unfused,
                              false);
            std::printf("%-22s chunk=%-8u mode=%d unfused=%d ios=%d fails=%d staged_bad=%d recreate_bad=%d\n",
                        kStagingName[how], cs, mode, (int)unfused, c.ios, c.fails, c.staged_bad, c.create_bad);
            std::fflush(stdout);
            total_fail += c.fails;
          }
    for (bool nt : {true, false}) {
      const int f = run_probe(nt, 20 * stress, 77 + nt);
      std::printf("probe nt=%d rounds=%d fails=%d\n", (int)nt, 20 * stress, f);
      total_fail += f;
    }
  }
  hf3fs_crc_shutdown();
  std::printf("%s (%d failures)\n", total_fail ? "FAILED" : "ALL OK", total_fail);
  return total_fail ? 1 : 0;
}
