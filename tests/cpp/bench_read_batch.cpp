// The read path INTEGRATION.md §2.1 recommends, measured at 3FS's own call shape
// (VERDICT r03 next #3): each of 32 AioReadWorker threads reaps a batch of completed
// reads (src/storage/aio/AioReadWorker.cc:60-94; batch reads are split at 1024,
// src/storage/service/StorageOperator.cc:163-167) and runs AioReadJob::setResult's
// checksum part for all of them (src/storage/aio/BatchReadJob.cc:24-63).
//
// Modes (one per run, one JSON line on stdout):
//   cpu      the reference: setResult per read on the reaping thread (the oracle's
//            restatement, orc_read_result_checksum, SSE4.2 crc32c)
//   gpu-reg  one hf3fs_crc_read_result_batch per reaped batch; the read bytes stay in
//            hf3fs_crc_host_register'ed host memory (3FS's registered BufferPool slabs,
//            src/storage/service/BufferPool.h:24-27): the kernel reads them over PCIe
//   gpu-hbm  the same call with the read bytes in HBM (upper bound: reads that landed
//            in device memory)
// IO records live in pinned, mapped host memory (the worker fills them, the kernels
// read and complete them in place); one HIP stream per thread.  Reads are {4..64} KiB
// at 4 KiB-aligned offsets of a 1 GiB arena (BASELINE config 5 sizes) at a random
// offset inside a 4 MiB chunk, i.e. partial reads whose checksum is computed
// (BatchReadJob.cc:33-35); every 16th read is a full-chunk read of the stored type
// (reuse, :30-31).  Every result of the first 64 batches per thread is checked
// against the oracle.
// --wait: how a worker waits for its batch -- spin (hipStreamSynchronize, HIP's default busy
// wait), block (an hipEventBlockingSync event: the thread sleeps until the interrupt) or
// yield (hf3fs_crc_stream_wait: hipStreamQuery polled with a 20 us sleep between polls).
//   bench_read_batch --mode M --threads T --batch B --seconds S [--wait spin|block|yield]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hf3fs_crc.h"
extern "C" {
#include "../../oracle/crc_oracle.h"
}

#define HIP_ASSERT(x)                                                    \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e)); \
      std::exit(2);                                                      \
    }                                                                    \
  } while (0)
#define RC_ASSERT(x)                                                              \
  do {                                                                            \
    int rc = (x);                                                                 \
    if (rc) {                                                                     \
      std::fprintf(stderr, "%s failed: %d %s\n", #x, rc, hf3fs_crc_last_error()); \
      std::exit(3);                                                               \
    }                                                                             \
  } while (0)

using Clock = std::chrono::steady_clock;

int main(int argc, char** argv) {
  std::string mode = "gpu-reg", wait = "spin";
  int threads = 32, batch = 256;
  double seconds = 2.0;
  uint64_t arena = 1ull << 30;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&] { return std::string(i + 1 < argc ? argv[++i] : ""); };
    if (a == "--mode") mode = next();
    else if (a == "--threads") threads = std::atoi(next().c_str());
    else if (a == "--batch") batch = std::atoi(next().c_str());
    else if (a == "--seconds") seconds = std::atof(next().c_str());
    else if (a == "--arena-mib") arena = std::strtoull(next().c_str(), nullptr, 10) << 20;
    else if (a == "--wait") wait = next();
  }
  if (wait != "spin" && wait != "block" && wait != "yield") {
    std::fprintf(stderr, "unknown --wait %s\n", wait.c_str());
    return 1;
  }
  const uint64_t seed = 0x3F5C3C00;
  const uint32_t kChunk = 4u << 20, kMaxLen = 64u << 10;
  std::vector<uint8_t> hostv(arena);
  uint8_t* host = hostv.data();
  orc_fill_synth(host, arena, seed, 0, 0);
  const bool cpu = mode == "cpu";
  uint8_t* base = host;  // the read bytes as the hashing path addresses them
  uint8_t* dArena = nullptr;
  if (!cpu) {
    HIP_ASSERT(hipSetDevice(0));
    RC_ASSERT(hf3fs_crc_init(0));
  }
  if (mode == "gpu-reg") {
    void* d = nullptr;
    RC_ASSERT(hf3fs_crc_host_register(host, arena, &d));
    base = (uint8_t*)d;
  } else if (mode == "gpu-hbm") {
    HIP_ASSERT(hipMalloc(&dArena, arena));
    HIP_ASSERT(hipMemcpy(dArena, host, arena, hipMemcpyHostToDevice));
    base = dArena;
  } else if (!cpu) {
    std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 1;
  }

  struct Result {
    uint64_t ios = 0, batches = 0, bytes = 0, bad = 0, checked = 0;
    std::vector<float> lat_us;  // per reaped batch
  };
  std::vector<Result> res(threads);
  std::atomic<bool> go{false}, stop{false};
  std::atomic<int> ready{0};
  auto worker = [&](int t) {
    std::mt19937_64 rng(7000 + t);
    Result& r = res[t];
    r.lat_us.reserve(1 << 18);
    hipStream_t s = nullptr;
    hipEvent_t done = nullptr;
    hf3fs_crc_read_io* rec = nullptr;  // pinned + mapped: filled by this thread, completed by the kernels
    hf3fs_crc_read_io* drec = nullptr;
    std::vector<hf3fs_crc_read_io> cpu_rec;
    if (!cpu) {
      HIP_ASSERT(hipSetDevice(0));
      HIP_ASSERT(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      HIP_ASSERT(hipEventCreateWithFlags(&done, hipEventDisableTiming | (wait == "block" ? hipEventBlockingSync : 0)));
      HIP_ASSERT(hipHostMalloc((void**)&rec, batch * sizeof(hf3fs_crc_read_io), hipHostMallocMapped));
      HIP_ASSERT(hipHostGetDevicePointer((void**)&drec, rec, 0));
    } else {
      cpu_rec.resize(batch);
      rec = cpu_rec.data();
    }
    std::vector<uint64_t> offs(batch);
    ready.fetch_add(1);
    while (!go.load()) std::this_thread::yield();
    while (!stop.load()) {
      // a reaped batch of completions: the records AioReadJob carries
      uint64_t bytes = 0;
      for (int i = 0; i < batch; ++i) {
        const uint32_t len = 4096u << (rng() % 5);
        const uint64_t off = (rng() % ((arena - len) / 4096)) * 4096;
        offs[i] = off;
        hf3fs_crc_read_io& io = rec[i];
        std::memset(&io, 0, sizeof(io));
        io.data = (uint64_t)(base + off);
        const bool full = (rng() & 15) == 0;
        io.offset = full ? 0 : (uint32_t)(4096 * (1 + rng() % 512));
        io.length = len;
        io.chunk_len = full ? len : kChunk;
        io.batch_checksum_type = HF3FS_CHECKSUM_CRC32C;
        io.chunk_checksum_type = HF3FS_CHECKSUM_CRC32C;
        io.chunk_checksum = 0x12345678u + i;
        bytes += full ? 0 : len;
      }
      auto t0 = Clock::now();
      if (cpu) {
        for (int i = 0; i < batch; ++i) {
          hf3fs_crc_read_io& io = rec[i];
          orc_checksum out;
          io.status = orc_read_result_checksum(io.batch_checksum_type, {io.chunk_checksum_type, io.chunk_checksum},
                                               io.offset, io.length, io.chunk_len, host + offs[i], nullptr, 0, &out);
          io.out_checksum = out.value;
          io.out_checksum_type = out.type;
        }
      } else {
        RC_ASSERT(hf3fs_crc_read_result_batch(HF3FS_CHECKSUM_CRC32C, drec, batch, kMaxLen, s));
        if (wait == "spin") {
          HIP_ASSERT(hipStreamSynchronize(s));
        } else if (wait == "block") {
          HIP_ASSERT(hipEventRecord(done, s));
          HIP_ASSERT(hipEventSynchronize(done));
        } else {
          RC_ASSERT(hf3fs_crc_stream_wait(s, 20));
        }
      }
      auto t1 = Clock::now();
      r.lat_us.push_back(std::chrono::duration<float, std::micro>(t1 - t0).count());
      if (r.batches < 64) {
        for (int i = 0; i < batch; ++i) {
          const hf3fs_crc_read_io& io = rec[i];
          const bool full = io.offset == 0 && io.length == io.chunk_len;
          const uint32_t want = full ? io.chunk_checksum : orc_crc32c_hw(~0u, host + offs[i], io.length);
          ++r.checked;
          if (io.status != 0 || io.out_checksum != want || io.out_checksum_type != HF3FS_CHECKSUM_CRC32C) ++r.bad;
        }
      }
      ++r.batches;
      r.ios += batch;
      r.bytes += bytes;
    }
    if (s) {
      (void)hipEventDestroy(done);
      (void)hipStreamDestroy(s);
      (void)hipHostFree(rec);
    }
  };
  std::vector<std::thread> ths;
  for (int t = 0; t < threads; ++t) ths.emplace_back(worker, t);
  while (ready.load() < threads) std::this_thread::yield();
  auto t0 = Clock::now();
  go = true;
  std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
  stop = true;
  for (auto& th : ths) th.join();
  const double el = std::chrono::duration<double>(Clock::now() - t0).count();

  uint64_t ios = 0, batches = 0, bytes = 0, bad = 0, checked = 0;
  std::vector<float> lat;
  for (auto& r : res) {
    ios += r.ios;
    batches += r.batches;
    bytes += r.bytes;
    bad += r.bad;
    checked += r.checked;
    lat.insert(lat.end(), r.lat_us.begin(), r.lat_us.end());
  }
  std::sort(lat.begin(), lat.end());
  auto pct = [&](double p) { return lat.empty() ? 0.0 : (double)lat[std::min(lat.size() - 1, (size_t)(p * lat.size()))]; };
  if (mode == "gpu-reg") RC_ASSERT(hf3fs_crc_host_unregister(host));
  if (dArena) (void)hipFree(dArena);
  std::printf(
      "{\"mode\": \"%s\", \"threads\": %d, \"batch\": %d, \"seconds\": %.3f, \"ios\": %llu, \"ios_per_s\": %.0f, "
      "\"hashed_gbs\": %.2f, \"batch_lat_us_p50\": %.1f, \"batch_lat_us_p99\": %.1f, \"batches\": %llu, "
      "\"checked\": %llu, \"bad\": %llu, \"wait\": \"%s\"}\n",
      mode.c_str(), threads, batch, el, (unsigned long long)ios, ios / el, bytes / el / 1e9, pct(0.5), pct(0.99),
      (unsigned long long)batches, (unsigned long long)checked, (unsigned long long)bad, wait.c_str());
  return bad ? 4 : 0;
}
