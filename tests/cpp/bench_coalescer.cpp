// Per-IO checksum throughput from many threads: the shape
// of 3FS's read path, where each of 32 AioReadWorker threads hashes one
// completed read at a time (src/storage/aio/BatchReadJob.cc:24-35).
//
// Modes (one per run, JSON line on stdout):
//   coalesced-hbm   blocks in HBM, hf3fs_crc_coalescer_create_one per IO
//   coalesced-reg   blocks in hipHostRegister'ed host memory (zero copy)
//   coalesced-copy  blocks in plain host memory, HF3FS_CRC_REQ_HOST_COPY
//   service-hbm     blocks in HBM, coalescer in service mode (persistent kernel polling a ring)
//   service-reg     same, blocks in registered host memory
//   service-copy    same, blocks copied into the ring's pinned per-slot stage
//   direct-hbm      one hf3fs_crc_create_batch(n = 1) launch + sync per IO (no coalescing)
//   cpu             the reference's per-IO CPU path: the oracle's SSE4.2
//                   restatement of folly::crc32c on the calling thread
// Block sizes are uniform over {4,8,16,32,64} KiB at 4 KiB-aligned offsets of
// a 1 GiB arena filled with the synthetic generator (BASELINE config 5 sizes).
// The first 32 results of every thread are checked against the oracle.
//
// Built by 3fs_amd/build.py (host code only); run by bench_suite.py.
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
#define RC_ASSERT(x)                                                                 \
  do {                                                                               \
    int rc = (x);                                                                    \
    if (rc) {                                                                        \
      std::fprintf(stderr, "%s failed: %d %s\n", #x, rc, hf3fs_crc_last_error()); \
      std::exit(3);                                                                  \
    }                                                                                \
  } while (0)

using Clock = std::chrono::steady_clock;

int main(int argc, char** argv) {
  std::string mode = "coalesced-hbm";
  int threads = 32;
  double seconds = 2.0;
  uint32_t max_wait_us = 0;
  uint32_t service_wgs = 32;
  uint64_t arena = 1ull << 30;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&] { return std::string(i + 1 < argc ? argv[++i] : ""); };
    if (a == "--mode") mode = next();
    else if (a == "--threads") threads = std::atoi(next().c_str());
    else if (a == "--seconds") seconds = std::atof(next().c_str());
    else if (a == "--max-wait-us") max_wait_us = (uint32_t)std::atoi(next().c_str());
    else if (a == "--arena-mib") arena = std::strtoull(next().c_str(), nullptr, 10) << 20;
    else if (a == "--service-wgs") service_wgs = (uint32_t)std::atoi(next().c_str());
  }
  const uint64_t seed = 0x3F5C3C00;
  std::vector<uint8_t> hostv(arena);
  uint8_t* host = hostv.data();
  orc_fill_synth(host, arena, seed, 0, 0);

  const bool cpu = mode == "cpu";
  uint8_t* base = nullptr;  // address handed to the hashing path
  uint8_t* dArena = nullptr;
  if (!cpu) {
    HIP_ASSERT(hipSetDevice(0));
    RC_ASSERT(hf3fs_crc_init(0));
  }
  const bool service = mode.rfind("service", 0) == 0;
  if (service) mode = "coalesced" + mode.substr(7);  // same data placement as the batch modes
  if (mode == "coalesced-hbm" || mode == "direct-hbm") {
    HIP_ASSERT(hipMalloc(&dArena, arena));
    RC_ASSERT(hf3fs_crc_fill_synth(dArena, arena, arena, 1, seed, 0, nullptr));
    HIP_ASSERT(hipDeviceSynchronize());
    base = dArena;
  } else if (mode == "coalesced-reg") {
    void* d = nullptr;
    RC_ASSERT(hf3fs_crc_host_register(host, arena, &d));
    base = (uint8_t*)d;
  } else if (mode == "coalesced-copy" || cpu) {
    base = host;
  } else {
    std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 1;
  }

  hf3fs_crc_coalescer* co = nullptr;
  const bool coalesced = mode.rfind("coalesced", 0) == 0;
  if (coalesced) {
    hf3fs_crc_coalescer_options o;
    hf3fs_crc_coalescer_default_options(&o);
    o.max_wait_us = max_wait_us;
    if (service) o.service_wgs = service_wgs;
    RC_ASSERT(hf3fs_crc_coalescer_create(&o, &co));
  }
  const uint32_t flags = mode == "coalesced-copy" ? HF3FS_CRC_REQ_HOST_COPY : 0;

  struct Result {
    uint64_t ios = 0, bytes = 0, bad = 0, checked = 0;
    std::vector<float> lat_us;
  };
  std::vector<Result> res(threads);
  std::atomic<bool> go{false}, stop{false};
  std::atomic<int> ready{0};
  auto worker = [&](int t) {
    std::mt19937_64 rng(1000 + t);
    Result& r = res[t];
    r.lat_us.reserve(1 << 20);
    hipStream_t s = nullptr;
    uint64_t* pdesc = nullptr;  // direct mode: [addr, len] pinned + mapped
    uint64_t* ddesc = nullptr;
    uint32_t* dout = nullptr;
    uint32_t* hout = nullptr;
    if (mode == "direct-hbm") {
      HIP_ASSERT(hipSetDevice(0));
      HIP_ASSERT(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      HIP_ASSERT(hipHostMalloc((void**)&pdesc, 16, hipHostMallocMapped));
      HIP_ASSERT(hipHostGetDevicePointer((void**)&ddesc, pdesc, 0));
      HIP_ASSERT(hipMalloc((void**)&dout, 4));
      HIP_ASSERT(hipHostMalloc((void**)&hout, 4, hipHostMallocDefault));
    }
    ready.fetch_add(1);
    while (!go.load()) std::this_thread::yield();
    while (!stop.load()) {
      const uint64_t len = (4096ull << (rng() % 5));
      const uint64_t off = (rng() % ((arena - len) / 4096)) * 4096;
      uint32_t v = 0;
      auto t0 = Clock::now();
      if (cpu) {
        v = orc_crc32c_hw(~0u, host + off, len);
      } else if (coalesced) {
        RC_ASSERT(hf3fs_crc_coalescer_create_one(co, HF3FS_CHECKSUM_CRC32C, base + off, len, ~0u, flags, &v));
      } else {
        pdesc[0] = (uint64_t)(base + off);
        pdesc[1] = len;
        RC_ASSERT(hf3fs_crc_create_batch(HF3FS_CHECKSUM_CRC32C, (const void* const*)ddesc, ddesc + 1, nullptr, dout,
                                         1, len, s));
        HIP_ASSERT(hipMemcpyAsync(hout, dout, 4, hipMemcpyDeviceToHost, s));
        HIP_ASSERT(hipStreamSynchronize(s));
        v = *hout;
      }
      auto t1 = Clock::now();
      r.lat_us.push_back(std::chrono::duration<float, std::micro>(t1 - t0).count());
      if (r.checked < 32) {
        ++r.checked;
        if (v != orc_crc32c_hw(~0u, host + off, len)) ++r.bad;
      }
      ++r.ios;
      r.bytes += len;
    }
    if (s) {
      (void)hipStreamDestroy(s);
      (void)hipHostFree(pdesc);
      (void)hipFree(dout);
      (void)hipHostFree(hout);
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

  uint64_t ios = 0, bytes = 0, bad = 0, checked = 0;
  std::vector<float> lat;
  for (auto& r : res) {
    ios += r.ios;
    bytes += r.bytes;
    bad += r.bad;
    checked += r.checked;
    lat.insert(lat.end(), r.lat_us.begin(), r.lat_us.end());
  }
  std::sort(lat.begin(), lat.end());
  auto pct = [&](double p) { return lat.empty() ? 0.0 : (double)lat[std::min(lat.size() - 1, (size_t)(p * lat.size()))]; };
  uint64_t st[4] = {0, 0, 0, 0};
  if (co) {
    RC_ASSERT(hf3fs_crc_coalescer_stats(co, st));
    hf3fs_crc_coalescer_destroy(co);
  }
  if (mode == "coalesced-reg") RC_ASSERT(hf3fs_crc_host_unregister(host));
  if (dArena) (void)hipFree(dArena);
  if (service) mode = "service" + mode.substr(9);
  std::printf(
      "{\"mode\": \"%s\", \"threads\": %d, \"seconds\": %.3f, \"ios\": %llu, \"ios_per_s\": %.0f, \"gbs\": %.2f, "
      "\"lat_us_p50\": %.1f, \"lat_us_p99\": %.1f, \"batches\": %llu, \"mean_batch\": %.1f, \"max_batch\": %llu, "
      "\"checked\": %llu, \"bad\": %llu, \"max_wait_us\": %u, \"service_wgs\": %u}\n",
      mode.c_str(), threads, el, (unsigned long long)ios, ios / el, bytes / el / 1e9, pct(0.5), pct(0.99),
      (unsigned long long)st[1], st[1] ? (double)st[0] / st[1] : 0.0, (unsigned long long)st[3],
      (unsigned long long)checked, (unsigned long long)bad, max_wait_us, service ? service_wgs : 0u);
  return bad ? 4 : 0;
}
