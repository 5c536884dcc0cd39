// C++ drop-in test: the reference's own checksum tests rewritten against
// include/hf3fs/storage/ChecksumInfo.h (GPU-backed) with folly::crc32c replaced
// by the CPU oracle (oracle/crc_oracle.c) as the independent checker.
//   tests/common/utils/TestFolly.cc:9-23                      -> FollyCombine
//   tests/storage/store/TestCommonStruct.cc:46-55 (semantics)  -> CreateCombine
//   tests/storage/client/TestStorageClientInterface.cc:357-462 -> VerifyChecksum
// Built by 3fs_amd/build.py (hipcc, host code only) and run by tests/test_cpp_dropin.py.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <random>
#include <thread>
#include <vector>

#include "../../include/hf3fs/storage/ChecksumInfo.h"
extern "C" {
#include "../../oracle/crc_oracle.h"
}

using hf3fs::storage::ChecksumInfo;
using hf3fs::storage::ChecksumType;

static int g_fail = 0;
#define EXPECT_EQ(a, b)                                                                                   \
  do {                                                                                                    \
    auto _a = (a);                                                                                        \
    auto _b = (b);                                                                                        \
    if (!(_a == _b)) {                                                                                    \
      std::fprintf(stderr, "%s:%d: EXPECT_EQ(%s, %s) failed: %llx vs %llx\n", __FILE__, __LINE__, #a, #b, \
                   (unsigned long long)_a, (unsigned long long)_b);                                       \
      ++g_fail;                                                                                           \
    }                                                                                                     \
  } while (0)
#define HIP_ASSERT(x)                                                                \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));             \
      std::exit(2);                                                                  \
    }                                                                                \
  } while (0)

namespace folly {  // the checker: folly semantics restated by the oracle
inline uint32_t crc32c(const uint8_t *d, size_t n, uint32_t start = ~0U) { return orc_crc32c_hw(start, d, n); }
inline uint32_t crc32c_combine(uint32_t a, uint32_t b, size_t n) { return orc_crc32c_combine(a, b, n); }
}  // namespace folly

static void FollyCombine() {
  std::string a = "hello", b = "world";
  auto crc1 = folly::crc32c(reinterpret_cast<const uint8_t *>(a.data()), a.size(), 0);
  auto crc2 = folly::crc32c(reinterpret_cast<const uint8_t *>(b.data()), b.size(), 0);
  // the product's combine against the checker
  EXPECT_EQ(hf3fs_crc32c_combine(crc1, crc2, b.size()),
            folly::crc32c(reinterpret_cast<const uint8_t *>(b.data()), b.size(), crc1));
  std::vector<uint8_t> zeros(1 << 20, 0);
  EXPECT_EQ(~ChecksumInfo::create(ChecksumType::CRC32C, zeros.data(), zeros.size()).value, 0x14298C12u);
  EXPECT_EQ(~ChecksumInfo::create(ChecksumType::CRC32C, zeros.data(), 1).value, 0x527D5351u);
  const char *kat = "123456789";
  EXPECT_EQ(~ChecksumInfo::create(ChecksumType::CRC32C, (const uint8_t *)kat, 9).value, 0xE3069283u);
}

static void CreateCombine() {
  std::mt19937_64 rng(7);
  std::vector<uint8_t> d(3 * ChecksumInfo::kChunkSize + 12345);
  for (auto &x : d) x = (uint8_t)rng();
  auto full = ChecksumInfo::create(ChecksumType::CRC32C, d.data(), d.size());
  EXPECT_EQ(full.value, folly::crc32c(d.data(), d.size()));
  EXPECT_EQ((int)full.type, (int)ChecksumType::CRC32C);
  // split + combine == whole
  size_t cut = 777777;
  auto a = ChecksumInfo::create(ChecksumType::CRC32C, d.data(), cut);
  auto b = ChecksumInfo::create(ChecksumType::CRC32C, d.data() + cut, d.size() - cut);
  EXPECT_EQ((bool)a.combine(b, d.size() - cut), true);
  EXPECT_EQ(a == full, true);
  // NONE / empty / mismatch semantics
  auto none = ChecksumInfo::create(ChecksumType::NONE, d.data(), d.size());
  EXPECT_EQ(none == (ChecksumInfo{ChecksumType::NONE, 0}), true);
  auto empty = ChecksumInfo::create(ChecksumType::CRC32C, (const uint8_t *)nullptr, 0);  // as ChunkReplica.cc:329
  EXPECT_EQ(empty.value, ~0u);
  ChecksumInfo c32 = ChecksumInfo::create(ChecksumType::CRC32, d.data(), 100);
  EXPECT_EQ(c32.value, orc_crc32_sw(~0u, d.data(), 100));
  auto mismatch = full.combine(c32, 100);
  EXPECT_EQ((bool)mismatch, false);
  EXPECT_EQ(mismatch.error().code(), HF3FS_CRC_CHECKSUM_MISMATCH);
  ChecksumInfo n0{};
  EXPECT_EQ((bool)n0.combine(c32, 0), true);
  EXPECT_EQ(n0 == ChecksumInfo{}, true);
  EXPECT_EQ((bool)n0.combine(c32, 100), true);
  EXPECT_EQ(n0 == c32, true);
}

// ---- the call shapes of ChunkReplica::updateChecksum (ChunkReplica.cc:319-394),
// written against this header: ChunkInfo / ChunkFileView / UpdateIO are minimal
// stand-ins with the members that body touches; the ChecksumInfo calls are the
// reference's (create with a null buffer, combine -> Result<Void> checked with
// `!`, .error(), makeError(...), Result<ChecksumInfo> with ->).
namespace mirror {
using hf3fs::makeError;
using hf3fs::Result;
using hf3fs::Void;
#define UNLIKELY(x) __builtin_expect(!!(x), 0)
struct ChunkMetadata {
  uint32_t size = 0;
  ChecksumType checksumType = ChecksumType::NONE;
  uint32_t checksumValue = 0;
  ChecksumInfo checksum() const { return ChecksumInfo{checksumType, checksumValue}; }
};
struct ChunkFileView {  // ChunkFileView::checksum(type, length, offset, meta) over the chunk bytes
  const std::vector<uint8_t> *bytes;
  Result<ChecksumInfo> checksum(ChecksumType type, uint32_t length, uint32_t offset, const ChunkMetadata &) const {
    if ((size_t)offset + length > bytes->size()) return makeError(4010, "read past the chunk");
    return ChecksumInfo::create(type, bytes->data() + offset, length);
  }
};
struct ChunkInfo {
  ChunkMetadata meta;
  ChunkFileView view;
};
struct UpdateIO {
  uint32_t offset = 0, length = 0;
  bool truncate = false, extend = false;
  ChecksumInfo checksum;
  bool isTruncate() const { return truncate; }
  bool isExtend() const { return extend; }
};

Result<Void> updateChecksum(ChunkInfo &chunkInfo, UpdateIO writeIO, uint32_t chunkSizeBeforeWrite,
                            bool isAppendWrite) {
  ChunkMetadata &meta = chunkInfo.meta;
  auto chunkChecksum = meta.checksum();
  bool combineChecksum = chunkSizeBeforeWrite > 0 && isAppendWrite;
  if (writeIO.isTruncate() || writeIO.isExtend()) {
    writeIO.checksum = ChecksumInfo::create(meta.checksumType, (const uint8_t *)nullptr, 0);
    writeIO.offset = meta.size;
    writeIO.length = 0;
  }
  if (writeIO.checksum.type == ChecksumType::NONE || meta.size == 0) {
    meta.checksumValue = 0;
  } else if (writeIO.offset == 0 && writeIO.length == meta.size) {
    meta.checksumValue = writeIO.checksum.value;
  } else if (writeIO.checksum.type == chunkChecksum.type && combineChecksum) {
    auto combinResult = chunkChecksum.combine(writeIO.checksum, writeIO.length);
    if (UNLIKELY(!combinResult)) {
      std::fprintf(stderr, "combine failed: %s\n", combinResult.error().describe().c_str());
      return makeError(combinResult.error());
    }
    meta.checksumValue = chunkChecksum.value;
  } else {
    auto prefixChecksum = chunkInfo.view.checksum(writeIO.checksum.type, writeIO.offset, 0, meta);
    if (UNLIKELY(!prefixChecksum)) return makeError(std::move(prefixChecksum.error()));
    uint32_t suffixStart = std::min(writeIO.offset + writeIO.length, meta.size);
    uint32_t suffixLength = meta.size - suffixStart;
    auto suffixChecksum = chunkInfo.view.checksum(writeIO.checksum.type, suffixLength, suffixStart, meta);
    if (UNLIKELY(!suffixChecksum)) return makeError(std::move(suffixChecksum.error()));
    prefixChecksum->combine(writeIO.checksum, writeIO.length);
    prefixChecksum->combine(*suffixChecksum, suffixLength);
    meta.checksumValue = prefixChecksum->value;
  }
  meta.checksumType = writeIO.checksum.type;
  return Void{};
}
}  // namespace mirror

// The mirrored body against the oracle's restatement of the same function, over
// random writes / appends / truncates with mixed chunk and write types.
static void UpdateChecksumCallShapes() {
  std::mt19937_64 rng(321);
  for (int it = 0; it < 60; ++it) {
    const uint32_t cap = 300000;
    std::vector<uint8_t> bytes(cap);
    for (auto &x : bytes) x = (uint8_t)rng();
    const uint32_t before = (uint32_t)(rng() % cap);
    const ChecksumType ctype = (ChecksumType)(rng() % 3), wtype = (ChecksumType)(rng() % 3);
    mirror::ChunkInfo info{{before, ctype, 0}, {&bytes}};
    info.meta.checksumValue = ctype == ChecksumType::NONE ? 0 : ChecksumInfo::create(ctype, bytes.data(), before).value;
    mirror::UpdateIO io;
    const int kind = (int)(rng() % 4);  // 0 write, 1 append, 2 truncate, 3 extend
    uint32_t after = before;
    if (kind == 2 || kind == 3) {
      io.truncate = kind == 2;
      io.extend = kind == 3;
      after = kind == 2 ? (uint32_t)(rng() % (before + 1)) : before + (uint32_t)(rng() % (cap - before));
    } else {
      io.offset = kind == 1 ? before : (uint32_t)(rng() % cap);
      io.length = 1 + (uint32_t)(rng() % (cap - io.offset));
      io.checksum = ChecksumInfo::create(wtype, bytes.data() + io.offset, io.length);
      after = std::max(before, io.offset + io.length);
    }
    info.meta.size = after;
    const orc_checksum chunk_ck{(uint8_t)ctype, ChecksumInfo{ctype, info.meta.checksumValue}.value};
    const bool isAppend = io.offset == before;
    auto r = mirror::updateChecksum(info, io, before, isAppend);
    orc_checksum want{};
    const int orc_rc = orc_replica_update_checksum(bytes.data(), after, chunk_ck,
                                                   orc_checksum{(uint8_t)io.checksum.type, io.checksum.value},
                                                   io.offset, io.length, kind >= 2, before, isAppend, &want);
    EXPECT_EQ((bool)r, orc_rc == 0);
    if (r && orc_rc == 0) {
      EXPECT_EQ((int)info.meta.checksumType, (int)want.type);
      EXPECT_EQ(info.meta.checksumValue, want.value);
    }
  }
  // serde form (TestCommonStruct.cc:46-55)
  ChecksumInfo ser{ChecksumType::CRC32, 0xff};
  auto out = ser.serialize();
  EXPECT_EQ(out.size(), (size_t)(1 + 1 + 4));
  auto des = ChecksumInfo::deserialize(out.data(), out.size());
  EXPECT_EQ((bool)des, true);
  EXPECT_EQ(*des == ser, true);
  EXPECT_EQ(ChecksumInfo::deserialize(out.data(), 3).error().code(), HF3FS_CRC_SERDE_INSUFFICIENT_LENGTH);
  // tryCreate reports the status create() hands to the device-failure handler
  ChecksumInfo t;
  std::vector<uint8_t> d(1000, 7);
  hf3fs::storage::ChecksumInfo::MemoryDataIterator iter(d.data(), d.size());
  EXPECT_EQ(ChecksumInfo::tryCreate(ChecksumType::CRC32C, &iter, d.size(), &t), HF3FS_CRC_OK);
  EXPECT_EQ(t.value, folly::crc32c(d.data(), d.size()));
}

// ChunkReplica semantics on device: 100 SEQ/JUMP/RAND writes per pattern; after
// each, the chunk checksum equals crc32c(chunk bytes) (TestStorageClientInterface.cc:433-435).
static void VerifyChecksum(uint32_t chunkSize, int mode) {
  std::mt19937_64 rng(chunkSize + mode);
  uint8_t *dChunk = nullptr, *dPayload = nullptr;
  hf3fs_crc_update_io *dIo = nullptr;
  HIP_ASSERT(hipMalloc(&dChunk, chunkSize));
  HIP_ASSERT(hipMalloc(&dPayload, chunkSize));
  HIP_ASSERT(hipMalloc(&dIo, sizeof(hf3fs_crc_update_io)));
  for (int pattern = 1; pattern <= 3; ++pattern) {  // SEQWRITE, JUMPWRITE, RANDWRITE
    std::vector<uint8_t> chunkData;
    HIP_ASSERT(hipMemset(dChunk, 0xAB, chunkSize));  // garbage beyond the chunk size
    static std::vector<uint8_t> prevData;  // the last payload staged (any earlier call): diagnostics
    uint32_t size = 0;
    ChecksumInfo meta{ChecksumType::NONE, 0};
    size_t offset = 0, length = 0;
    for (int w = 1; w <= 100; ++w) {
      if (pattern == 1) offset += length;
      else if (pattern == 2) offset += length + (length / 2 ? rng() % (length / 2 + 1) : 0);
      else offset = rng() % chunkSize;
      if (offset + 1 >= chunkSize) continue;
      length = 1 + rng() % ((chunkSize - offset) / 2);
      std::vector<uint8_t> writeData(length);
      for (auto &x : writeData) x = (uint8_t)rng();
      auto local = ChecksumInfo::create(ChecksumType::CRC32C, writeData.data(), length);  // client create
      EXPECT_EQ(folly::crc32c(writeData.data(), length), local.value);
      HIP_ASSERT(hipMemcpy(dPayload, writeData.data(), length, hipMemcpyHostToDevice));  // pageable, null stream
      hf3fs_crc_update_io io{};
      io.chunk = (uint64_t)dChunk;
      io.payload = (uint64_t)dPayload;
      io.offset = (uint32_t)offset;
      io.length = (uint32_t)length;
      io.chunk_size = size;
      io.update_type = HF3FS_UPDATE_WRITE;
      io.chunk_checksum_type = (uint8_t)meta.type;
      io.chunk_checksum = meta.value;
      io.write_checksum_type = (uint8_t)local.type;
      io.write_checksum = local.value;
      HIP_ASSERT(hipMemcpy(dIo, &io, sizeof(io), hipMemcpyHostToDevice));
      EXPECT_EQ(hf3fs::storage::gpu::updateChunks(ChecksumType::CRC32C, dIo, 1, chunkSize, mode), 0);
      HIP_ASSERT(hipMemcpy(&io, dIo, sizeof(io), hipMemcpyDeviceToHost));
      EXPECT_EQ(io.status, 0);
      if (io.status != 0) {
        std::fprintf(stderr, "  mode=%d chunkSize=%u pattern=%d write=%d offset=%zu length=%zu size=%u "
                     "client=%08x local_recheck=%08x\n", mode, chunkSize, pattern, w, offset, length, size,
                     local.value, folly::crc32c(writeData.data(), length));
        // what the device read as the descriptor: prep writes the IO it read back whole
        std::fprintf(stderr, "  device_io: offset=%u length=%u chunk_size=%u type=%u wtype=%u wck=%08x ctype=%u "
                     "cck=%08x out_size=%u case=%u\n", io.offset, io.length, io.chunk_size, io.update_type,
                     io.write_checksum_type, io.write_checksum, io.chunk_checksum_type, io.chunk_checksum,
                     io.out_size, io.checksum_case);
        std::fprintf(stderr, "  previous payload crc=%08x (len %zu)\n",
                     prevData.empty() ? 0u : folly::crc32c(prevData.data(), std::min(prevData.size(), length)),
                     prevData.size());
        // diagnostics: device hash of the staged payload, payload bytes, and a retry of the same IO
        std::vector<uint8_t> staged(length);
        HIP_ASSERT(hipMemcpy(staged.data(), dPayload, length, hipMemcpyDeviceToHost));
        uint64_t *dDesc = nullptr;
        uint32_t *dOut = nullptr;
        HIP_ASSERT(hipMalloc(&dDesc, 16));
        HIP_ASSERT(hipMalloc(&dOut, 4));
        uint64_t desc[2] = {(uint64_t)dPayload, length};
        HIP_ASSERT(hipMemcpy(dDesc, desc, 16, hipMemcpyHostToDevice));
        int rc = hf3fs_crc_create_batch(1, (const void *const *)dDesc, dDesc + 1, nullptr, dOut, 1, length, nullptr);
        uint32_t dev = 0;
        HIP_ASSERT(hipMemcpy(&dev, dOut, 4, hipMemcpyDeviceToHost));
        std::fprintf(stderr, "  staged_ok=%d device_create=%08x rc=%d\n", (int)(staged == writeData), dev, rc);
        hf3fs_crc_update_io again = io;
        again.status = 0;
        again.chunk_size = size;
        again.chunk_checksum_type = (uint8_t)meta.type;
        again.chunk_checksum = meta.value;
        HIP_ASSERT(hipMemcpy(dIo, &again, sizeof(again), hipMemcpyHostToDevice));
        hf3fs::storage::gpu::updateChunks(ChecksumType::CRC32C, dIo, 1, chunkSize, mode);
        HIP_ASSERT(hipMemcpy(&again, dIo, sizeof(again), hipMemcpyDeviceToHost));
        std::fprintf(stderr, "  retry status=%d out=%08x\n", again.status, again.out_checksum);
        HIP_ASSERT(hipFree(dDesc));
        HIP_ASSERT(hipFree(dOut));
      }
      prevData = writeData;
      if (offset + length > chunkData.size()) chunkData.resize(offset + length);
      std::memcpy(&chunkData[offset], writeData.data(), length);
      size = io.out_size;
      meta = ChecksumInfo{(ChecksumType)io.out_checksum_type, io.out_checksum};
      EXPECT_EQ((size_t)size, chunkData.size());
      EXPECT_EQ(folly::crc32c(chunkData.data(), chunkData.size()), meta.value);
      std::vector<uint8_t> back(size);
      HIP_ASSERT(hipMemcpy(back.data(), dChunk, size, hipMemcpyDeviceToHost));
      EXPECT_EQ(back == chunkData, true);
    }
  }
  HIP_ASSERT(hipFree(dChunk));
  HIP_ASSERT(hipFree(dPayload));
  HIP_ASSERT(hipFree(dIo));
}

// 32 threads, each creating the checksum of its own reads one IO at a time
// (AioReadJob::setResult on 32 AioReadWorker threads, BatchReadJob.cc:30-35),
// through one gpu::Coalescer; every value equals folly::crc32c of the bytes.
static void CoalescedCreate() {
  std::mt19937_64 rng(99);
  std::vector<uint8_t> d(8 << 20);
  for (auto &x : d) x = (uint8_t)rng();
  hf3fs::storage::gpu::Coalescer co;
  EXPECT_EQ(co.status(), HF3FS_CRC_OK);
  std::atomic<int> bad{0};
  std::vector<std::thread> ths;
  for (int t = 0; t < 32; ++t)
    ths.emplace_back([&, t] {
      std::mt19937_64 r(t);
      for (int k = 0; k < 40; ++k) {
        size_t len = (r() % 3 == 0) ? r() % 300 : (size_t(4096) << (r() % 5)) + r() % 7;
        size_t off = r() % (d.size() - len);
        auto c = co.create(ChecksumType::CRC32C, d.data() + off, len);
        if (c.type != ChecksumType::CRC32C || c.value != folly::crc32c(d.data() + off, len)) ++bad;
      }
    });
  for (auto &th : ths) th.join();
  EXPECT_EQ(bad.load(), 0);
  uint64_t st[4];
  EXPECT_EQ(hf3fs_crc_coalescer_stats(co.handle(), st), HF3FS_CRC_OK);
  EXPECT_EQ(st[0] <= 32 * 40, true);
}

int main() {
  FollyCombine();
  CoalescedCreate();
  CreateCombine();
  UpdateChecksumCallShapes();
  for (int mode : {HF3FS_UPDATE_MODE_REFERENCE, HF3FS_UPDATE_MODE_DELTA}) {
    VerifyChecksum(512, mode);
    VerifyChecksum(128 * 1024, mode);
  }
  // the update self-check's record: a contradicted verify would show here
  hf3fs_crc_anomaly an{};
  if (hf3fs_crc_anomalies(0, &an, 0) == 0) {
    std::printf("self-check anomalies=%u kinds=%#x\n", an.count, an.kinds);
    if (an.count) {
      std::printf("  first: io=%llu pipeline=%#x hash=%08x rehash=%08x client=%08x pre_max=%u pre_len=%llu len=%llu\n",
                  (unsigned long long)an.io, an.pipeline, an.pipeline_hash, an.rehash, an.client_checksum, an.pre_max,
                  (unsigned long long)an.pre_len, (unsigned long long)an.length);
      ++g_fail;
    }
  }
  hf3fs_crc_shutdown();
  std::printf("%s (%d failures)\n", g_fail ? "FAILED" : "ALL OK", g_fail);
  return g_fail ? 1 : 0;
}
