// hf3fs/storage/ChecksumInfo.h -- drop-in for hf3fs::storage::ChecksumInfo
// (src/fbs/storage/Common.h:66-70 ChecksumType, :113-202 ChecksumInfo) whose
// bytes are hashed on MI355X through the C ABI of libhf3fs_crc.so.
//
// Same field layout ({ChecksumType type; uint32_t value;}), same raw folly
// register convention, same special cases:
//   create(NONE, ...)              -> {NONE, 0}
//   create(type, ..., length 0)    -> {type, startingChecksum}
//   iterator yields != length      -> {NONE, 0} + warning
//   combine with a different type  -> error kChecksumMismatch (4080)
//   combine with length 0          -> no-op;  NONE.combine(o) -> copy o
// The reference returns Result<Void> from combine; here CombineResult carries
// the same status code (see INTEGRATION.md for the two-line mapping).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <utility>
#include <vector>

#include "../../hf3fs_crc.h"

namespace hf3fs::storage {

enum class ChecksumType : uint8_t {
  NONE = 0,
  CRC32C = 1,
  CRC32 = 2,
};

struct CombineResult {
  int code = HF3FS_CRC_OK;  // 0 or StorageCode::kChecksumMismatch (4080)
  explicit operator bool() const { return code == HF3FS_CRC_OK; }
  bool hasError() const { return code != HF3FS_CRC_OK; }
};

struct ChecksumInfo {
  ChecksumType type = ChecksumType::NONE;
  uint32_t value{};

  static constexpr size_t kChunkSize = size_t(1) << 20;  // 1_MB (Common.h:118)

  class DataIterator {
   public:
    virtual ~DataIterator() = default;
    virtual std::pair<const uint8_t *, size_t> next() = 0;
  };

  class MemoryDataIterator : public DataIterator {
   public:
    MemoryDataIterator(const uint8_t *buffer, size_t length)
        : buffer_(buffer),
          length_(length) {}

    std::pair<const uint8_t *, size_t> next() override {
      if (length_ == 0) return {nullptr, 0};
      const uint8_t *data = buffer_;
      size_t size = length_ < kChunkSize ? length_ : kChunkSize;
      buffer_ += size;
      length_ -= size;
      return {data, size};
    }

   private:
    const uint8_t *buffer_;
    size_t length_;
  };

  // Common.h:146-172: each iterator slice continues the running register.
  static ChecksumInfo create(ChecksumType type, DataIterator *iter, size_t length, uint32_t startingChecksum = ~0U) {
    ChecksumInfo checksum{type, startingChecksum};
    size_t iterBytes = 0;
    if (type == ChecksumType::NONE) return ChecksumInfo{ChecksumType::NONE, 0U};
    for (auto data = iter->next(); data.first != nullptr && iterBytes < length; data = iter->next()) {
      iterBytes += data.second;
      if (checksum.type == ChecksumType::NONE) continue;
      const void *buf = data.first;
      const uint64_t len = data.second;
      uint32_t out = 0;
      int rc = hf3fs_crc_create_host(static_cast<uint8_t>(checksum.type), &buf, &len, &checksum.value, &out, 1);
      if (rc != HF3FS_CRC_OK) {
        std::fprintf(stderr, "[hf3fs_crc] create failed (%d): %s\n", rc, hf3fs_crc_last_error());
        return ChecksumInfo{ChecksumType::NONE, 0U};
      }
      checksum.value = out;
    }
    if (iterBytes != length) {
      std::fprintf(stderr, "[hf3fs_crc] Iterated bytes %zu not equal to length %zu\n", iterBytes, length);
      return ChecksumInfo{ChecksumType::NONE, 0U};
    }
    return checksum;
  }

  static ChecksumInfo create(ChecksumType type, const uint8_t *buffer, size_t length,
                             uint32_t startingChecksum = ~0U) {
    MemoryDataIterator iter(buffer, length);
    return create(type, &iter, length, startingChecksum);
  }

  // Common.h:179-198
  CombineResult combine(const ChecksumInfo &o, size_t length) {
    uint8_t t = static_cast<uint8_t>(type);
    int rc = hf3fs_checksum_combine(&t, &value, static_cast<uint8_t>(o.type), o.value, length);
    type = static_cast<ChecksumType>(t);
    return CombineResult{rc};
  }

  bool operator==(const ChecksumInfo &) const = default;
};

// ---- batched additions (device-resident bytes, asynchronous on a HIP stream) ----
namespace gpu {

// ChecksumInfo::create for n device buffers; out receives raw values.
inline int createBatch(ChecksumType type, const void *const *d_bufs, const uint64_t *d_lens, uint32_t *d_out,
                       uint64_t n, uint64_t maxLen, void *stream = nullptr, const uint32_t *d_starts = nullptr) {
  return hf3fs_crc_create_batch(static_cast<uint8_t>(type), d_bufs, d_lens, d_starts, d_out, n, maxLen, stream);
}

// Verify n device buffers against expected raw values (mismatch flags + count).
inline int verifyBatch(ChecksumType type, const void *const *d_bufs, const uint64_t *d_lens,
                       const uint32_t *d_expected, uint8_t *d_mismatch, uint32_t *d_count, uint32_t *d_computed,
                       uint64_t n, uint64_t maxLen, void *stream = nullptr) {
  return hf3fs_crc_verify_batch(static_cast<uint8_t>(type), d_bufs, d_lens, d_expected, d_mismatch, d_count,
                                d_computed, n, maxLen, stream);
}

// ChunkReplica::update + updateChecksum for n chunk replicas in HBM.
inline int updateChunks(ChecksumType type, hf3fs_crc_update_io *d_ios, uint64_t n, uint32_t chunkSize,
                        int mode = HF3FS_UPDATE_MODE_DELTA, void *stream = nullptr) {
  return hf3fs_crc_update_batch(static_cast<uint8_t>(type), d_ios, n, chunkSize, mode, stream);
}

// Per-IO creates from many threads batched into shared launches (the shape of
// AioReadJob::setResult, BatchReadJob.cc:24-35, on 32 AioReadWorker threads).
class Coalescer {
 public:
  explicit Coalescer(const hf3fs_crc_coalescer_options *opt = nullptr) { status_ = hf3fs_crc_coalescer_create(opt, &co_); }
  ~Coalescer() { hf3fs_crc_coalescer_destroy(co_); }
  Coalescer(const Coalescer &) = delete;
  Coalescer &operator=(const Coalescer &) = delete;
  int status() const { return status_; }

  // ChecksumInfo::create(type, buffer, length, startingChecksum) for one IO; blocks
  // the calling thread until its batch lands.  hostCopy: `buffer` is plain host
  // memory (else HBM or hf3fs_crc_host_register'ed memory).  {NONE, 0} on failure,
  // as create reports a failed iteration.
  ChecksumInfo create(ChecksumType type, const void *buffer, size_t length, bool hostCopy = true,
                      uint32_t startingChecksum = ~0U) {
    if (type == ChecksumType::NONE || !co_) return ChecksumInfo{ChecksumType::NONE, 0U};
    uint32_t v = 0;
    int rc = hf3fs_crc_coalescer_create_one(co_, static_cast<uint8_t>(type), buffer, length, startingChecksum,
                                            hostCopy ? HF3FS_CRC_REQ_HOST_COPY : 0u, &v);
    if (rc != HF3FS_CRC_OK) {
      std::fprintf(stderr, "[hf3fs_crc] coalesced create failed (%d): %s\n", rc, hf3fs_crc_last_error());
      return ChecksumInfo{ChecksumType::NONE, 0U};
    }
    return ChecksumInfo{type, v};
  }

  hf3fs_crc_coalescer *handle() const { return co_; }

 private:
  hf3fs_crc_coalescer *co_ = nullptr;
  int status_ = HF3FS_CRC_OK;
};

}  // namespace gpu
}  // namespace hf3fs::storage
