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
// combine returns Result<Void> as the reference does, so the call sites
// (ChunkReplica.cc:342-351 `if (!r) ... r.error() ... makeError(r.error())`,
// StorageClientImpl.cc:1630) compile unchanged.  Inside the 3FS tree define
// HF3FS_CRC_USE_HF3FS_RESULT and include common/utils/Result.h first: the real
// hf3fs::Result / makeError are used.  Standalone, a minimal hf3fs::Result,
// Status, Void and makeError with the same member names stand in.
//
// Compiling unchanged is not running as fast: create() of one host buffer is a
// synchronous staged GPU call, 21-158 us per IO against ~2.5 us for the host
// CPU's crc32c at {4..64} KiB.  The GPU pays for batches:
// hf3fs::storage::gpu::updateChunks / verifyBatch / createBatch at UpdateWorker,
// AioReadWorker and client-verify granularity, or the Coalescer below for
// per-IO callers on many threads.
//
// A HIP failure while hashing is not data corruption: create() reports it
// through the device-failure handler (default: print and abort -- a {NONE, 0}
// result would reach ChunkReplica.cc:194-205 as a checksum mismatch and a
// fatal event, ReliableForwarding.cc:263-276), and tryCreate() returns it as a
// status (9001) for callers that handle it themselves.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "../../hf3fs_crc.h"

#ifndef HF3FS_CRC_USE_HF3FS_RESULT
namespace hf3fs {
struct Void {};
// status_code_t + message, as hf3fs::Status (src/common/utils/Status.h)
class Status {
 public:
  explicit Status(int code, std::string msg = {})
      : code_(code),
        msg_(std::move(msg)) {}
  int code() const { return code_; }
  std::string_view message() const { return msg_; }
  std::string describe() const { return std::to_string(code_) + "(" + msg_ + ")"; }

 private:
  int code_;
  std::string msg_;
};
struct Unexpected {
  Status status;
};
inline Unexpected makeError(int code, std::string msg = {}) { return Unexpected{Status(code, std::move(msg))}; }
inline Unexpected makeError(Status s) { return Unexpected{std::move(s)}; }
// The folly::Expected surface the call sites use: bool / !, hasError(), error(),
// value(), *, ->.
template <class T>
class Result {
 public:
  Result(T v)
      : ok_(true),
        value_(std::move(v)),
        status_(0) {}
  Result(Unexpected e)
      : ok_(false),
        status_(std::move(e.status)) {}
  explicit operator bool() const { return ok_; }
  bool hasValue() const { return ok_; }
  bool hasError() const { return !ok_; }
  const Status &error() const { return status_; }
  T &value() { return value_; }
  const T &value() const { return value_; }
  T &operator*() { return value_; }
  const T &operator*() const { return value_; }
  T *operator->() { return &value_; }
  const T *operator->() const { return &value_; }

 private:
  bool ok_;
  T value_{};
  Status status_;
};
}  // namespace hf3fs
#endif

namespace hf3fs::storage {

enum class ChecksumType : uint8_t {
  NONE = 0,
  CRC32C = 1,
  CRC32 = 2,
};

// Device-failure handler of ChecksumInfo::create (see the top of this file).
using DeviceFailureHandler = void (*)(int status, const char *message);
inline void defaultDeviceFailure(int status, const char *message) {
  std::fprintf(stderr, "[hf3fs_crc] device failure %d while hashing: %s\n", status, message);
  std::abort();
}
inline DeviceFailureHandler &deviceFailureHandler() {
  static DeviceFailureHandler h = &defaultDeviceFailure;
  return h;
}

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
  // A device failure goes to deviceFailureHandler() (it must not return a value
  // that reads as corruption); tryCreate reports it instead.
  static ChecksumInfo create(ChecksumType type, DataIterator *iter, size_t length, uint32_t startingChecksum = ~0U) {
    ChecksumInfo out;
    int rc = tryCreate(type, iter, length, &out, startingChecksum);
    if (rc != HF3FS_CRC_OK) {
      deviceFailureHandler()(rc, hf3fs_crc_last_error());
      return ChecksumInfo{ChecksumType::NONE, 0U};  // only if the handler returns
    }
    return out;
  }

  static ChecksumInfo create(ChecksumType type, const uint8_t *buffer, size_t length,
                             uint32_t startingChecksum = ~0U) {
    MemoryDataIterator iter(buffer, length);
    return create(type, &iter, length, startingChecksum);
  }

  // create() with the device status returned: HF3FS_CRC_OK with *out set exactly as
  // create sets it ({NONE, 0} for NONE or a short iterator), or HF3FS_CRC_DEVICE_ERROR.
  static int tryCreate(ChecksumType type, DataIterator *iter, size_t length, ChecksumInfo *out,
                       uint32_t startingChecksum = ~0U) {
    ChecksumInfo checksum{type, startingChecksum};
    size_t iterBytes = 0;
    if (type == ChecksumType::NONE) {
      *out = ChecksumInfo{ChecksumType::NONE, 0U};
      return HF3FS_CRC_OK;
    }
    for (auto data = iter->next(); data.first != nullptr && iterBytes < length; data = iter->next()) {
      iterBytes += data.second;
      if (checksum.type == ChecksumType::NONE) continue;
      const void *buf = data.first;
      const uint64_t len = data.second;
      uint32_t value = 0;
      int rc = hf3fs_crc_create_host(static_cast<uint8_t>(checksum.type), &buf, &len, &checksum.value, &value, 1);
      if (rc != HF3FS_CRC_OK) return rc;
      checksum.value = value;
    }
    if (iterBytes != length) {
      std::fprintf(stderr, "[hf3fs_crc] Iterated bytes %zu not equal to length %zu\n", iterBytes, length);
      *out = ChecksumInfo{ChecksumType::NONE, 0U};
      return HF3FS_CRC_OK;
    }
    *out = checksum;
    return HF3FS_CRC_OK;
  }

  // Common.h:179-198
  Result<Void> combine(const ChecksumInfo &o, size_t length) {
    uint8_t t = static_cast<uint8_t>(type);
    int rc = hf3fs_checksum_combine(&t, &value, static_cast<uint8_t>(o.type), o.value, length);
    if (rc != HF3FS_CRC_OK) return makeError(rc, hf3fs_crc_last_error());
    type = static_cast<ChecksumType>(t);
    return Void{};
  }

  // serde binary form, 6 bytes (TestCommonStruct.cc:46-55; hf3fs_checksum_serialize)
  std::array<uint8_t, 6> serialize() const {
    std::array<uint8_t, 6> out{};
    hf3fs_checksum_serialize(static_cast<uint8_t>(type), value, out.data());
    return out;
  }
  static Result<ChecksumInfo> deserialize(const void *data, size_t n) {
    uint8_t t = 0;
    uint32_t v = 0;
    int rc = hf3fs_checksum_deserialize(data, n, &t, &v, nullptr);
    if (rc != HF3FS_CRC_OK) return makeError(rc, hf3fs_crc_last_error());
    return ChecksumInfo{static_cast<ChecksumType>(t), v};
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

// ChunkReplica::update + updateChecksum for n chunk replicas in HBM.  The default
// REFERENCE mode re-derives from the chunk bytes as the reference does; DELTA
// (faster) trusts the stored checksum (see hf3fs_crc_update_batch).
inline int updateChunks(ChecksumType type, hf3fs_crc_update_io *d_ios, uint64_t n, uint32_t chunkSize,
                        int mode = HF3FS_UPDATE_MODE_REFERENCE, void *stream = nullptr) {
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
  // memory (else HBM or hf3fs_crc_host_register'ed memory).  A device failure goes
  // to deviceFailureHandler(), as in ChecksumInfo::create.
  ChecksumInfo create(ChecksumType type, const void *buffer, size_t length, bool hostCopy = true,
                      uint32_t startingChecksum = ~0U) {
    if (type == ChecksumType::NONE) return ChecksumInfo{ChecksumType::NONE, 0U};
    uint32_t v = 0;
    int rc = co_ ? hf3fs_crc_coalescer_create_one(co_, static_cast<uint8_t>(type), buffer, length, startingChecksum,
                                                  hostCopy ? HF3FS_CRC_REQ_HOST_COPY : 0u, &v)
                 : status_;
    if (rc != HF3FS_CRC_OK) {  // a device failure, not corruption (see the top of this file)
      deviceFailureHandler()(rc, hf3fs_crc_last_error());
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
