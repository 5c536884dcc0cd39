// host_codec.cc -- the host-only half of the C ABI (include/hf3fs_crc.h): the
// calling thread's last error, the O(log n) checksum algebra on 32-bit values
// (ChecksumInfo::combine, folly::crc32c_combine, Common.h:179-198), and the
// parsers of untrusted bytes -- ChecksumInfo serde (Serde.h:209-223,282-290,
// 422-432,692-702), the serde frame walk (Processor::unpackMsg, Processor.h:
// 85-120; MessageHeader.h:13-37) and the chunk engine's ChunkMeta
// (chunk_engine/src/types/chunk_meta.rs:7-31).  Plain C++ with no HIP: it is
// linked into libhf3fs_crc.so and, with -fsanitize=address,undefined, into
// tests/cpp/fuzz_host_codec (tests/test_sanitizers.py).
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/hf3fs_crc.h"
#include "gf2.h"
#include "internal.h"

namespace hf3fs_crc {

namespace {
thread_local std::string g_last_error;

inline void put_le(uint8_t* p, uint64_t v, int bytes) {
  for (int k = 0; k < bytes; ++k) p[k] = (uint8_t)(v >> (8 * k));
}
inline uint64_t get_le(const uint8_t* p, int bytes) {
  uint64_t v = 0;
  for (int k = 0; k < bytes; ++k) v |= (uint64_t)p[k] << (8 * k);
  return v;
}
}  // namespace

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

int set_error(int code, const char* msg) { return fail(code, "%s", msg); }

}  // namespace hf3fs_crc

using namespace hf3fs_crc;

extern "C" {

const char* hf3fs_crc_last_error(void) { return g_last_error.c_str(); }

uint32_t hf3fs_crc32c_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
  return combine_raw(crc1, crc2, len2, kPolyCrc32c);
}
uint32_t hf3fs_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
  return combine_raw(crc1, crc2, len2, kPolyCrc32);
}
uint32_t hf3fs_crc_shift(uint8_t type, uint32_t crc, uint64_t nbytes) {
  return shift_bytes(crc, nbytes, poly_of(type));
}

int hf3fs_checksum_combine(uint8_t* type, uint32_t* value, uint8_t other_type, uint32_t other_value,
                           uint64_t length) {
  if (!type || !value) return fail(HF3FS_CRC_INVALID_ARG, "null checksum");
  if (*type != kTypeNone && *type != other_type)
    return fail(HF3FS_CRC_CHECKSUM_MISMATCH, "different type %u != %u", *type, other_type);
  if (length == 0) return HF3FS_CRC_OK;
  switch (*type) {
    case kTypeNone:
      *type = other_type;
      *value = other_value;
      return HF3FS_CRC_OK;
    case kTypeCrc32c:
      *value = combine_raw(~*value, other_value, length, kPolyCrc32c);
      return HF3FS_CRC_OK;
    case kTypeCrc32:
      *value = combine_raw(~*value, other_value, length, kPolyCrc32);
      return HF3FS_CRC_OK;
  }
  return fail(HF3FS_CRC_INVALID_ARG, "unknown checksum type %u", *type);
}

uint32_t hf3fs_checksum_serialize(uint8_t type, uint32_t value, uint8_t* out6) {
  // Serde.h:282-290 + 422-432: DownwardBytes prepends, fields are visited last
  // to first, so the table reads forward: varint32 length, type, value (LE).
  out6[0] = 5;
  out6[1] = type;
  put_le(out6 + 2, value, 4);
  return 6;
}

int hf3fs_checksum_deserialize(const void* in, uint64_t n, uint8_t* type, uint32_t* value, uint64_t* consumed) {
  if ((!in && n) || !type || !value) return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  const uint8_t* p = (const uint8_t*)in;
  uint64_t length = 0, k = 0;  // Varint64 table length (Serde.h:209-223, 692-702)
  for (uint32_t shift = 0;; shift += 7) {
    if (shift > 63 || k >= n) return fail(HF3FS_CRC_SERDE_INSUFFICIENT_LENGTH, "varint64 is short");
    const uint64_t byte = p[k++];
    length |= (byte & 127) << shift;
    if (!(byte & 128)) break;
  }
  if (length > n - k)
    return fail(HF3FS_CRC_SERDE_INSUFFICIENT_LENGTH, "string short %llu > %llu", (unsigned long long)length,
                (unsigned long long)(n - k));
  const uint8_t* t = p + k;
  uint8_t ty = kTypeNone;
  uint32_t v = 0;
  if (length >= 1) ty = t[0];  // fields missing at the table's end keep their defaults (:505-506)
  if (length > 1) {
    if (length < 5)
      return fail(HF3FS_CRC_SERDE_INSUFFICIENT_LENGTH, "trivially copyable 4 > %llu", (unsigned long long)(length - 1));
    v = (uint32_t)get_le(t + 1, 4);
  }
  *type = ty;
  *value = v;
  if (consumed) *consumed = k + length;
  return HF3FS_CRC_OK;
}

uint32_t hf3fs_crc32c_combine_fin(uint32_t fin1, uint32_t fin2, uint64_t len2) {
  return combine_raw(fin1, fin2, len2, kPolyCrc32c);
}

int hf3fs_crc_frame_walk(const void* h_buf, uint64_t len, hf3fs_crc_frame* h_frames, uint64_t max_frames,
                         uint64_t* n_frames, uint64_t* consumed) {
  if (!n_frames || !consumed || (!h_buf && len) || (!h_frames && max_frames))
    return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  const uint8_t* p = (const uint8_t*)h_buf;
  uint64_t off = 0, k = 0;
  *n_frames = 0;
  *consumed = 0;
  while (off < len && k < max_frames) {
    if (len - off < 8) return fail(HF3FS_CRC_INVALID_ARG, "message header incomplete at %llu", (unsigned long long)off);
    const uint32_t checksum = (uint32_t)get_le(p + off, 4), size = (uint32_t)get_le(p + off + 4, 4);
    if (len - off - 8 < size)
      return fail(HF3FS_CRC_INVALID_ARG, "message incomplete at %llu: %llu < %u", (unsigned long long)off,
                  (unsigned long long)(len - off - 8), size);
    if ((checksum & 0xfeu) != 0x86u)  // MessageHeader::isSerdeMessage (MessageHeader.h:24)
      return fail(HF3FS_CRC_INVALID_ARG, "message at %llu is not a serde message", (unsigned long long)off);
    h_frames[k] = hf3fs_crc_frame{off + 8, size, checksum, 0u, HF3FS_CRC_OK};
    off += 8 + (uint64_t)size;
    *n_frames = ++k;
    *consumed = off;
  }
  return HF3FS_CRC_OK;
}

int hf3fs_crc_engine_meta_decode(const void* h_bytes, uint64_t n, hf3fs_crc_engine_meta* out, uint64_t* consumed) {
  if (!h_bytes || !out) return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  const uint8_t* p = (const uint8_t*)h_bytes;
  if (n < 1) return fail(HF3FS_CRC_INVALID_ARG, "empty ChunkMeta");
  const uint64_t body = p[0];
  if (body & 0x80) return fail(HF3FS_CRC_INVALID_ARG, "multi-byte derse length is not supported");
  if (n < 1 + body) return fail(HF3FS_CRC_INVALID_ARG, "ChunkMeta truncated: %llu < %llu", (unsigned long long)n,
                                (unsigned long long)(1 + body));
  const uint8_t* q = p + 1;
  const uint64_t fixed = 8 + 4 * 4 + 8 * 4;
  if (body < fixed + 2) return fail(HF3FS_CRC_INVALID_ARG, "ChunkMeta body too short (%llu)", (unsigned long long)body);
  hf3fs_crc_engine_meta m{};
  m.pos = get_le(q, 8);
  m.chain_ver = (uint32_t)get_le(q + 8, 4);
  m.chunk_ver = (uint32_t)get_le(q + 12, 4);
  m.len = (uint32_t)get_le(q + 16, 4);
  m.checksum = (uint32_t)get_le(q + 20, 4);
  m.timestamp = get_le(q + 24, 8);
  m.last_request_id = get_le(q + 32, 8);
  m.last_client_low = get_le(q + 40, 8);
  m.last_client_high = get_le(q + 48, 8);
  const uint64_t elen = q[fixed];
  if (elen & 0x80) return fail(HF3FS_CRC_INVALID_ARG, "multi-byte derse length is not supported");
  if (elen > sizeof(m.etag)) return fail(HF3FS_CRC_INVALID_ARG, "etag longer than %zu bytes", sizeof(m.etag));
  if (fixed + 1 + elen + 1 != body)
    return fail(HF3FS_CRC_INVALID_ARG, "ChunkMeta body length %llu does not match its fields",
                (unsigned long long)body);
  m.etag_len = (uint8_t)elen;
  memcpy(m.etag, q + fixed + 1, elen);
  const uint8_t unc = q[fixed + 1 + elen];
  if (unc > 1) return fail(HF3FS_CRC_INVALID_ARG, "bad bool %u", unc);
  m.uncommitted = unc;
  *out = m;
  if (consumed) *consumed = 1 + body;
  return HF3FS_CRC_OK;
}

int hf3fs_crc_engine_meta_encode(const hf3fs_crc_engine_meta* m, void* h_out, uint64_t cap, uint64_t* written) {
  if (!m || !h_out) return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  if (m->etag_len > sizeof(m->etag) || m->uncommitted > 1) return fail(HF3FS_CRC_INVALID_ARG, "bad ChunkMeta");
  const uint64_t body = 8 + 4 * 4 + 8 * 4 + 1 + m->etag_len + 1;
  if (body >= 0x80) return fail(HF3FS_CRC_INVALID_ARG, "multi-byte derse length is not supported");
  if (cap < 1 + body) return fail(HF3FS_CRC_INVALID_ARG, "output too small");
  uint8_t* p = (uint8_t*)h_out;
  p[0] = (uint8_t)body;
  uint8_t* q = p + 1;
  put_le(q, m->pos, 8);
  put_le(q + 8, m->chain_ver, 4);
  put_le(q + 12, m->chunk_ver, 4);
  put_le(q + 16, m->len, 4);
  put_le(q + 20, m->checksum, 4);
  put_le(q + 24, m->timestamp, 8);
  put_le(q + 32, m->last_request_id, 8);
  put_le(q + 40, m->last_client_low, 8);
  put_le(q + 48, m->last_client_high, 8);
  q[56] = m->etag_len;
  memcpy(q + 57, m->etag, m->etag_len);
  q[57 + m->etag_len] = m->uncommitted;
  if (written) *written = 1 + body;
  return HF3FS_CRC_OK;
}

uint32_t hf3fs_crc_default_etag(uint32_t checksum_fin, char* out8) {
  static const char kHex[] = "0123456789ABCDEF";
  char tmp[8];
  uint32_t k = 0;
  do {
    tmp[k++] = kHex[checksum_fin & 15];
    checksum_fin >>= 4;
  } while (checksum_fin);
  if (out8)
    for (uint32_t i = 0; i < k; ++i) out8[i] = tmp[k - 1 - i];
  return k;
}

}  // extern "C"
