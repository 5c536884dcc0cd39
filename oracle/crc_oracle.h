/*
 * crc_oracle.h -- CPU restatement of the 3FS chunk-integrity path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle and the CPU baseline
 * (`cpu_baseline.kind = "port"` in bench.py).  It is never linked into, loaded
 * by, or called from the product library (3fs_amd/lib/libhf3fs_crc.so).  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
 *
 * What it restates (citations are /root/reference paths):
 *   - folly::crc32c / folly::crc32 (folly/hash/Checksum.h, not vendored in the
 *     reference; called at src/fbs/storage/Common.h:158,161): raw reflected
 *     register update, caller-chosen start value, NO final xor.
 *   - folly::crc32c_combine / folly::crc32_combine (Common.h:191,195):
 *     combine(c1, c2, n) = c1 * x^(8n) mod P  xor  c2.
 *   - Rust crate crc32c 0.6.8 (Cargo.lock:399-405; used at
 *     src/storage/chunk_engine/src/core/engine.rs:300 and alloc/chunk.rs:157,
 *     195,213,229,266): finalized CRC (~raw from ~0), append, combine.
 *   - ChecksumInfo::create / combine / == (src/fbs/storage/Common.h:113-202).
 *   - ChunkReplica::updateChecksum (src/storage/store/ChunkReplica.cc:319-394).
 *   - Chunk::safe_write / copy_on_write checksum maintenance
 *     (src/storage/chunk_engine/src/alloc/chunk.rs:89-281).
 *   - AioReadJob::setResult checksum cases (src/storage/aio/BatchReadJob.cc:24-63).
 *   - Checksum::calcSerde (src/common/net/MessageHeader.h:33-37).
 *
 * Parity pins (checked in tests/test_oracle.py): the reference's own known
 * answers in tests/common/utils/TestFolly.cc:11-21 (combine identity asserted;
 * CRC-32C(1 MiB zeros)=0x14298C12 and CRC-32C(1 zero byte)=0x527D5351 logged),
 * the RFC 3720 check value CRC-32C("123456789")=0xE3069283, zlib.crc32 for the
 * IEEE variant, and golden vectors from an independent bitwise Python CRC
 * (tests/golden/make_golden.py).
 */
#ifndef HF3FS_CRC_ORACLE_H
#define HF3FS_CRC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_POLY_CRC32C 0x82F63B78u /* reflected Castagnoli */
#define ORC_POLY_CRC32 0xEDB88320u  /* reflected IEEE 802.3 */

enum { ORC_NONE = 0, ORC_CRC32C = 1, ORC_CRC32 = 2 };
enum {
  ORC_OK = 0,
  ORC_INVALID_ARG = 3,
  ORC_INVALID_FORMAT = 33,
  ORC_CHUNK_READ_FAILED = 4010,
  ORC_CHECKSUM_MISMATCH = 4080,
  ORC_CHUNK_NOT_FOUND = 7007
};

/* ---- folly-equivalent raw register arithmetic ---- */
uint32_t orc_crc32c_sw(uint32_t crc, const uint8_t *p, size_t n);  /* slicing-by-8 */
uint32_t orc_crc32c_hw(uint32_t crc, const uint8_t *p, size_t n);  /* SSE4.2, 3-way interleave */
int orc_have_sse42(void);
/* Carry-less-multiply folding crc32c (PCLMULQDQ 8 x 128-bit lanes / AVX-512 VPCLMULQDQ
 * 16 lanes), the algorithm class of folly's large-buffer x86 dispatch: the CPU-speed bar
 * of bench.py's cpu_baseline.  Same raw register semantics as orc_crc32c_hw. */
uint32_t orc_crc32c_clmul(uint32_t crc, const uint8_t *p, size_t n);     /* best form this CPU has */
uint32_t orc_crc32c_pclmul128(uint32_t crc, const uint8_t *p, size_t n); /* the 128-bit form */
int orc_have_clmul(void);
int orc_have_vpclmul(void);
uint32_t orc_crc32_sw(uint32_t crc, const uint8_t *p, size_t n);   /* IEEE, slicing-by-8 */
uint32_t orc_crc_bitwise(uint32_t crc, const uint8_t *p, size_t n, uint32_t poly); /* tiny cases */

uint32_t orc_gf2_mulmod(uint32_t a, uint32_t b, uint32_t poly); /* reflected: x^0 == 0x80000000 */
uint32_t orc_x8n(uint64_t n, uint32_t poly);                     /* x^(8n) mod P */
uint32_t orc_shift(uint32_t crc, uint64_t n, uint32_t poly);     /* crc fed n zero bytes */
uint32_t orc_crc32c_combine(uint32_t c1, uint32_t c2, uint64_t len2); /* folly::crc32c_combine */
uint32_t orc_crc32_combine(uint32_t c1, uint32_t c2, uint64_t len2);  /* folly::crc32_combine */

/* ---- Rust crc32c 0.6.8 (finalized convention) ---- */
uint32_t orc_rs_crc32c(const uint8_t *p, size_t n);
uint32_t orc_rs_crc32c_append(uint32_t crc, const uint8_t *p, size_t n);
uint32_t orc_rs_crc32c_combine(uint32_t c1, uint32_t c2, size_t len2);

/* ---- ChecksumInfo (Common.h:113-202) ---- */
typedef struct {
  uint8_t type;
  uint32_t value;
} orc_checksum;

orc_checksum orc_checksum_create(uint8_t type, const uint8_t *p, size_t len, uint32_t start);
int orc_checksum_combine(orc_checksum *self, orc_checksum o, size_t len);

/* ---- ChunkReplica::updateChecksum (ChunkReplica.cc:319-394) ----
 * chunk_after: chunk bytes after the write was applied (gap zero-filled),
 * size_after: meta.size after the write; chunk_ck: meta checksum before;
 * write_ck/off/len: UpdateIO; trunc_or_extend: isTruncate()||isExtend();
 * size_before: chunkSizeBeforeWrite; is_append: writeIO.offset == meta.size
 * (evaluated before the write, ChunkReplica.cc:243). Result in *out.        */
int orc_replica_update_checksum(const uint8_t *chunk_after, uint32_t size_after, orc_checksum chunk_ck,
                                orc_checksum write_ck, uint32_t off, uint32_t len, int trunc_or_extend,
                                uint32_t size_before, int is_append, orc_checksum *out);
/* The same, and *kase = the counter the reference bumps for the IO (ChunkReplica.cc:25-28):
 * 1 checksum_none, 2 checksum_reuse, 3 checksum_combine, 4 checksum_read_chunk. */
int orc_replica_update_checksum_case(const uint8_t *chunk_after, uint32_t size_after, orc_checksum chunk_ck,
                                     orc_checksum write_ck, uint32_t off, uint32_t len, int trunc_or_extend,
                                     uint32_t size_before, int is_append, orc_checksum *out, int *kase);

/* ---- chunk engine (chunk.rs) checksum maintenance, finalized convention ----
 * Applies one write to an in-memory chunk image `buf` (capacity >= off+len)
 * of current length *len_io and finalized checksum *ck_io, following
 * Engine::update_chunk's dispatch (engine.rs:373-420) between copy_on_write
 * and safe_write. `capacity` is the allocated chunk capacity. */
int orc_engine_write(uint8_t *buf, uint32_t *len_io, uint32_t *ck_io, uint32_t capacity, const uint8_t *data,
                     uint32_t dlen, uint32_t off, uint32_t data_ck, int truncate, int is_syncing, int exists);
/* The same, and *kase = the engine's checksum counter for the write (chunk.rs:153,156,188,217,233,
 * 273): 1 none, 2 checksum_reuse, 3 checksum_combine, 4 checksum_recalculate. */
int orc_engine_write_case(uint8_t *buf, uint32_t *len_io, uint32_t *ck_io, uint32_t capacity, const uint8_t *data,
                          uint32_t dlen, uint32_t off, uint32_t data_ck, int truncate, int is_syncing, int exists,
                          int *kase);

/* ---- AioReadJob::setResult (BatchReadJob.cc:24-63) ---- */
int orc_read_result_checksum(uint8_t batch_type, orc_checksum chunk_ck, uint32_t read_off, uint32_t read_len,
                             uint32_t chunk_len, const uint8_t *read_data, const uint8_t *full_chunk,
                             int recalculate, orc_checksum *out);

/* ---- Checksum::calcSerde (MessageHeader.h:33-37) ---- */
uint32_t orc_calc_serde(const uint8_t *p, size_t n, int compressed);

/* ---- batched helpers used by the CPU baseline leg of bench.py ---- */
/* Each of n chunks of `len` bytes at base + i*stride; results raw, start ~0.
 * threads<=1 runs inline.  kind: 0 = SSE4.2 3-way, 1 = slicing-by-8, 2 = clmul folding.      */
/* CPU baselines (bench: tests/bench_suite.py "cpu" fields): ChunkReplica::update
 * with the prefix/suffix re-hash per IO (CRC32C; sizes/cks updated in place) and
 * KV-block read verify, over `threads` pthreads. */
void orc_replica_update_batch(uint8_t *chunks, size_t chunk_stride, const uint8_t *payload, size_t payload_stride,
                              uint32_t *sizes, uint32_t *cks, uint32_t *offs, uint32_t *lens, uint32_t *wcks,
                              int32_t *status, size_t n, int threads);
/* FileWrapper::readFile's checksum fold (FileWrapper.cc:119-164), one file per call;
 * blocks in the layout of hf3fs_crc_block_digest (include/hf3fs_crc.h). */
typedef struct {
  uint64_t read_len, block_len;
  uint32_t checksum;
  uint8_t type, missing, res[2];
} orc_block_digest;
typedef struct {
  int32_t status;
  uint8_t type;
  uint32_t value;
} orc_file_result;
int orc_file_digest(const orc_block_digest *b, uint64_t nb, int fill_zero, orc_checksum *out);
void orc_file_digest_batch(const orc_block_digest *blocks, const uint64_t *file_off, uint64_t nfiles, int fill_zero,
                           orc_file_result *out, int threads);
void orc_combine_batch(uint32_t *acc, const uint32_t *crc2, const uint64_t *len2, size_t n, uint32_t poly,
                       int threads);
size_t orc_verify_blocks(const uint8_t *arena, const uint64_t *offs, const uint32_t *lens, const uint32_t *expected,
                         uint8_t *mismatch, size_t n, int threads);
void orc_create_batch(const uint8_t *base, size_t stride, size_t len, size_t n, uint32_t *out, int threads,
                      int kind);

/* Deterministic synthetic data: splitmix64(seed ^ (chunk_id << 32) ^ word_index)
 * as little-endian 8-byte words.  Fills n bytes starting at
 * byte offset `byte_off` within chunk `chunk_id`. */
void orc_fill_synth(uint8_t *dst, size_t n, uint64_t seed, uint64_t chunk_id, uint64_t byte_off);

#ifdef __cplusplus
}
#endif
#endif
