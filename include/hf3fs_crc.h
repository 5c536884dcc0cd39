/*
 * hf3fs_crc.h -- C ABI of the MI355X chunk-integrity engine (libhf3fs_crc.so).
 *
 * Drop-in boundary for 3FS's ChecksumInfo path.  Every value
 * is the RAW folly register (no final xor) unless the name ends in _fin, as in
 * the reference: ChecksumInfo.value == folly::crc32c(data, n, ~0U)
 * (src/fbs/storage/Common.h:146-177) and the formatter prints ~value (:771).
 *
 * Conventions
 *   - `stream` is a hipStream_t passed as void* (NULL = the legacy default
 *     stream of the current device).  Batched calls are asynchronous on it and
 *     never retain caller pointers after the stream work completes.
 *   - d_* arguments are device-accessible addresses (hipMalloc'd HBM, or
 *     hipHostRegister'ed / hipHostMalloc'ed host memory mapped to the device);
 *     h_* arguments are plain host memory.
 *   - The calls operate on the current HIP device of the calling thread; the
 *     per-device constant tables are built on first use (or hf3fs_crc_init).
 *   - No exceptions cross the ABI; return values are the reference's status
 *     codes.  Thread-safe and re-entrant (tables are immutable after init).
 */
#ifndef HF3FS_CRC_H
#define HF3FS_CRC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* enum class ChecksumType : uint8_t (src/fbs/storage/Common.h:66-70) */
enum { HF3FS_CHECKSUM_NONE = 0, HF3FS_CHECKSUM_CRC32C = 1, HF3FS_CHECKSUM_CRC32 = 2 };

/* enum class UpdateType : uint8_t (src/fbs/storage/Common.h:51-57) */
enum { HF3FS_UPDATE_WRITE = 1, HF3FS_UPDATE_TRUNCATE = 4, HF3FS_UPDATE_EXTEND = 8 };

/* Status codes: the reference's numeric codes (src/common/utils/StatusCodeDetails.h). */
enum {
  HF3FS_CRC_OK = 0,
  HF3FS_CRC_INVALID_ARG = 3,                  /* StatusCode::kInvalidArg (:24) */
  HF3FS_CRC_INVALID_FORMAT = 33,              /* StatusCode::kInvalidFormat (:42) */
  HF3FS_CRC_SERDE_INSUFFICIENT_LENGTH = 40,   /* StatusCode::kSerdeInsufficientLength (:44) */
  HF3FS_CRC_CHUNK_READ_FAILED = 4010,         /* StorageCode::kChunkReadFailed (:160) */
  HF3FS_CRC_CHECKSUM_MISMATCH = 4080,         /* StorageCode::kChecksumMismatch (:186) */
  HF3FS_CRC_CHUNK_NOT_FOUND = 7007,           /* StorageClientCode::kChunkNotFound (:228) */
  HF3FS_CRC_CLIENT_CHECKSUM_MISMATCH = 7015,  /* StorageClientCode::kChecksumMismatch (:236) */
  HF3FS_CRC_DEVICE_ERROR = 9001               /* HIP runtime failure, or an update IO whose verify the
                                                 self-check contradicted (no reference equivalent) */
};

/* ------------------------------------------------------------------------ */
/* context                                                                   */
/* ------------------------------------------------------------------------ */
int hf3fs_crc_init(int device);            /* optional: build device tables eagerly */
void hf3fs_crc_shutdown(void);             /* free every device context */
const char *hf3fs_crc_last_error(void);    /* thread-local message of the last failure */
const char *hf3fs_crc_version(void);

/* Scratch lifetime.  Batch calls without caller scratch (verify with d_computed ==
 * NULL, update, read results, scrub, frames, file digest) run on device buffers the
 * library owns per (stream, calling thread); they grow to the largest call and are
 * kept until one of these calls (or hf3fs_crc_shutdown).  release_stream: after the
 * stream's queued work, free every thread's buffers of `stream`, its side streams and
 * its update-apply grid hints (call it before destroying a stream the library was used
 * on; no thread may use the stream during the call).  Calls captured into a graph (any of the above, and every ticket counter
 * and balance region of a captured launch) get memory of their own, owned by the
 * graph through one hipUserObject per capture (small requests share 256 KiB slabs of
 * the capture): when the graph and every executable graph instantiated from it are
 * destroyed, the buffers are freed by release_graph_scratch, release_stream, at
 * shutdown (after which no graph captured earlier may be replayed), or by an
 * uncaptured call once 64 MiB await freeing (hipFree waits for the whole device, so
 * no call pays it routinely; that wait also covers a replay still in flight when its
 * executable graph was destroyed).  Other graphs are never affected.
 * release_graph_scratch also frees buffers no graph could take a reference to.
 * graph_scratch_stats: live captured buffers (and their bytes), and those whose graph
 * is gone and that await the next free; any pointer may be NULL. */
int hf3fs_crc_release_stream(void *stream);
int hf3fs_crc_release_graph_scratch(void);
int hf3fs_crc_graph_scratch_stats(uint64_t *live_buffers, uint64_t *live_bytes, uint64_t *dead_buffers);

/* Tuning and test switches: read once per process from
 * HF3FS_CRC_<NAME> (upper case) at the first call; set_option overrides one for
 * every later call (tests, in-process A/B).  Unknown names or values -> kInvalidArg.
 * Names: nt, seg_kib, static, pipe (auto|0|1), balance, record_direct,
 * update_pipeline (mode|unfused|fused), apply_pieces, apply_min_kib, apply_nt,
 * apply_grid (-1 auto, 0 ticketed, 1 one-shot, 2 one-shot on a small grid), apply_piece_kib
 * (4|8|16), frame_stream (auto|0|1), frame_segw, debug, audit, range_stream, list_runs,
 * prehash_rep (1..8 byte runs per wave for the update pre hash and list_runs batches).
 * Test only, settable through set_option alone (the environment is ignored for them):
 * poison (every library scratch word handed to a call is first set to this value,
 * 0 = off) and fault_io (IO fault_io - 1 of every update batch is hashed from a wrong
 * start value, 0 = off: the self-check's end-to-end test). */
int hf3fs_crc_set_option(const char *name, const char *value);
int hf3fs_crc_get_option(const char *name, char *out, size_t cap);

/* Self-check record.  Every payload an update batch reports as
 * mismatched is re-hashed by the batch's last kernel with an independent method
 * (per-lane serial slicing, no shared code with the pipeline's hash).  If the
 * re-hash equals the client's checksum, the pipeline's verdict was wrong: the IO
 * gets HF3FS_CRC_DEVICE_ERROR instead (chunk untouched, retry the IO) and the
 * inconsistency is recorded here with what the scratch held at that point. */
enum {
  HF3FS_ANOMALY_PAYLOAD_HASH = 1, /* the pipeline's payload hash != the re-hash == the client checksum */
  HF3FS_ANOMALY_PRE_JOB = 2,      /* the payload job's (address, length) != the IO's */
  HF3FS_ANOMALY_PRE_MAX = 4,      /* the job-length maximum word < the payload length */
  HF3FS_ANOMALY_START_ONLY = 8,   /* the pipeline's hash is the start value alone (it saw no bytes) */
  HF3FS_ANOMALY_RUN_COVER = 16    /* the pre hash's byte runs do not cover the payload exactly once */
};
typedef struct hf3fs_crc_anomaly {
  uint32_t count;      /* inconsistencies since the last reset */
  uint32_t kinds;      /* OR of HF3FS_ANOMALY_* over all of them */
  uint32_t kind;       /* the first one: its HF3FS_ANOMALY_* bits */
  uint32_t pipeline;   /* its batch: 0 three-pass, 1 fused; | mode << 8 */
  uint64_t io;         /* its IO index in the batch */
  uint32_t pipeline_hash, rehash, client_checksum, pre_max;
  uint64_t pre_addr, pre_len, payload, length;
} hf3fs_crc_anomaly;
/* Device-synchronizes, copies device `device`'s record to *out, then zeroes it if reset. */
int hf3fs_crc_anomalies(int device, hf3fs_crc_anomaly *out, int reset);

/* ------------------------------------------------------------------------ */
/* scalar algebra (no data bytes; replaces folly/Rust combine calls)          */
/* ------------------------------------------------------------------------ */
/* folly::crc32c_combine (called at Common.h:191): crc1 * x^(8 len2) ^ crc2.
 * Also equals Rust crc32c::crc32c_combine on finalized values (chunk.rs:229). */
uint32_t hf3fs_crc32c_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);
/* folly::crc32_combine (Common.h:195) */
uint32_t hf3fs_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);
/* crc fed `nbytes` zero bytes, for `type` in {CRC32C, CRC32}. */
uint32_t hf3fs_crc_shift(uint8_t type, uint32_t crc, uint64_t nbytes);
/* ChecksumInfo::combine (Common.h:179-198) on {*type,*value} in place:
 * HF3FS_CRC_CHECKSUM_MISMATCH on a type mismatch (self not NONE), no-op for
 * length 0, copy when self is NONE. */
int hf3fs_checksum_combine(uint8_t *type, uint32_t *value, uint8_t other_type, uint32_t other_value,
                           uint64_t length);

/* ChecksumInfo in serde's binary form (src/common/serde/Serde.h:422-445 over
 * DownwardBytes): a table = varint32 byte length (5), then the fields in
 * declaration order -- type (1 byte), value (4 bytes, little-endian); 6 bytes,
 * as tests/storage/store/TestCommonStruct.cc:46-55 asserts.  Returns 6. */
uint32_t hf3fs_checksum_serialize(uint8_t type, uint32_t value, uint8_t *out6);
/* Inverse (Serde.h:465-512, 683-735): a table shorter than its length prefix or
 * a field cut short -> HF3FS_CRC_SERDE_INSUFFICIENT_LENGTH; fields missing at
 * the table's end keep their defaults ({NONE, 0}); bytes past the known fields
 * are skipped.  *consumed = bytes of the table including its prefix. */
int hf3fs_checksum_deserialize(const void *in, uint64_t n, uint8_t *type, uint32_t *value, uint64_t *consumed);

/* ------------------------------------------------------------------------ */
/* batched create / verify / combine on device-resident bytes                */
/* ------------------------------------------------------------------------ */
/* ChecksumInfo::create(type, buf, len, start) for n buffers (Common.h:146-177).
 * d_bufs[i]/d_lens[i]: device address and byte length of buffer i (any
 * alignment, any length including 0).  d_starts: per-buffer startingChecksum
 * or NULL for ~0U.  max_len >= every d_lens[i] (sizes the task grid).
 * d_out[i] receives the raw value; type NONE writes 0 (create's {NONE,0}). */
int hf3fs_crc_create_batch(uint8_t type, const void *const *d_bufs, const uint64_t *d_lens,
                           const uint32_t *d_starts, uint32_t *d_out, uint64_t n, uint64_t max_len, void *stream);

/* Same for n equal-length buffers at d_base + i*stride (the bulk write path:
 * one launch over a resident batch, BASELINE config 2). */
int hf3fs_crc_create_strided(uint8_t type, const void *d_base, uint64_t stride, uint64_t len, uint64_t n,
                             uint32_t start, uint32_t *d_out, void *stream);

/* Write/read verify (ChunkReplica.cc:193-207, StorageClientImpl.cc:1720-1737,
 * BatchReadJob.cc:43-54): recompute create(type, buf_i, len_i) and compare with
 * d_expected[i].  d_mismatch[i] = 1 on mismatch else 0; *d_mismatch_count is
 * SET to the number of mismatches.  d_computed (n u32, may be NULL) receives
 * the recomputed values; when NULL the library uses a scratch buffer of the
 * calling (stream, thread) pair, so concurrent calls never share it, on one
 * stream or on many (a larger n than any earlier call of that pair grows the
 * buffer after a stream synchronize).  A call captured into a graph uses a
 * buffer owned by that graph instead (scratch lifetime, above). */
int hf3fs_crc_verify_batch(uint8_t type, const void *const *d_bufs, const uint64_t *d_lens,
                           const uint32_t *d_expected, uint8_t *d_mismatch, uint32_t *d_mismatch_count,
                           uint32_t *d_computed, uint64_t n, uint64_t max_len, void *stream);
int hf3fs_crc_verify_strided(uint8_t type, const void *d_base, uint64_t stride, uint64_t len, uint64_t n,
                             const uint32_t *d_expected, uint8_t *d_mismatch, uint32_t *d_mismatch_count,
                             uint32_t *d_computed, void *stream);

/* KVCache read-verify (BASELINE config 5): n blocks addressed into one arena by
 * byte offset.  Same outputs as hf3fs_crc_verify_batch.  Graph-capturable. */
int hf3fs_crc_verify_blocks(uint8_t type, const void *d_arena, const uint64_t *d_offsets, const uint32_t *d_lens,
                            const uint32_t *d_expected, uint8_t *d_mismatch, uint32_t *d_mismatch_count,
                            uint32_t *d_computed, uint64_t n, uint32_t max_len, void *stream);

/* ChecksumInfo::combine element-wise on same-typed values: d_acc[i] =
 * combine(~d_acc[i], d_crc2[i], d_len2[i]) (Common.h:191,195); len2 == 0 leaves
 * d_acc[i] unchanged.  type NONE is a no-op. */
int hf3fs_crc_combine_batch(uint8_t type, uint32_t *d_acc, const uint32_t *d_crc2, const uint64_t *d_len2,
                            uint64_t n, void *stream);

/* The typed digest table of n chunks in the reference's wire form: d_out =
 * n x 6 bytes, element i = hf3fs_checksum_serialize(type, d_values[i]). */
int hf3fs_crc_serialize_batch(uint8_t type, const uint32_t *d_values, uint64_t n, uint8_t *d_out, void *stream);

/* _fin helpers: the chunk engine and the Rust crc32c crate carry FINALIZED
 * values (fin = ~raw, ChunkEngine.cc:42,66; chunk.rs:157,229).  In place
 * raw <-> fin for n device values (the map is its own inverse). */
int hf3fs_crc_finalize_batch(uint32_t *d_values, uint64_t n, void *stream);
/* crc32c::crc32c_combine on finalized values (chunk.rs:229): the same algebra
 * as the raw form, fin(A||B) = fin(A) * x^(8 len2) ^ fin(B). */
uint32_t hf3fs_crc32c_combine_fin(uint32_t fin1, uint32_t fin2, uint64_t len2);

/* ------------------------------------------------------------------------ */
/* chunk checksum maintenance: ChunkReplica::update + updateChecksum          */
/* ------------------------------------------------------------------------ */
/* One UpdateIO applied to one device-resident chunk replica.  Field meanings
 * follow UpdateIO (Common.h:331-345) and ChunkMetadata (Common.h:652-677).   */
typedef struct hf3fs_crc_update_io {
  uint64_t chunk;           /* device address of the chunk bytes (capacity >= max(size, offset+length)) */
  uint64_t payload;         /* device address of the write payload (`length` bytes); 0 for truncate/extend */
  uint32_t offset;          /* UpdateIO.offset */
  uint32_t length;          /* UpdateIO.length (truncate/extend: the target chunk length) */
  uint32_t chunk_size;      /* ChunkMetadata.size before this IO */
  uint8_t update_type;      /* HF3FS_UPDATE_{WRITE,TRUNCATE,EXTEND} */
  uint8_t chunk_checksum_type;  /* ChunkMetadata.checksumType */
  uint8_t write_checksum_type;  /* UpdateIO.checksum.type */
  uint8_t flags;            /* HF3FS_UPDATE_FLAG_* */
  uint32_t chunk_checksum;  /* ChunkMetadata.checksumValue (raw) */
  uint32_t write_checksum;  /* UpdateIO.checksum.value (raw) */
  /* outputs */
  uint32_t out_size;        /* ChunkMetadata.size after this IO */
  uint32_t out_checksum;    /* ChunkMetadata.checksumValue after this IO (raw) */
  uint8_t out_checksum_type;
  uint8_t checksum_case;    /* HF3FS_CKCASE_*: which checksum path the reference takes for this IO (0 = not applied) */
  uint8_t reserved1[2];
  int32_t status;           /* HF3FS_CRC_OK, _CHECKSUM_MISMATCH (payload verify failed: chunk untouched), _INVALID_ARG,
                               _DEVICE_ERROR (the self-check contradicted the verify: chunk untouched, retry) */
} hf3fs_crc_update_io;

/* hf3fs_crc_update_io.checksum_case: the reference's per-update checksum
 * counters, so a caller keeps feeding its metrics.
 * Replica IOs (ChunkReplica::updateChecksum, ChunkReplica.cc:25-28,334-389):
 *   NONE -> storage.chunk_update.checksum_none, REUSE -> _reuse,
 *   COMBINE -> _combine, RECOMPUTE -> _read_chunk (prefix + suffix re-read; the
 *   DELTA mode reports the case the reference takes, whatever it computed).
 * Engine IOs (HF3FS_UPDATE_FLAG_ENGINE, chunk.rs:153,156,188,217,233,273):
 *   REUSE -> checksum_reuse (copy_on_write without read), COMBINE ->
 *   checksum_combine (safe_write padding / direct or indirect append),
 *   RECOMPUTE -> checksum_recalculate (copy_on_write with read, truncate
 *   shorten), NONE -> no counter.  The engine's choice between copy_on_write
 *   and safe_write also depends on the allocated capacity (engine.rs:383-385);
 *   it is taken as the chunk size (max_len), which no write exceeds here. */
enum {
  HF3FS_CKCASE_NONE = 1,
  HF3FS_CKCASE_REUSE = 2,
  HF3FS_CKCASE_COMBINE = 3,
  HF3FS_CKCASE_RECOMPUTE = 4
};

enum {
  HF3FS_UPDATE_MODE_REFERENCE = 0, /* ChunkReplica.cc:356-389: recompute prefix + suffix after the write */
  HF3FS_UPDATE_MODE_DELTA = 1      /* read only the overwritten old bytes: new = old*x^(8 dsize) ^ lin(old^new)*x^(...) */
};

/* hf3fs_crc_update_io.flags */
enum {
  /* Chunk-engine semantics (ChunkEngine::update, src/storage/store/ChunkEngine.cc:15-66, over the Rust
   * engine, chunk_engine/src/core/engine.rs:288-420 and alloc/chunk.rs:89-281): the chunk checksum is
   * always CRC32C and always the CRC of the chunk bytes (an empty chunk is ~0 raw = 0 finalized); a write
   * whose checksum type is not CRC32C is taken "without_checksum" (hashed, not verified).  Values stay
   * raw at this ABI, as at the C++ bridge (finalized = ~raw, ChunkEngine.cc:42,66). */
  HF3FS_UPDATE_FLAG_ENGINE = 1
};

/* Applies n IOs to n DISTINCT chunks: verify the payload checksum
 * (ChunkReplica.cc:193-207), write it with gap zero-fill (:281-292), and set
 * the new chunk checksum (:319-394).  d_ios is device-accessible and updated in
 * place.  max_len = the chunk size (UpdateIO.chunkSize): offset >= max_len or
 * offset + length > max_len is kInvalidArg (ChunkReplica.cc:139-145).
 * `type` is the checksum type the batch hashes bytes in: a write's checksum
 * type must be NONE or `type`; the chunk's stored type may be any type -- a
 * write whose type differs from the chunk's recomputes the prefix and suffix
 * in the write's type and the chunk takes the write's type (ChunkReplica.cc:
 * 340, 356-392).  A truncate / extend hashes in the chunk's type, so its chunk
 * type must be NONE or `type` (else kInvalidArg for that IO).
 * Modes: REFERENCE recomputes prefix + suffix from the chunk bytes, as the
 * reference does.  DELTA reads only the overwritten old bytes and derives the
 * new value from the stored chunk checksum: identical results whenever the
 * stored checksum matches the chunk bytes (the invariant the reference keeps);
 * if metadata and bytes disagree (corruption, stale metadata) DELTA carries
 * the disagreement forward where REFERENCE re-derives from the bytes.
 * Stream behaviour: asynchronous on `stream`.  The three-pass pipeline (DELTA's
 * default) forks the verdicts' finalize onto a side stream the library keeps per
 * (stream, calling thread) and joins it back before the call's last launch
 * (capturable); its apply launches one workgroup per 8 KiB piece on a grid sized
 * from the pair's previous call (option apply_grid). */
int hf3fs_crc_update_batch(uint8_t type, hf3fs_crc_update_io *d_ios, uint64_t n, uint32_t max_len, int mode,
                           void *stream);
/* Bytes of scratch one hf3fs_crc_update_batch of n IOs in `mode` takes.  Outside
 * a stream capture the call uses a buffer the library keeps per (stream, calling
 * thread), grown with a stream synchronize when a call needs more (make one call
 * of the largest size first where that stall matters); a captured call gets a
 * buffer of its own (hipMalloc in relaxed capture mode, kept for the graph's
 * replays; see hf3fs_crc_release_graph_scratch).  Never the stream-ordered pool.
 * Every word the call reads is written by the call first (checked with option poison).
 * The figure is for the ticketed apply; a call with the one-shot apply adds a piece
 * table of 4 B per 8 KiB piece, n * (max_len / 8 KiB + 4) entries. */
size_t hf3fs_crc_update_scratch_bytes(uint64_t n, int mode);

/* ------------------------------------------------------------------------ */
/* read results: AioReadJob::setResult checksum part                          */
/* ------------------------------------------------------------------------ */
/* One completed chunk read (src/storage/aio/BatchReadJob.cc:24-63). */
typedef struct hf3fs_crc_read_io {
  uint64_t data;            /* device address of the read bytes (localbuf + headLength) */
  uint32_t offset;          /* ReadIO.offset */
  uint32_t length;          /* bytes actually read (*lengthInfo) */
  uint32_t chunk_len;       /* state_.chunkLen */
  uint8_t batch_checksum_type;  /* BatchReadReq checksumType */
  uint8_t chunk_checksum_type;  /* state_.chunkChecksum.type */
  uint8_t recalculate;      /* batch_.recalculateChecksum() (resync full-chunk reads) */
  uint8_t reserved0;
  uint32_t chunk_checksum;  /* state_.chunkChecksum.value (raw) */
  /* outputs */
  uint32_t out_checksum;    /* IOResult.checksum.value */
  uint8_t out_checksum_type;
  uint8_t reserved1[3];
  int32_t status;           /* 0, or 4080 when the recalculated full-chunk checksum differs */
  uint32_t reserved2;
} hf3fs_crc_read_io;

/* For n completed reads: NONE batch -> {NONE,0}; a full-chunk read of the
 * stored type reuses the chunk checksum; otherwise the read bytes are hashed;
 * with `recalculate`, full-chunk reads are re-hashed and compared with the
 * stored checksum (status 4080 on mismatch).  Non-NONE types must equal
 * `type`.  max_len >= every length. */
int hf3fs_crc_read_result_batch(uint8_t type, hf3fs_crc_read_io *d_ios, uint64_t n, uint32_t max_len, void *stream);

/* ------------------------------------------------------------------------ */
/* file digest: admin `checksum --fill-zero`                                  */
/* ------------------------------------------------------------------------ */
/* One chunk read of a file, in file order (FileWrapper.cc:133-160). */
typedef struct hf3fs_crc_block_digest {
  uint64_t read_len;        /* *lengthInfo; 0 for kChunkNotFound */
  uint64_t block_len;       /* ReadIO.length (the bytes the file holds there) */
  uint32_t checksum;        /* readIO.result.checksum.value (raw) */
  uint8_t checksum_type;    /* readIO.result.checksum.type; NONE for a missing chunk */
  uint8_t missing;          /* 1: the read failed with kChunkNotFound (read_len and checksum ignored) */
  uint8_t reserved[2];
} hf3fs_crc_block_digest;

/* Digest of one file (or one replica of it). */
typedef struct hf3fs_crc_file_digest {
  uint64_t length;          /* sum of block_len */
  uint32_t value;           /* ChecksumInfo.value (raw) */
  uint8_t type;             /* ChecksumInfo.type */
  uint8_t reserved[3];
  int32_t status;           /* 0; 3 if any block has an unknown type, or (fill-zero) read_len > block_len
                               (checked before the fold); else the first error in file order: 4080 on a
                               type mismatch, and without fill-zero 7007 for a missing chunk, 33 for a
                               read whose length differs from block_len */
  uint32_t reserved2;
} hf3fs_crc_file_digest;

/* FileWrapper::readFile's checksum fold with fillZero (FileWrapper.cc:119-164;
 * called per replica by Checksum.cc:43-88), for n_files files at once: file f
 * owns blocks [d_file_off[f], d_file_off[f+1]) of d_blocks.  Short reads are
 * zero-filled with CRC32C, each block is folded with ChecksumInfo::combine
 * (block, block_len); the result (or the first error's status) goes to
 * d_out[f].  max_blocks >= every file's block count (sizes the grid). */
int hf3fs_crc_file_digest_batch(const hf3fs_crc_block_digest *d_blocks, const uint64_t *d_file_off,
                                hf3fs_crc_file_digest *d_out, uint64_t n_files, uint64_t max_blocks, void *stream);

/* The same fold with the admin command's options (Checksum.cc:43-88 passes --fill-zero to
 * FileWrapper::readFile, FileWrapper.cc:133-160).  HF3FS_DIGEST_FILL_ZERO: as above.
 * Without it, blocks are taken in file order and the first failing one ends the
 * fold: a missing chunk -> HF3FS_CRC_CHUNK_NOT_FOUND (the read error, :134-139), a
 * read of another length than block_len -> HF3FS_CRC_INVALID_FORMAT ("read is
 * short", :153-160), a type mismatch of the combine -> HF3FS_CRC_CHECKSUM_MISMATCH. */
enum { HF3FS_DIGEST_FILL_ZERO = 1 };
int hf3fs_crc_file_digest_batch_ex(const hf3fs_crc_block_digest *d_blocks, const uint64_t *d_file_off,
                                   hf3fs_crc_file_digest *d_out, uint64_t n_files, uint64_t max_blocks,
                                   uint32_t flags, void *stream);

/* ------------------------------------------------------------------------ */
/* stored-chunk scrub against persisted checksums         */
/* ------------------------------------------------------------------------ */
/* One stored chunk and the checksum its metadata persists: either C++
 * ChunkMetadata {size, checksumType, checksumValue} (src/fbs/storage/
 * Common.h:652-677, raw value) or the chunk engine's ChunkMeta {len, checksum}
 * (src/storage/chunk_engine/src/types/chunk_meta.rs:7-20, finalized value,
 * type CRC32C, bridged with ~ at src/storage/store/ChunkEngine.cc:42,66). */
typedef struct hf3fs_crc_scrub_io {
  uint64_t data;            /* device address of the chunk bytes */
  uint32_t length;          /* ChunkMetadata.size / ChunkMeta.len */
  uint8_t checksum_type;    /* ChunkMetadata.checksumType (engine records: CRC32C) */
  uint8_t fin;              /* 1: `checksum` is finalized (ChunkMeta.checksum), 0: raw */
  uint16_t reserved;
  uint32_t checksum;        /* persisted value */
  uint32_t computed;        /* out: raw create(type, data, length) (0 for NONE) */
  int32_t status;           /* out: 0; 4080 on mismatch; 3 for a bad record */
  uint32_t reserved2;
} hf3fs_crc_scrub_io;

/* Recompute every typed chunk and compare with its persisted checksum, as the
 * full-chunk resync check of AioReadJob::setResult does per read
 * (BatchReadJob.cc:43-54).  NONE chunks pass unchecked.  Non-NONE types must
 * equal `type`.  *d_mismatch_count is SET to the number of non-zero statuses. */
int hf3fs_crc_scrub_batch(uint8_t type, hf3fs_crc_scrub_io *d_ios, uint64_t n, uint32_t max_len,
                          uint32_t *d_mismatch_count, void *stream);

/* The chunk engine's persisted ChunkMeta (chunk_meta.rs:7-20) in its derse
 * wire form: a one-byte body length, then pos u64, chain_ver, chunk_ver, len,
 * checksum (u32 each), timestamp, last_request_id, last_client_low/high (u64
 * each, all little-endian), etag (length byte + bytes), uncommitted (bool).
 * Pinned by the reference's own vector (chunk_meta.rs:59-87).  Bodies of 128
 * bytes or more use a multi-byte length whose derse encoding is not pinned by
 * any reference vector: rejected with kInvalidArg. */
typedef struct hf3fs_crc_engine_meta {
  uint64_t pos;
  uint32_t chain_ver;
  uint32_t chunk_ver;
  uint32_t len;
  uint32_t checksum;        /* finalized CRC32C of the chunk's [0, len) */
  uint64_t timestamp;
  uint64_t last_request_id;
  uint64_t last_client_low;
  uint64_t last_client_high;
  uint8_t etag_len;
  uint8_t uncommitted;
  uint8_t etag[62];
} hf3fs_crc_engine_meta;

int hf3fs_crc_engine_meta_decode(const void *h_bytes, uint64_t n, hf3fs_crc_engine_meta *out, uint64_t *consumed);
int hf3fs_crc_engine_meta_encode(const hf3fs_crc_engine_meta *m, void *h_out, uint64_t cap, uint64_t *written);
/* ChunkMeta::set_default_etag_if_need (chunk_meta.rs:30-34): format!("{:X}",
 * checksum) into out (no terminator); returns its length (1..8). */
uint32_t hf3fs_crc_default_etag(uint32_t checksum_fin, char *out8);

/* ------------------------------------------------------------------------ */
/* serde message frames                                   */
/* ------------------------------------------------------------------------ */
/* One framed message: MessageHeader {u32 checksum; u32 size} + payload
 * (src/common/net/MessageHeader.h:20-27). */
typedef struct hf3fs_crc_frame {
  uint64_t offset;          /* payload offset in the receive buffer (header at offset - 8) */
  uint32_t size;            /* MessageHeader.size */
  uint32_t checksum;        /* MessageHeader.checksum as received */
  uint32_t computed;        /* out: Checksum::calcSerde(payload, size, checksum & 1) */
  int32_t status;           /* out: 0; 4080 when computed != checksum; 3 for size > max_size */
} hf3fs_crc_frame;

/* The framing walk of Processor::unpackMsg (src/common/net/Processor.h:85-107)
 * over host bytes: records every complete serde frame in order (at most
 * max_frames).  Returns 0 when the buffer is a whole number of serde frames,
 * kInvalidArg at the first incomplete or non-serde frame (what the reference
 * treats as a broken transport); n_frames and consumed cover the frames before it. */
int hf3fs_crc_frame_walk(const void *h_buf, uint64_t len, hf3fs_crc_frame *h_frames, uint64_t max_frames,
                         uint64_t *n_frames, uint64_t *consumed);
/* Checksum::calcSerde (MessageHeader.h:33-37: crc32c with init 0, low byte =
 * 0x86 | compressed) of every frame payload at d_buf + offset, compared with
 * the received header (Processor.h:111-120).  `computed` also serves the send
 * side (WriteItem.h:100).  *d_mismatch_count is SET to the non-zero statuses. */
int hf3fs_crc_frame_verify_batch(const void *d_buf, hf3fs_crc_frame *d_frames, uint64_t n, uint32_t max_size,
                                 uint32_t *d_mismatch_count, void *stream);

/* ------------------------------------------------------------------------ */
/* host-memory entry points (synchronous)                                    */
/* ------------------------------------------------------------------------ */
/* ChecksumInfo::create over host buffers: bytes are streamed H2D through a
 * pinned staging ring (two streams) and hashed on the current device. */
int hf3fs_crc_create_host(uint8_t type, const void *const *h_bufs, const uint64_t *h_lens, const uint32_t *h_starts,
                          uint32_t *h_out, uint64_t n);

/* ------------------------------------------------------------------------ */
/* per-IO request coalescer                               */
/* ------------------------------------------------------------------------ */
/* The reference hashes one IO per call on the thread that completes it:
 * AioReadJob::setResult (src/storage/aio/BatchReadJob.cc:24-35, 32
 * AioReadWorker threads), ChunkReplica::update's payload verify
 * (src/storage/store/ChunkReplica.cc:193-207, 32 UpdateWorker threads) and the
 * client's per-IO create/verify (src/client/storage/StorageClientImpl.cc:
 * 1720-1737, 1878-1882).  A coalescer accepts such single ChecksumInfo::create
 * requests from any number of threads and hashes whatever arrived while the
 * previous batch was on the device in one launch. */
typedef struct hf3fs_crc_coalescer hf3fs_crc_coalescer;

/* Completion callback: status 0 and the raw value of create(type, buf, len,
 * start), or an error status and 0.  Runs on the coalescer's completion
 * thread, in launch order; it must not block. */
typedef void (*hf3fs_crc_done_fn)(void *arg, int status, uint32_t value);

typedef struct hf3fs_crc_coalescer_options {
  int device;            /* HIP device that hashes the requests */
  uint32_t max_batch;    /* requests per type per launch (default 4096) */
  uint32_t max_wait_us;  /* an idle device waits this long for company (default 0) */
  uint32_t slots;        /* batches open + in flight (default 4, >= 2) */
  uint32_t inflight;     /* launch early only while fewer batches are on the device (default 2, < slots) */
  uint32_t service_wgs;  /* 0: batch mode.  > 0: service mode, CRC32C requests are served by this many
                            resident workgroups polling a request ring (no launch per request) */
  uint64_t stage_bytes;  /* pinned stage per slot for HOST_COPY requests (default 32 MiB) */
  uint32_t service_ring;     /* service ring slots, power of two (default 1024) */
  uint32_t service_idle_us;  /* the service kernel exits after this long without requests and is
                                relaunched on demand (default 2000) */
  uint64_t service_stage;    /* pinned stage per ring slot for HOST_COPY requests (default 64 KiB;
                                larger requests take the batch path) */
} hf3fs_crc_coalescer_options;

/* request flags */
enum {
  /* `buf` is plain host memory: the submitting thread copies it into a pinned
   * stage that the kernel reads over PCIe.  Without the flag `buf` must be
   * device-accessible (HBM, or host memory from hf3fs_crc_host_register) and
   * stay valid until the callback runs. */
  HF3FS_CRC_REQ_HOST_COPY = 1
};

void hf3fs_crc_coalescer_default_options(hf3fs_crc_coalescer_options *opt); /* device = current device */
int hf3fs_crc_coalescer_create(const hf3fs_crc_coalescer_options *opt, hf3fs_crc_coalescer **out);
/* Launches what is pending, completes every request, joins the threads. */
void hf3fs_crc_coalescer_destroy(hf3fs_crc_coalescer *co);
/* Asynchronous ChecksumInfo::create(type, buf, len, start) (Common.h:146-177):
 * NONE -> value 0 and length 0 -> value `start` complete at once on the
 * calling thread.  A HOST_COPY request larger than stage_bytes is hashed
 * through hf3fs_crc_create_host before returning. */
int hf3fs_crc_coalescer_submit(hf3fs_crc_coalescer *co, uint8_t type, const void *buf, uint64_t len, uint32_t start,
                               uint32_t flags, hf3fs_crc_done_fn fn, void *arg);
/* Blocking form: returns the submit/batch status, *out = raw value. */
int hf3fs_crc_coalescer_create_one(hf3fs_crc_coalescer *co, uint8_t type, const void *buf, uint64_t len,
                                   uint32_t start, uint32_t flags, uint32_t *out);
/* out4 = {requests, batches launched, bytes, largest batch}. */
int hf3fs_crc_coalescer_stats(hf3fs_crc_coalescer *co, uint64_t *out4);

/* Page-lock and map host memory (3FS registers its RDMA BufferPool slabs,
 * src/storage/service/BufferPool.h:24-27, and client IOBuffers the same way)
 * so kernels read it in place; *d_ptr is the device address of h_ptr. */
int hf3fs_crc_host_register(void *h_ptr, uint64_t len, void **d_ptr);
int hf3fs_crc_host_unregister(void *h_ptr);

/* Wait for `stream`'s queued work without spinning: hipStreamQuery polled with a sleep of
 * poll_us microseconds between polls (poll_us == 0: hipStreamSynchronize, HIP's busy wait).
 * For many caller threads on few cores -- 3FS's 32 AioReadWorker threads on a storage node's
 * CPU quota: 32 spinning waits on a 16-CPU quota were throttled by the cgroup for tens of
 * milliseconds at a time (p99 batch latency 58 ms against 4.3 ms polled). */
int hf3fs_crc_stream_wait(void *stream, uint32_t poll_us);

/* ------------------------------------------------------------------------ */
/* synthetic data (benchmarks/tests)                                         */
/* ------------------------------------------------------------------------ */
/* Fills n_chunks chunks of chunk_len bytes at d_dst + i*stride with
 * splitmix64(seed ^ ((first_chunk_id + i) << 32) ^ word_index) little-endian
 * words, byte-identical to oracle/orc_fill_synth. */
int hf3fs_crc_fill_synth(void *d_dst, uint64_t stride, uint64_t chunk_len, uint64_t n_chunks, uint64_t seed,
                         uint64_t first_chunk_id, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* HF3FS_CRC_H */
