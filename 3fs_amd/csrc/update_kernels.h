// update_kernels.h -- device side of hf3fs_crc_update_batch: ChunkReplica::update
// (verify payload, write with gap zero-fill) + ChunkReplica::updateChecksum
// (src/storage/store/ChunkReplica.cc:132-394) for a batch of chunk replicas
// resident in HBM.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hf3fs_crc.h"
#include "crc_kernels.h"

namespace hf3fs_crc {

// One IO of the single-read DELTA pipeline (prep -> k_update_delta), byte
// ranges relative to the chunk, empty when lo == hi:
//   W [w0, w1)  bytes stored: the payload over [p0, p1), zeros elsewhere (gap, extend)
//   P [p0, p1)  payload position in the chunk (payload byte x - p0 lands at x)
//   O [o0, o1)  old bytes hashed (delta identity), read before the piece is stored
// Pieces: the kDeltaPiece-aligned windows of (chunk + [u0, u1)), u = W u P u O.
struct DeltaDesc {
  uint64_t chunk, payload, base;  // base = (chunk + u0) & ~(kDeltaPiece - 1)
  uint32_t w0, w1, p0, p1, o0, o1;
  uint32_t u0, u1;
  uint32_t npieces;   // pieces (task list entries, <= 32)
  uint32_t reserved;
  uint32_t wval;      // client checksum (raw) when verify
  uint8_t verify;     // stores wait for the payload verdict
  uint8_t hashp;      // payload hash needed (verify, or engine without_checksum)
  uint8_t hash;       // any hash needed (payload or old bytes): hash pieces publish
  uint8_t pad;
};
static_assert(sizeof(DeltaDesc) == 72, "DeltaDesc layout");
// Per-IO words of the fused DELTA pipeline (zeroed before prep): on a 128-byte
// line of its own, two 64-bit {arrival mask << 32 | xor of partial CRCs} words
// (payload, old bytes; piece j is bit j), and a verdict word per IO in a
// separate array (polled).
constexpr int kSyncWords = 16;  // u64 per IO
constexpr int kSyncO = 1;       // the old-byte word
// verdict bits: payload hashed, old bytes hashed (both: the piece's bytes may be
// overwritten), payload mismatch (do not store), aborted (do not store)
enum { kVerdictP = 1, kVerdictO = 2, kVerdictMismatch = 4, kVerdictAborted = 8 };

// Scratch used by one update_batch call (device memory, stream-ordered).
struct UpdateScratch {
  uint32_t* max_len;   // [0] longest pre job, [1] longest post job (atomicMax in prep)
  uint64_t* pre_addr;  // [2n] jobs hashed BEFORE the write: payload (verify), old bytes (delta)
  uint64_t* pre_len;
  uint32_t* pre_start;
  uint32_t* pre_out;
  uint64_t* post_addr;  // [2n] jobs hashed AFTER the write: prefix, suffix (reference algorithm)
  uint64_t* post_len;
  uint32_t* post_start;
  uint32_t* post_out;
  // apply tasks, compacted by prep: (IO << 8) | gap << 7 | piece.  A range of
  // len bytes is cut into ceil(len / piece_bytes) pieces, piece_bytes =
  // max(piece_min, len / pieces), so one long write does not hold a
  // workgroup while the rest of the grid idles.  Count: the u64 at max_len + 2.
  uint64_t* tasks;
  uint32_t pieces;     // most pieces per range (+1 for the 16-byte alignment of the cuts)
  uint32_t piece_min;  // bytes, multiple of 16
  // single-read DELTA pipeline (null otherwise): tasks = (IO << 16) | piece
  DeltaDesc* dd;
  uint64_t* dsync;     // [n][kSyncWords]
  uint32_t* verdict;   // [n]
  uint32_t dpiece;     // fused DELTA: piece bytes (power of two, <= 32 pieces per IO)
  uint32_t dlag;       // fused DELTA: pieces between a piece's hash and its copy
};

// delta_len: the chunk size when the single-read DELTA pipeline runs, else 0.
size_t update_scratch_bytes(uint64_t n, uint32_t pieces, uint32_t delta_len);
void update_scratch_carve(void* base, uint64_t n, uint32_t pieces, uint32_t piece_min, uint32_t delta_len,
                          UpdateScratch* s);

hipError_t launch_update_prep(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type, int mode,
                              const UpdateScratch& s, hipStream_t st);
hipError_t launch_update_apply(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type,
                               const UpdateScratch& s, uint32_t grid, uint32_t* queue, hipStream_t st);
// Fused prep + payload verify + write (+ delta old-byte hash), one workgroup
// per IO; leaves the scratch as prep -> ranges(pre) -> apply would.
hipError_t launch_update_fused(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type, int mode,
                               const UpdateScratch& s, const DeviceTables* tabs, uint32_t grid, uint32_t* queue,
                               hipStream_t st);
// Single-read DELTA: prep (descriptors + piece tasks) and the piece kernel that
// reads each payload byte once -- verify hash, old-byte hash and the store.
hipError_t launch_update_delta_prep(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type,
                                    const UpdateScratch& s, hipStream_t st);
hipError_t launch_update_delta(hf3fs_crc_update_io* ios, uint8_t type, const UpdateScratch& s,
                               const DeviceTables* tabs, uint32_t grid, uint32_t* queue, hipStream_t st);
hipError_t launch_update_finalize(hf3fs_crc_update_io* ios, uint64_t n, uint8_t type, int mode,
                                  const UpdateScratch& s, const DeviceTables* tabs, uint32_t max_len,
                                  hipStream_t st);

// AioReadJob::setResult batch: prep selects the reads to hash (addr/len jobs,
// longest job in *maxl), finalize applies the reuse / NONE / recalculate rules.
hipError_t launch_read_prep(hf3fs_crc_read_io* ios, uint64_t n, uint8_t type, uint32_t max_len, uint64_t* addr,
                            uint64_t* len, uint32_t* maxl, hipStream_t st);
hipError_t launch_read_finalize(hf3fs_crc_read_io* ios, uint64_t n, const uint32_t* v, hipStream_t st);

}  // namespace hf3fs_crc
