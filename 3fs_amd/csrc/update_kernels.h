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
};

size_t update_scratch_bytes(uint64_t n, uint32_t pieces);
void update_scratch_carve(void* base, uint64_t n, uint32_t pieces, uint32_t piece_min, UpdateScratch* s);

hipError_t launch_update_prep(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type, int mode,
                              const UpdateScratch& s, hipStream_t st);
hipError_t launch_update_apply(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type,
                               const UpdateScratch& s, uint32_t grid, uint32_t* queue, hipStream_t st);
// Fused prep + payload verify + write (+ delta old-byte hash), one workgroup
// per IO; leaves the scratch as prep -> ranges(pre) -> apply would.
hipError_t launch_update_fused(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type, int mode,
                               const UpdateScratch& s, const DeviceTables* tabs, uint32_t grid, uint32_t* queue,
                               hipStream_t st);
hipError_t launch_update_finalize(hf3fs_crc_update_io* ios, uint64_t n, uint8_t type, int mode,
                                  const UpdateScratch& s, const DeviceTables* tabs, uint32_t max_len,
                                  hipStream_t st);

// AioReadJob::setResult batch: prep selects the reads to hash (addr/len jobs,
// longest job in *maxl), finalize applies the reuse / NONE / recalculate rules.
hipError_t launch_read_prep(hf3fs_crc_read_io* ios, uint64_t n, uint8_t type, uint32_t max_len, uint64_t* addr,
                            uint64_t* len, uint32_t* maxl, hipStream_t st);
hipError_t launch_read_finalize(hf3fs_crc_read_io* ios, uint64_t n, const uint32_t* v, hipStream_t st);

}  // namespace hf3fs_crc
