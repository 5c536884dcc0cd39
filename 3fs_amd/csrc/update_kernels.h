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

// One apply task (prep emits them, compacted): a piece of an IO's payload
// copy (src != 0) or of its gap zero-fill (src == 0), cut at a 16-byte
// aligned destination address.  `verify`: the copy runs only if the payload
// hash pre_out[2 io] equals wval (ChunkReplica.cc:193-207).
struct ApplyTask {
  uint64_t dst, src;
  uint32_t len, io;
  uint32_t wval, verify;
};
static_assert(sizeof(ApplyTask) == 32, "ApplyTask layout");

// Control words of one update_batch call, zeroed by ONE launch at its start.
enum {
  kCtlPreMax = 0,    // longest pre job (atomicMax in prep)
  kCtlPostMax = 1,   // longest post job
  kCtlTasks = 2,     // [2..3] apply task count (u64)
  kCtlQueuePre = 4,  // ticket counters: pre hash, apply, post hash, fused kernel
  kCtlQueueApply = 5,
  kCtlQueuePost = 6,
  kCtlQueueFused = 7,
  kCtlPieces = 8,    // [8..9] apply pieces of 2^piece_shift bytes (u64): the one-shot apply's
                     // piece table length; in ticket mode counted for the next call's grid
  kCtlWords = 10
};

// Scratch used by one update_batch call (device memory, stream-ordered).
struct UpdateScratch {
  uint32_t* ctl;       // kCtlWords control words
  uint64_t* pre_addr;  // [2n] jobs hashed BEFORE the write: payload (verify), old bytes (delta)
  uint64_t* pre_len;
  uint32_t* pre_start;
  uint32_t* pre_out;   // zeroed by prep (the hash XORs segment values into it)
  uint64_t* post_addr;  // [2n] jobs hashed AFTER the write: prefix, suffix (reference algorithm)
  uint64_t* post_len;
  uint32_t* post_start;
  uint32_t* post_out;
  // apply tasks (three-pass pipeline): a range of len bytes is cut into
  // ceil(len / piece_bytes) pieces, piece_bytes = max(piece_min, len / pieces),
  // so one long write does not hold a workgroup while the rest of the grid idles.
  ApplyTask* tasks;
  uint32_t pieces;     // most pieces per range (+1 for the 16-byte alignment of the cuts)
  uint32_t piece_min;  // bytes, multiple of 16
  // one-shot apply: every range is cut at 2^piece_shift-aligned destination
  // addresses; one workgroup copies one piece and exits.  tasks[2 i] / tasks[2 i + 1] are IO
  // i's payload / gap range records (verify = first piece | verify << 31), ptab[p] the
  // record of piece p.  one_shot = 0: the ticketed tasks above.
  uint32_t* ptab;
  uint32_t piece_shift;
  uint32_t one_shot;
  // byte runs of the pre hash: per wave the first range and the byte offset in it, placed
  // by an extra prep workgroup (run_partial: launch_balance's per-block byte sums, unused then)
  uint64_t* run_partial;
  uint32_t* run_bal;
  uint64_t* run_boff;
  uint32_t run_blocks;
  uint32_t run_waves;   // waves of the hash launches: run_bal / run_boff hold run_waves + 1 entries
  uint32_t runs_used;   // the pre hash ran as byte runs (three-pass pipeline)
  hf3fs_crc_anomaly* diag;  // the self-check's record (finalize audit)
  uint32_t fault_io;        // test only (option fault_io): IO fault_io - 1 hashes its payload from ~0 ^ 1
};
constexpr uint32_t kRunBlocksMax = 64;  // k_bal_sums blocks for the byte runs of 2n pre jobs

// nw: waves of the hash launches (byte-run boundaries)
// ptab_cap: piece-table entries (one-shot apply), 0 for the ticketed apply
size_t update_scratch_bytes(uint64_t n, uint32_t pieces, uint32_t nw, uint64_t ptab_cap);
void update_scratch_carve(void* base, uint64_t n, uint32_t pieces, uint32_t piece_min, uint32_t nw,
                          uint64_t ptab_cap, UpdateScratch* s);
// Piece-table entries a batch of n IOs of at most max_len bytes can need (payload + gap).
uint64_t update_piece_cap(uint64_t n, uint32_t max_len, uint32_t piece_shift);

// prep for every IO; with place_runs (2n <= kPrepRunJobs) one extra workgroup places the
// byte runs of the 2n pre jobs over s.run_waves waves meanwhile (s.run_bal / s.run_boff,
// launch_balance's boff form).
constexpr uint32_t kPrepRunJobs = 8192;  // pre jobs the runs workgroup places (8 per thread, in registers)
constexpr uint32_t kPrepThreads = 1024;  // prep workgroup size (the runs workgroup's)
constexpr uint32_t kPrepIoThreads = 256;  // threads per prep workgroup deriving IOs
hipError_t launch_update_prep(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type, int mode,
                              const UpdateScratch& s, bool place_runs, hipStream_t st);
// Copies the verified payloads and zero-fills gaps (apply tasks).  With
// finalize_delta, the apply workgroups also give every IO its payload verdict
// (ChunkReplica.cc:193-207) and finalize every IO that needs no post job
// (:319-394 new checksum): all of DELTA except type-changing recomputes, so only
// those are left for launch_update_finalize(post_only = true).
// hint (pinned host word or null): the apply stores (pieces << 32 | n) there for the next
// call's one-shot grid.  With s.one_shot the grid is one workgroup per piece as far as it
// reaches (more pieces than workgroups: each takes every grid-th piece), and the apply
// finalizes no IO (finalize_delta is ignored: launch_update_finalize with post_only = false);
// ptab_cap: the piece table's capacity (entries), >= grid.
hipError_t launch_update_apply(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type, int mode,
                               const UpdateScratch& s, const DeviceTables* tabs, bool finalize_delta, uint32_t grid,
                               int nt, uint64_t ptab_cap, uint64_t* hint, hipStream_t st);
// Fused prep + payload verify + write (+ delta old-byte hash), one workgroup
// per IO; leaves the scratch as prep -> ranges(pre) -> apply would.
hipError_t launch_update_fused(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type, int mode,
                               const UpdateScratch& s, const DeviceTables* tabs, uint32_t grid, int nt,
                               hipStream_t st);
// New chunk checksums (and the payload verdict).  which: 0 every IO; 1 every verdict and
// the IOs that need no post job; 2 only those whose case-4 recompute needs the post jobs
// (returns at once when no post job exists and there is no audit).  With audit, every IO
// whose status is then a payload checksum mismatch is re-hashed independently; a re-hash
// equal to the client checksum turns the status into HF3FS_CRC_DEVICE_ERROR and fills s.diag.
hipError_t launch_update_finalize(hf3fs_crc_update_io* ios, uint64_t n, uint8_t type, int mode,
                                  const UpdateScratch& s, const DeviceTables* tabs, uint32_t max_len, int which,
                                  bool audit, hipStream_t st);

// AioReadJob::setResult batch: prep selects the reads to hash (addr/len jobs,
// longest job in *maxl), finalize applies the reuse / NONE / recalculate rules.
hipError_t launch_read_prep(hf3fs_crc_read_io* ios, uint64_t n, uint8_t type, uint32_t max_len, uint64_t* addr,
                            uint64_t* len, uint32_t* maxl, hipStream_t st);
hipError_t launch_read_finalize(hf3fs_crc_read_io* ios, uint64_t n, const uint32_t* v, hipStream_t st);

}  // namespace hf3fs_crc
