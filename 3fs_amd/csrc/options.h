// options.h -- tuning and test switches of libhf3fs_crc.so.
//
// Every switch is read ONCE per process, from HF3FS_CRC_<NAME> at the library's
// first call; a call never looks at the environment.  hf3fs_crc_set_option()
// (include/hf3fs_crc.h) overrides one for every later call -- the tests and the
// in-process A/B scripts use it.  Values are atomics: an override is seen by
// the next call of any thread.
#pragma once
#include <atomic>
#include <stdint.h>

namespace hf3fs_crc {

struct Options {
  std::atomic<int> nt{1};                  // nt: non-temporal streamed loads (profiles/r01_ab_bulk.json)
  std::atomic<uint32_t> seg_kib{0};        // seg_kib: fixed task size, 0 = the planner
  std::atomic<int> static_stride{0};       // static: static stride instead of tickets for ragged task sets
  std::atomic<int> pipe{-1};               // pipe: cross-task head prefetch, -1 = ranges <= 16 KiB, 0 never, 1 always
  std::atomic<int> balance{1};             // balance: byte-balanced task runs for > 16 whole-range tasks per wave
  std::atomic<int> record_direct{1};       // record_direct: whole-buffer record jobs
  std::atomic<int> update_pipeline{-1};    // update_pipeline: -1 per mode (DELTA unfused, REFERENCE fused), 0, 1
  std::atomic<uint32_t> apply_pieces{8};   // apply_pieces: most apply pieces per range
  std::atomic<uint32_t> apply_min_kib{64}; // apply_min_kib: smallest apply piece
  std::atomic<uint32_t> apply_nt{6};       // apply_nt: bit 0 nt payload loads, bit 1 nt stores, bit 2 hw body (A/B)
  std::atomic<int> apply_grid{-1};         // apply_grid: -1 one-shot apply once a call on the (stream, thread) has
                                           // counted pieces, 0 ticketed tasks, 1 one-shot always, 2 (test) one-shot
                                           // on a small grid (every workgroup takes several pieces)
  std::atomic<uint32_t> apply_piece_kib{8};  // apply_piece_kib: one-shot piece (4, 8 or 16 KiB)
  std::atomic<uint32_t> prehash_rep{1};    // prehash_rep: byte runs per wave of the update pre hash (A/B)
  std::atomic<int> frame_stream{-1};       // frame_stream: -1 = for >= 256 frames, 0 never, 1 always
  std::atomic<uint32_t> frame_segw{2};     // frame_segw: segments per wave of the frame stream path
  std::atomic<int> debug{0};               // debug: update pipeline diagnostics on stderr
  std::atomic<uint32_t> poison{0};         // poison (test only): fill every call scratch with this word first
  std::atomic<int> audit{1};               // audit: re-hash every payload reported as mismatched (§7)
  std::atomic<int> range_stream{0};        // range_stream: balanced whole-range tasks as one block stream per wave
  std::atomic<int> list_runs{0};           // list_runs: create_batch hashes its ranges as byte runs (A/B, probes)
  std::atomic<uint32_t> fault_io{0};       // fault_io (test only): IO fault_io - 1 of every update batch hashes
                                           // its payload from a wrong start value (exercises the audit)
};

// The process's switches (environment snapshot taken on the first call).
Options& options();

}  // namespace hf3fs_crc
