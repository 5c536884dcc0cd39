// frame_kernels.h -- serde frame checksum verification:
// Checksum::calcSerde of every payload of a received buffer, compared with its
// MessageHeader (src/common/net/Processor.h:111-120, MessageHeader.h:33-37).
//
// Two device paths, chosen on the device per batch:
//  * stream (frames sorted and non-overlapping, all sizes <= max_size -- what
//    the framing walk produces): the receive span is hashed ONCE as contiguous
//    1 KiB blocks in byte segments (no per-frame load latency), and at every
//    frame boundary p the wave records E(p) = lin(segment bytes before the
//    16 B granule of p) referenced to the end of p's block.  A per-frame
//    finalize turns two boundaries into the payload's CRC:
//      lin(frame) = Q(e) ^ Q(s) * x^(8 size)   (same segment)
//  * record (anything else): one k_crc_ranges job per frame.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hf3fs_crc.h"
#include "crc_kernels.h"

namespace hf3fs_crc {

// Written by the map kernel when the stream path runs.
struct FrameStreamParams {
  uint64_t a0;    // segment grid origin: the 1 KiB block holding lo
  uint64_t seg;   // segment bytes, a multiple of 1 KiB
  uint64_t nseg;  // segments covering [lo, hi]
  uint64_t lo;    // first payload byte (absolute address)
  uint64_t hi;    // one past the last payload byte
};

// Batches below this many frames take the record path (HF3FS_CRC_FRAME_STREAM=1/0 forces).
constexpr uint64_t kFrameStreamMinFrames = 256;
// Segments per wave (each wave takes a contiguous run of them; nseg <= segw
// waves); HF3FS_CRC_FRAME_SEGW overrides (tuning).
constexpr uint64_t kFrameSegsPerWave = 2;
inline uint64_t frame_stream_cap(uint64_t waves, uint64_t segw) { return segw * waves + 4; }
// Payloads spanning more segments than this read the segment prefix table.
constexpr uint64_t kFrameHornerSegs = 16;
// A payload starting at most this many bytes after the previous one ends (the
// 8-byte MessageHeader of walked frames) is not a boundary of its own.
constexpr uint64_t kFrameGapMax = 16;
// Blocks with at most this many boundaries compute each one by a masked step
// and a fold; denser blocks fold once and take the lane prefix of the block.
// With the lane-weight fold the prefix path costs about two sparse boundaries
// (in one process, f4 mix: 1 -> 1.154 ms, 2 -> 1.180, 3 -> 1.220;
// profiles/r03_f4_sparse_threshold_ab.log).
constexpr uint32_t kFrameSparse = 1;

// Bytes between walked frames that are not payload: the MessageHeader (MessageHeader.h:13).
constexpr uint64_t kFrameHeaderBytes = 8;

// The batch's 8-word scratch `flags`: [0] longest frame (record path), [1] set
// when the stream path runs (the record kernels then return at once), [2]
// non-zero when the check found frames the stream path cannot take, [3] set
// when a payload spans more than kFrameHornerSegs segments, [4..5] payload
// bytes and [6..7] gap bytes beyond the headers (u64): a batch whose gaps
// exceed its payload stays on the record path.
hipError_t launch_frame_check(const hf3fs_crc_frame* frames, uint64_t n, uint32_t max_size, uint32_t* flags,
                              hipStream_t st);
// Path decision + stream-path segment map, or (record path: not try_stream, a bad or
// sparse batch, a span too long) the record jobs: job i = (base + offset_i, size_i), longest
// job -> flags[0], v[i] = 0 (the hash XORs segment values into it).  Also zeroes *count (the
// finalize's mismatch count), so a batch needs ONE zeroing launch (flags[0..15]; flags[8] is
// the record path's ticket counter).
constexpr uint32_t kFrameFlagWords = 16;
hipError_t launch_frame_map(const uint8_t* base, hf3fs_crc_frame* frames, uint64_t n, uint64_t seg_target,
                            uint64_t waves, uint32_t* flags, FrameStreamParams* prm, uint32_t* seg_first,
                            uint32_t max_size, uint64_t* addr, uint64_t* len, uint32_t* v, uint32_t* count,
                            bool try_stream, hipStream_t st);
// Stream path: boundary values ev[2i] (payload start), ev[2i + 1] (end) and
// seg_lin[k] = lin(segment k) referenced to its end.
hipError_t launch_frame_stream(const uint8_t* base, const hf3fs_crc_frame* frames, uint64_t n,
                               const uint32_t* flags, const FrameStreamParams* prm, const uint32_t* seg_first,
                               uint32_t* seg_lin, uint32_t* ev, uint32_t workgroups, const DeviceTables* tabs,
                               hipStream_t st);
// seg_pre[k] = lin(segments before k) when flags[3] (one workgroup).
hipError_t launch_frame_seg_scan(const uint32_t* flags, const FrameStreamParams* prm, const uint32_t* seg_lin,
                                 uint32_t* seg_pre, const DeviceTables* tabs, hipStream_t st);
// computed = calcSerde (from v on the record path, from the boundaries on the
// stream path), status/count vs the header.
hipError_t launch_frame_finalize(const uint8_t* base, hf3fs_crc_frame* frames, uint64_t n, const uint32_t* v,
                                 const uint32_t* flags, const FrameStreamParams* prm, const uint32_t* ev,
                                 const uint32_t* seg_lin, const uint32_t* seg_pre, uint32_t* count,
                                 const DeviceTables* tabs, hipStream_t st);

}  // namespace hf3fs_crc
