// aux_kernels.h -- prep/finalize kernels around k_crc_ranges for the callers on
// either side of the chunk-checksum path: serde frame checksums
// (f4) and scrubbing stored chunks against their persisted checksums (f3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hf3fs_crc.h"

namespace hf3fs_crc {

// Frames: job i = (base + offset_i, size_i); longest job -> *maxl.
hipError_t launch_frame_prep(const uint8_t* base, hf3fs_crc_frame* frames, uint64_t n, uint32_t max_size,
                             uint64_t* addr, uint64_t* len, uint32_t* maxl, hipStream_t st);
// computed = calcSerde(v_i) (MessageHeader.h:33-37), status/count vs the header.
hipError_t launch_frame_finalize(hf3fs_crc_frame* frames, uint64_t n, const uint32_t* v, uint32_t* count,
                                 hipStream_t st);

// Scrub: job i = (data_i, length_i) for typed chunks, empty for NONE.
hipError_t launch_scrub_prep(hf3fs_crc_scrub_io* ios, uint64_t n, uint8_t type, uint32_t max_len, uint64_t* addr,
                             uint64_t* len, uint32_t* maxl, hipStream_t st);
hipError_t launch_scrub_finalize(hf3fs_crc_scrub_io* ios, uint64_t n, const uint32_t* v, uint32_t* count,
                                 hipStream_t st);

// Digest tables: n raw values -> n serde ChecksumInfo records (6 bytes each),
// and raw <-> finalized in place.
hipError_t launch_serialize(uint8_t type, const uint32_t* values, uint64_t n, uint8_t* out, hipStream_t st);
hipError_t launch_finalize_values(uint32_t* values, uint64_t n, hipStream_t st);

}  // namespace hf3fs_crc
