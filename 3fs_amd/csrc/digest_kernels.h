// digest_kernels.h -- file-level digest reduction (see digest_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/hf3fs_crc.h"
#include "crc_kernels.h"

namespace hf3fs_crc {

uint32_t digest_splits(uint64_t max_blocks);
// fill_zero = false adds a per-file first-error word (the strict mode's scan)
size_t digest_scratch_bytes(uint64_t nfiles, uint32_t splits, bool fill_zero);
// max_blocks <= 1024: one wave per file; else one workgroup per (file, split) + a pass over splits
hipError_t launch_file_digest(const hf3fs_crc_block_digest* blocks, const uint64_t* file_off, uint64_t nfiles,
                              uint64_t max_blocks, uint32_t splits, bool fill_zero, void* scratch,
                              hf3fs_crc_file_digest* out, const DeviceTables* tabs, hipStream_t s);

}  // namespace hf3fs_crc
