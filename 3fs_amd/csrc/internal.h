// internal.h -- helpers shared by the host-side translation units of libhf3fs_crc.so.
#pragma once

namespace hf3fs_crc {

struct DeviceTables;

// Records `msg` as the calling thread's hf3fs_crc_last_error() and returns code
// (host_codec.cc).
int set_error(int code, const char* msg);
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// Constant tables of the calling thread's current device (context created on first use).
int current_tables(const DeviceTables** out);

}  // namespace hf3fs_crc
