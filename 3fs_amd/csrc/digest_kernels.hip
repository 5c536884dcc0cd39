// digest_kernels.hip -- file-level digest: the admin `checksum --fill-zero` fold
// (src/client/cli/admin/Checksum.cc:43-88 over FileWrapper::readFile,
// src/client/cli/admin/FileWrapper.cc:119-164) as a segmented two-pass device
// reduction, one segment (file or replica) per digest.
//
// Per block (FileWrapper.cc:133-160), with returned checksum {t, v} over r read
// bytes of an expected L:
//   r == L : e = {t, v}
//   r <  L : e = {t, v}.combine(create(CRC32C, zeros, L - r), L - r), i.e.
//            t == NONE   -> {CRC32C, ~0 * x^(8 (L - r))}   (the r bytes are not hashed)
//            t == CRC32C -> {CRC32C,  v * x^(8 (L - r))}
//            t == CRC32  -> kChecksumMismatch
//   then S.combine(e, L)  (Common.h:179-198: type check first, then length 0 is a
//   no-op, NONE state copies e, else S.v = combine(~S.v, e.v, L)).
// The left fold is made associative by summarising a run of blocks as
//   - before its first typed block with L > 0: the set of types seen (`pre`)
//     and the last NONE block with L > 0 (`nv`, what a NONE state would copy);
//   - from that block on: its type `tf` and the raw concatenation (v, len),
//     (a, La).(b, Lb) = ((~a) x^(8 Lb) ^ b, La + Lb);
// and joining A.B checks B's types against A.tf when A is typed.
// Without --fill-zero (FileWrapper.cc:134-139,153-160) a pre-pass finds each
// file's first block that is missing or of another length than expected
// (atomicMin of index << 2 | code), and the fold runs over the blocks before
// it; a type mismatch there comes first, else that block's error is the status.
#include "digest_kernels.h"

namespace hf3fs_crc {
namespace {

constexpr uint8_t kHasTyped = 1, kHasNv = 2;
constexpr uint8_t kErrMismatch = 1, kErrInvalid = 2;
constexpr uint64_t kNoErr = ~0ull;                       // first-error word: none
constexpr uint64_t kCodeMissing = 1, kCodeLength = 2;    // index << 2 | code

struct Sum {
  uint64_t len;  // bytes from the first typed block on
  uint32_t v;    // raw value of those bytes
  uint32_t nv;   // value of the last NONE block with L > 0 (state stays NONE)
  uint8_t flags, tf, pre, err;
  uint32_t pad;
};
static_assert(sizeof(Sum) == 24, "partial layout");

__device__ __forceinline__ uint32_t xpow8(uint64_t nbytes, const PolyTables* T, uint32_t poly) {
  return xpow8_bytes((int64_t)nbytes, T, poly);
}

__device__ __forceinline__ Sum identity() { return Sum{0, 0, 0, 0, 0, 0, 0, 0}; }

__device__ Sum join(const Sum& a, const Sum& b, const DeviceTables* tabs) {
  Sum r = a;
  r.err = a.err | b.err;
  if (a.flags & kHasTyped) {
    if (b.pre & ~(1u << a.tf)) r.err |= kErrMismatch;
    if (b.flags & kHasTyped) {
      if (b.tf != a.tf) r.err |= kErrMismatch;
      const uint32_t poly = poly_of(a.tf);
      r.v = gf_mul(~a.v, xpow8(b.len, &tabs->poly[a.tf == kTypeCrc32 ? 1 : 0], poly), poly) ^ b.v;
      r.len = a.len + b.len;
    }
    return r;
  }
  if (b.flags & kHasTyped) {
    r = b;
    r.err = a.err | b.err;
    r.pre = a.pre | b.pre;
    return r;
  }
  r.pre = a.pre | b.pre;
  if (b.flags & kHasNv) r.nv = b.nv;
  r.flags |= b.flags & kHasNv;
  return r;
}

__device__ Sum of_block(const hf3fs_crc_block_digest& bd, const DeviceTables* tabs) {
  Sum s = identity();
  const uint64_t L = bd.block_len;
  // a missing chunk with --fill-zero: nothing read, the default checksum {NONE, 0} (:134-135)
  const uint64_t r = bd.missing ? 0 : bd.read_len;
  uint8_t t = bd.missing ? kTypeNone : bd.checksum_type;
  uint32_t v = bd.missing ? 0u : bd.checksum;
  if (bd.checksum_type > kTypeCrc32) {
    s.err = kErrInvalid;
    return s;
  }
  if (r > L) {
    s.err = kErrInvalid;  // needFill would underflow (reference: undefined)
    return s;
  }
  if (r < L) {  // zero fill with CRC32C (FileWrapper.cc:151-153)
    const uint64_t fill = L - r;
    const uint32_t z = xpow8(fill, &tabs->poly[0], kPolyCrc32c);
    if (t == kTypeNone) {
      t = kTypeCrc32c;
      v = gf_mul(~0u, z, kPolyCrc32c);
    } else if (t == kTypeCrc32c) {
      v = gf_mul(v, z, kPolyCrc32c);
    } else {
      s.err = kErrMismatch;
      return s;
    }
  }
  if (t != kTypeNone && L > 0) {
    s.flags = kHasTyped;
    s.tf = t;
    s.v = v;
    s.len = L;
  } else {
    s.pre = (uint8_t)(1u << t);
    if (t == kTypeNone && L > 0) {
      s.flags = kHasNv;
      s.nv = v;
    }
  }
  return s;
}

// Ordered workgroup reduction (blockDim = 256).
__device__ Sum block_reduce(Sum s, const DeviceTables* tabs) {
  __shared__ Sum sh[256];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (unsigned d = 1; d < 256; d <<= 1) {
    const bool act = (threadIdx.x & (2 * d - 1)) == 0;
    Sum r;
    if (act) r = join(sh[threadIdx.x], sh[threadIdx.x + d], tabs);
    __syncthreads();
    if (act) sh[threadIdx.x] = r;
    __syncthreads();
  }
  return sh[0];
}

// fe: the file's first-error word (strict mode) or kNoErr.
__device__ void emit(const Sum& s, uint64_t file_len, uint64_t fe, hf3fs_crc_file_digest* out) {
  hf3fs_crc_file_digest o{};
  o.length = file_len;
  o.status = (s.err & kErrInvalid) ? HF3FS_CRC_INVALID_ARG : (s.err & kErrMismatch) ? HF3FS_CRC_CHECKSUM_MISMATCH : 0;
  if (o.status == 0 && fe != kNoErr)
    o.status = (fe & 3) == kCodeMissing ? HF3FS_CRC_CHUNK_NOT_FOUND : HF3FS_CRC_INVALID_FORMAT;
  if (o.status == 0) {
    if (s.flags & kHasTyped) {
      o.type = s.tf;
      o.value = s.v;
    } else {
      o.type = kTypeNone;
      o.value = (s.flags & kHasNv) ? s.nv : 0u;
    }
  }
  *out = o;
}

// Strict mode: first[f] = ~0, then the first missing / wrong-length block of
// each file (same slicing as pass 1).
__global__ void k_digest_first_init(uint64_t* __restrict__ first, uint64_t nfiles) {
  for (uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; f < nfiles; f += (uint64_t)gridDim.x * blockDim.x)
    first[f] = kNoErr;
}

__global__ __launch_bounds__(256) void k_digest_first_err(const hf3fs_crc_block_digest* __restrict__ blocks,
                                                          const uint64_t* __restrict__ file_off, uint32_t splits,
                                                          uint64_t* __restrict__ first) {
  const uint64_t f = blockIdx.x / splits, p = blockIdx.x % splits;
  const uint64_t b0 = file_off[f], b1 = file_off[f + 1];
  const uint64_t nb = b1 > b0 ? b1 - b0 : 0;
  const uint64_t span = (nb + splits - 1) / splits;
  const uint64_t s0 = b0 + p * span, s1 = min(b1, s0 + span);
  const uint64_t run = (span + 255) / 256;
  uint64_t m = kNoErr;
  for (uint64_t i = s0 + threadIdx.x * run, e = min(s1, i + run); i < e; ++i) {
    const hf3fs_crc_block_digest bd = blocks[i];
    if (bd.missing || bd.read_len != bd.block_len) {
      m = ((i - b0) << 2) | (bd.missing ? kCodeMissing : kCodeLength);
      break;  // runs are in order: the thread's first one is its least
    }
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    const uint64_t o = __shfl_xor(m, d, 64);
    m = o < m ? o : m;
  }
  if ((threadIdx.x & 63) == 0 && m != kNoErr) atomicMin(reinterpret_cast<unsigned long long*>(first + f), m);
}

// Pass 1: workgroup (file f, split p) folds its slice of f's blocks; each
// thread a contiguous run, then the ordered workgroup tree.  With one split
// the workgroup emits the digest directly.  first (strict mode): blocks from
// the file's first error on contribute only an unknown-type check.
__global__ __launch_bounds__(256) void k_digest_pass1(const hf3fs_crc_block_digest* __restrict__ blocks,
                                                      const uint64_t* __restrict__ file_off, uint32_t splits,
                                                      Sum* __restrict__ part, hf3fs_crc_file_digest* __restrict__ out,
                                                      const DeviceTables* __restrict__ tabs,
                                                      const uint64_t* __restrict__ first) {
  const uint64_t f = blockIdx.x / splits, p = blockIdx.x % splits;
  const uint64_t b0 = file_off[f], b1 = file_off[f + 1];
  const uint64_t nb = b1 > b0 ? b1 - b0 : 0;
  const uint64_t span = (nb + splits - 1) / splits;
  const uint64_t s0 = b0 + p * span, s1 = min(b1, s0 + span);
  const uint64_t run = (span + 255) / 256;
  const uint64_t fe = first ? first[f] : kNoErr;
  const uint64_t limit = fe == kNoErr ? ~0ull : (fe >> 2);  // blocks [0, limit) of the file are folded
  Sum acc = identity();
  uint64_t bytes = 0;
  for (uint64_t i = s0 + threadIdx.x * run, e = min(s1, i + run); i < e; ++i) {
    const hf3fs_crc_block_digest bd = blocks[i];
    bytes += bd.block_len;
    if (i - b0 < limit) {
      acc = join(acc, of_block(bd, tabs), tabs);
    } else if (bd.checksum_type > kTypeCrc32) {
      acc.err |= kErrInvalid;
    }
  }
  // the file length is a plain sum; carry it in `pad`-free form via a second reduction
  __shared__ unsigned long long total;
  if (threadIdx.x == 0) total = 0;
  __syncthreads();
  if (bytes) atomicAdd(&total, (unsigned long long)bytes);
  const Sum w = block_reduce(acc, tabs);  // contains __syncthreads
  if (threadIdx.x == 0) {
    if (splits == 1) {
      emit(w, total, fe, out + f);
    } else {
      Sum o = w;
      o.pad = 0;
      part[blockIdx.x] = o;
      reinterpret_cast<unsigned long long*>(part + gridDim.x)[blockIdx.x] = total;
    }
  }
}

// Pass 2: one thread per file folds its `splits` partials in order.
__global__ __launch_bounds__(256) void k_digest_pass2(const Sum* __restrict__ part, uint64_t nfiles, uint32_t splits,
                                                      hf3fs_crc_file_digest* __restrict__ out,
                                                      const DeviceTables* __restrict__ tabs,
                                                      const uint64_t* __restrict__ first) {
  const uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nfiles) return;
  const unsigned long long* lens = reinterpret_cast<const unsigned long long*>(part + nfiles * splits);
  Sum acc = identity();
  uint64_t total = 0;
  for (uint32_t p = 0; p < splits; ++p) {
    acc = join(acc, part[f * splits + p], tabs);
    total += lens[f * splits + p];
  }
  emit(acc, total, first ? first[f] : kNoErr, out + f);
}

// Small files (max_blocks <= kWaveFileBlocks): one WAVE per file, four files per workgroup.
// Lane l folds its contiguous run of the file's blocks, then the ordered tree runs over the
// wave in registers (DPP / permute shuffles, no LDS, no barrier): a 64-block file pays 6 join
// levels instead of the workgroup tree's 8 levels and 16 barriers, and 3/4 of a 256-thread
// workgroup no longer idles.  Same Sum algebra, same results.
constexpr uint32_t kWaveFileBlocks = 1024;

__device__ __forceinline__ Sum shfl_down_sum(const Sum& s, int d) {
  Sum r;
  r.len = __shfl_down(s.len, d, 64);
  r.v = __shfl_down(s.v, d, 64);
  r.nv = __shfl_down(s.nv, d, 64);
  const uint32_t packed = (uint32_t)s.flags | (uint32_t)s.tf << 8 | (uint32_t)s.pre << 16 | (uint32_t)s.err << 24;
  const uint32_t q = __shfl_down(packed, d, 64);
  r.flags = (uint8_t)q;
  r.tf = (uint8_t)(q >> 8);
  r.pre = (uint8_t)(q >> 16);
  r.err = (uint8_t)(q >> 24);
  r.pad = 0;
  return r;
}

// Strict mode: the first missing / wrong-length block of each file, one wave per file.
__global__ __launch_bounds__(256) void k_digest_first_err_wave(const hf3fs_crc_block_digest* __restrict__ blocks,
                                                               const uint64_t* __restrict__ file_off, uint64_t nfiles,
                                                               uint64_t* __restrict__ first) {
  const uint64_t f = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (f >= nfiles) return;  // wave-uniform
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b0 = file_off[f], b1 = file_off[f + 1];
  const uint64_t nb = b1 > b0 ? b1 - b0 : 0, run = (nb + 63) / 64;
  uint64_t m = kNoErr;
  for (uint64_t i = b0 + lane * run, e = min(b1, i + run); i < e; ++i) {
    const hf3fs_crc_block_digest bd = blocks[i];
    if (bd.missing || bd.read_len != bd.block_len) {
      m = ((i - b0) << 2) | (bd.missing ? kCodeMissing : kCodeLength);
      break;
    }
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    const uint64_t o = __shfl_xor(m, d, 64);
    m = o < m ? o : m;
  }
  if (lane == 0) first[f] = m;
}

__global__ __launch_bounds__(256) void k_digest_wave(const hf3fs_crc_block_digest* __restrict__ blocks,
                                                     const uint64_t* __restrict__ file_off, uint64_t nfiles,
                                                     hf3fs_crc_file_digest* __restrict__ out,
                                                     const DeviceTables* __restrict__ tabs,
                                                     const uint64_t* __restrict__ first) {
  const uint64_t f = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (f >= nfiles) return;  // wave-uniform: no barrier below
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b0 = file_off[f], b1 = file_off[f + 1];
  const uint64_t nb = b1 > b0 ? b1 - b0 : 0, run = (nb + 63) / 64;
  const uint64_t fe = first ? first[f] : kNoErr;
  const uint64_t limit = fe == kNoErr ? ~0ull : (fe >> 2);  // blocks [0, limit) of the file are folded
  Sum acc = identity();
  uint64_t bytes = 0;
  for (uint64_t i = b0 + lane * run, e = min(b1, i + run); i < e; ++i) {
    const hf3fs_crc_block_digest bd = blocks[i];
    bytes += bd.block_len;
    if (i - b0 < limit) {
      acc = join(acc, of_block(bd, tabs), tabs);
    } else if (bd.checksum_type > kTypeCrc32) {
      acc.err |= kErrInvalid;
    }
  }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {  // ordered: lane l joins lane l + d's summary on its right
    const Sum o = shfl_down_sum(acc, d);
    if ((lane & (2 * d - 1)) == 0) acc = join(acc, o, tabs);
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) bytes += __shfl_xor(bytes, d, 64);
  if (lane == 0) emit(acc, bytes, fe, out + f);
}

}  // namespace

size_t digest_scratch_bytes(uint64_t nfiles, uint32_t splits, bool fill_zero) {
  const size_t parts = splits > 1 ? (size_t)nfiles * splits * (sizeof(Sum) + sizeof(uint64_t)) : 0;
  return parts + (fill_zero ? 0 : (size_t)nfiles * sizeof(uint64_t));
}

uint32_t digest_splits(uint64_t max_blocks) {
  // ~2048 blocks per workgroup, at most 64 workgroups per file
  const uint64_t s = (max_blocks + 2047) / 2048;
  return (uint32_t)(s < 1 ? 1 : (s > 64 ? 64 : s));
}

hipError_t launch_file_digest(const hf3fs_crc_block_digest* blocks, const uint64_t* file_off, uint64_t nfiles,
                              uint64_t max_blocks, uint32_t splits, bool fill_zero, void* scratch,
                              hf3fs_crc_file_digest* out, const DeviceTables* tabs, hipStream_t s) {
  if (max_blocks <= kWaveFileBlocks) {  // splits == 1: one wave per file
    uint64_t* first = fill_zero ? nullptr : static_cast<uint64_t*>(scratch);
    const uint32_t g = (uint32_t)((nfiles + 3) / 4);
    if (!fill_zero)
      hipLaunchKernelGGL(k_digest_first_err_wave, dim3(g), dim3(256), 0, s, blocks, file_off, nfiles, first);
    hipLaunchKernelGGL(k_digest_wave, dim3(g), dim3(256), 0, s, blocks, file_off, nfiles, out, tabs,
                       (const uint64_t*)first);
    return hipGetLastError();
  }
  Sum* part = static_cast<Sum*>(scratch);
  uint64_t* first = nullptr;
  if (!fill_zero) {
    first = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(scratch) +
                                        (splits > 1 ? (size_t)nfiles * splits * (sizeof(Sum) + sizeof(uint64_t)) : 0));
    const uint64_t g = (nfiles + 255) / 256;
    hipLaunchKernelGGL(k_digest_first_init, dim3((uint32_t)(g < 4096 ? g : 4096)), dim3(256), 0, s, first, nfiles);
    hipLaunchKernelGGL(k_digest_first_err, dim3((uint32_t)(nfiles * splits)), dim3(256), 0, s, blocks, file_off,
                       splits, first);
  }
  hipLaunchKernelGGL(k_digest_pass1, dim3((uint32_t)(nfiles * splits)), dim3(256), 0, s, blocks, file_off, splits,
                     part, out, tabs, (const uint64_t*)first);
  if (splits > 1)
    hipLaunchKernelGGL(k_digest_pass2, dim3((uint32_t)((nfiles + 255) / 256)), dim3(256), 0, s, part, nfiles, splits,
                       out, tabs, (const uint64_t*)first);
  return hipGetLastError();
}

}  // namespace hf3fs_crc
