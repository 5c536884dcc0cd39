// update_kernels.hip -- batched ChunkReplica::update / updateChecksum on HBM-resident chunks.
//
// Pipeline per batch (hf3fs_crc_update_batch):
//   prep      derive each IO's effective sizes / case (ChunkReplica.cc:319-394),
//             emit "pre" hash jobs: payload (verify, :193-207) and, for the
//             delta method, the old bytes about to be overwritten / truncated;
//   ranges    hash the pre jobs (crc_kernels.hip);
//   apply     copy verified payloads into the chunks, zero-fill gaps (:281-292);
//   ranges    hash the "post" jobs: prefix [0,off) and suffix [off+len,size)
//             of the written chunk (reference algorithm :356-389);
//   finalize  pick the case and stitch the new chunk checksum with GF(2) shifts.
#include "update_kernels.h"


#include "crc_device.h"

#include <algorithm>

namespace hf3fs_crc {
namespace {

struct Eff {
  uint32_t s0, s1;          // chunk size before / after
  uint32_t off, len;        // the UpdateIO as updateChecksum sees it (truncate: off = size, len = 0)
  uint32_t wval, cval;      // write / chunk checksum values
  uint32_t zero_from, zero_to;
  uint8_t wtype, ctype;
  uint8_t kase;             // 1 none/empty, 2 reuse, 3 append-combine, 4 recompute
  bool delta;               // case 4 via the delta identity
  bool verify;              // payload checksum must be verified
  bool te;                  // truncate / extend
  bool ok;                  // IO is well formed
  bool engine;              // chunk-engine semantics (HF3FS_UPDATE_FLAG_ENGINE)
  bool hash_payload;        // the payload job must run (verify, or engine without_checksum)
};

__device__ __forceinline__ Eff derive(const hf3fs_crc_update_io& io, uint32_t max_len, uint8_t type, int mode) {
  Eff e{};
  e.s0 = io.chunk_size;
  e.ctype = io.chunk_checksum_type;
  e.cval = io.chunk_checksum;
  e.ok = true;
  e.zero_from = e.zero_to = 0;
  // The batch hashes bytes in `type`: a write's payload and (when the types differ)
  // its prefix / suffix recompute, ChunkReplica.cc:340,356-392 -- the chunk's stored
  // type may differ for a write; a truncate / extend hashes in the chunk's type.
  if (io.chunk_size > max_len || e.ctype > kTypeCrc32) e.ok = false;
  if (io.update_type != HF3FS_UPDATE_WRITE && e.ctype != kTypeNone && e.ctype != type) e.ok = false;
  if (io.update_type == HF3FS_UPDATE_WRITE) {
    // ChunkReplica.cc:139-145: offset >= chunkSize || offset + length > chunkSize -> kInvalidArg
    if (io.offset >= max_len || (uint64_t)io.offset + io.length > max_len) e.ok = false;
    if (io.length && !io.payload) e.ok = false;
    if (io.write_checksum_type != kTypeNone && io.write_checksum_type != type) e.ok = false;
    e.off = io.offset;
    e.len = io.length;
    e.s1 = e.s0 > io.offset + io.length ? e.s0 : io.offset + io.length;
    if (io.offset > e.s0) {
      e.zero_from = e.s0;
      e.zero_to = io.offset;
    }
    e.wtype = io.write_checksum_type;
    e.wval = io.write_checksum;
    e.verify = e.wtype != kTypeNone && e.len != 0;
  } else if (io.update_type == HF3FS_UPDATE_TRUNCATE || io.update_type == HF3FS_UPDATE_EXTEND) {
    const uint32_t target = io.length;  // ChunkReplica.cc:255-269
    if (target > max_len) e.ok = false;
    if (target <= e.s0) {
      e.s1 = io.update_type == HF3FS_UPDATE_TRUNCATE ? target : e.s0;
    } else {
      e.s1 = target;
      e.zero_from = e.s0;
      e.zero_to = target;
    }
    e.te = true;
    e.wtype = e.ctype;  // create(meta.checksumType, nullptr, 0) (:328-332)
    e.wval = e.ctype == kTypeNone ? 0u : ~0u;
    e.off = e.s1;
    e.len = 0;
  } else {
    e.ok = false;
  }
  e.hash_payload = e.verify;
  const bool is_append = io.offset == e.s0;  // :243, before the write
  if (io.flags & HF3FS_UPDATE_FLAG_ENGINE) {
    // ChunkEngine.cc:41-45: a CRC32C write checksum is verified (engine.rs:297-311), anything else
    // is "without_checksum" -- hashed and used.  The stored checksum is always the CRC32C of the
    // chunk bytes (chunk.rs:89-281), an empty chunk included (~0 raw).
    e.engine = true;
    if (type != kTypeCrc32c) e.ok = false;
    e.ctype = kTypeCrc32c;
    if (e.s0 == 0) e.cval = ~0u;
    if (!e.te) {
      e.verify = io.write_checksum_type == kTypeCrc32c && e.len != 0;
      e.hash_payload = e.len != 0;
      if (e.wtype != kTypeCrc32c) e.ok = e.ok && io.write_checksum_type == kTypeNone;
    }
    e.wtype = kTypeCrc32c;
    if (e.te) e.wval = ~0u;
    if (e.s1 == 0)
      e.kase = 1;
    else if (e.off == 0 && e.len == e.s1)
      e.kase = 2;  // copy_on_write skip_read: reuse (chunk.rs:110,150-155)
    else if (e.s0 > 0 && is_append)
      e.kase = 3;  // direct / indirect append: combine (chunk.rs:229,266)
    else
      e.kase = 4;
    e.delta = e.kase == 4 && mode == HF3FS_UPDATE_MODE_DELTA;
    return e;
  }
  const bool combine = e.s0 > 0 && is_append;
  if (e.wtype == kTypeNone || e.s1 == 0)
    e.kase = 1;
  else if (e.off == 0 && e.len == e.s1)
    e.kase = 2;
  else if (e.wtype == e.ctype && combine)
    e.kase = 3;
  else
    e.kase = 4;
  e.delta = e.kase == 4 && mode == HF3FS_UPDATE_MODE_DELTA && (e.s0 == 0 || e.ctype == e.wtype);
  return e;
}

template <uint32_t POLY>
__device__ __forceinline__ uint32_t xpow8(int64_t nbytes, const PolyTables* T) {
  return xpow8_bytes(nbytes, T, POLY);
}

// ChecksumInfo::combine on raw values of one type (Common.h:179-198).
template <uint32_t POLY>
__device__ __forceinline__ uint32_t ck_combine(uint32_t a, uint32_t b, uint32_t len, const PolyTables* T) {
  return len == 0 ? a : gf_mul(~a, xpow8<POLY>(len, T), POLY) ^ b;
}

// k_update_prep for one IO: status and output defaults, the "pre" jobs
// (payload; old bytes for the delta method) and the "post" jobs (prefix +
// suffix after the write, reference algorithm).  Returns the derived IO.
__device__ __forceinline__ Eff prep_one(hf3fs_crc_update_io* __restrict__ ios, uint64_t i, uint32_t max_len,
                                        uint8_t type, int mode, const UpdateScratch& s) {
  hf3fs_crc_update_io io = ios[i];
  const Eff e = derive(io, max_len, type, mode);
  io.status = e.ok ? HF3FS_CRC_OK : HF3FS_CRC_INVALID_ARG;
  io.out_size = io.chunk_size;
  io.out_checksum = io.chunk_checksum;
  io.out_checksum_type = io.chunk_checksum_type;
  ios[i] = io;
  uint64_t a0 = 0, l0 = 0, a1 = 0, l1 = 0, pa = 0, pl = 0, sa = 0, sl = 0;
  if (e.ok) {
    if (e.hash_payload) {
      a0 = io.payload;
      l0 = e.len;
    }
    if (e.kase == 4 && e.delta) {
      if (!e.te && e.off < e.s0) {  // old bytes under the write
        a1 = io.chunk + e.off;
        l1 = (e.off + e.len < e.s0 ? e.off + e.len : e.s0) - e.off;
      } else if (e.te && e.s1 < e.s0) {  // truncated tail
        a1 = io.chunk + e.s1;
        l1 = e.s0 - e.s1;
      }
    } else if (e.kase == 4) {  // reference: prefix + suffix after the write
      const uint32_t suffix_start = e.off + e.len < e.s1 ? e.off + e.len : e.s1;
      pa = io.chunk;
      pl = e.off;
      sa = io.chunk + suffix_start;
      sl = e.s1 - suffix_start;
    }
  }
  s.pre_addr[2 * i] = a0;
  s.pre_len[2 * i] = l0;
  s.pre_start[2 * i] = ~0u;
  s.pre_addr[2 * i + 1] = a1;
  s.pre_len[2 * i + 1] = l1;
  s.pre_start[2 * i + 1] = 0u;
  s.post_addr[2 * i] = pa;
  s.post_len[2 * i] = pl;
  s.post_start[2 * i] = ~0u;
  s.post_addr[2 * i + 1] = sa;
  s.post_len[2 * i + 1] = sl;
  s.post_start[2 * i + 1] = ~0u;
  const uint64_t pre_max = l0 > l1 ? l0 : l1, post_max = pl > sl ? pl : sl;
  if (pre_max) atomicMax(&s.max_len[0], (uint32_t)pre_max);
  if (post_max) atomicMax(&s.max_len[1], (uint32_t)post_max);
  return e;
}

// Apply pieces of a range of len bytes at dst: cuts at 16-byte aligned
// destination addresses, piece j = [max(0, j ps - h), min(len, (j + 1) ps - h)).
__device__ __forceinline__ uint64_t piece_bytes(uint64_t len, const UpdateScratch& s) {
  const uint64_t even = ((len + s.pieces - 1) / s.pieces + 15) & ~uint64_t(15);
  return even > s.piece_min ? even : s.piece_min;
}
__device__ __forceinline__ uint32_t piece_count(uint64_t dst, uint64_t len, const UpdateScratch& s) {
  if (!len) return 0;
  const uint64_t ps = piece_bytes(len, s);
  return (uint32_t)(((dst & 15) + len + ps - 1) / ps);
}

// prep for every IO (one thread each) and the compacted apply task list:
// each wave scans its lanes' piece counts and reserves their slots with one
// atomic.  The loop bound is wave-uniform (blockDim is a multiple of 64).
__global__ __launch_bounds__(256) void k_update_prep(hf3fs_crc_update_io* __restrict__ ios, uint64_t n,
                                                     uint32_t max_len, uint8_t type, int mode, UpdateScratch s) {
  const uint32_t lane = threadIdx.x & 63;
  unsigned long long* count = reinterpret_cast<unsigned long long*>(s.max_len + 2);
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); i0 < n;
       i0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = i0 + lane;
    uint32_t np = 0, ng = 0;
    if (i < n) {
      const Eff e = prep_one(ios, i, max_len, type, mode, s);
      if (e.ok) {
        const uint64_t chunk = ios[i].chunk;
        if (!e.te) np = piece_count(chunk + e.off, e.len, s);
        if (e.zero_to > e.zero_from) ng = piece_count(chunk + e.zero_from, e.zero_to - e.zero_from, s);
      }
    }
    const uint32_t k = np + ng;
    uint32_t incl = k;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d);
      if (lane >= (uint32_t)d) incl += y;
    }
    const uint32_t total = __shfl(incl, 63);
    unsigned long long base = 0;
    if (lane == 63 && total) base = atomicAdd(count, (unsigned long long)total);
    base = __shfl(base, 63);
    uint64_t at = base + incl - k;
    for (uint32_t j = 0; j < np; ++j) s.tasks[at++] = (i << 8) | j;
    for (uint32_t j = 0; j < ng; ++j) s.tasks[at++] = (i << 8) | 0x80u | j;
  }
}

// ---------------------------------------------------------------------------
// byte copy with arbitrary source/destination alignment (doRealWrite on HBM)
// dst[0, len) = src ? src[0, len) : 0, executed by `nthreads` cooperating
// threads (tid = 0..nthreads-1: a workgroup or one wave): full 16-byte
// destination granules are written with aligned dwordx4 stores, four in flight
// per thread; the (at most two) partial granules at the ends byte by byte.
// 16 bytes at byte offset sh (1..15) into the 32-byte window A:B.
__device__ __forceinline__ u32x4 funnel16(const u32x4& A, const u32x4& B, uint32_t sh) {
  const uint32_t w[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
  const uint32_t q = sh >> 2, r = sh & 3;
  uint32_t t[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) t[k] = q == 0 ? w[k] : q == 1 ? w[k + 1] : q == 2 ? w[k + 2] : w[k + 3];
  u32x4 o;
  o.x = __builtin_amdgcn_alignbyte(t[1], t[0], r);
  o.y = __builtin_amdgcn_alignbyte(t[2], t[1], r);
  o.z = __builtin_amdgcn_alignbyte(t[3], t[2], r);
  o.w = __builtin_amdgcn_alignbyte(t[4], t[3], r);
  return o;
}

// Copy rows of full destination granules from a source misaligned by sh != 0
// with ONE aligned source load per granule: a wave's 64 lanes cover 64
// consecutive granules, lane l takes the upper neighbour granule from lane
// l + 1 (ds_bpermute) and lane 63 loads it.  Returns the first granule index
// (per thread) not yet copied; only wave-uniform rows are taken here.
template <int U, bool NT>
__device__ __forceinline__ uint64_t copy_rows_shfl(uint64_t gdst, uint64_t sg0, uint32_t sh, uint64_t ng,
                                                   uint64_t g, uint64_t stride) {
  const uint32_t lane = (uint32_t)(g & 63);  // stride and the thread's start are multiples of 64 apart
  uint64_t gw = g - lane;                    // the wave's first granule of the row
  for (; gw + 63 + (U - 1) * stride < ng; gw += U * stride) {  // wave-uniform
    u32x4 a[U], b[U];
#pragma unroll
    for (int k = 0; k < U; ++k) a[k] = ld16<NT>(sg0 + (gw + lane + k * stride) * 16);
#pragma unroll
    for (int k = 0; k < U; ++k) b[k] = lane == 63 ? ld16<NT>(sg0 + (gw + 64 + k * stride) * 16) : a[k];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const u32x4 nb{(uint32_t)__shfl_down((int)a[k].x, 1, 64), (uint32_t)__shfl_down((int)a[k].y, 1, 64),
                     (uint32_t)__shfl_down((int)a[k].z, 1, 64), (uint32_t)__shfl_down((int)a[k].w, 1, 64)};
      st16<NT>(gdst + (gw + lane + k * stride) * 16, funnel16(a[k], lane == 63 ? b[k] : nb, sh));
    }
  }
  return gw + lane;
}

template <int U = 4, bool NT = false, bool SHFL = false, int ALIGN = 0>
__device__ void copy_range(uint64_t dst, uint64_t src, uint64_t len, uint32_t tid, uint32_t nthreads) {
  const uint64_t d0 = dst, d1 = dst + len;
  const uint64_t gfirst = (d0 + 15) & ~uint64_t(15);  // first full granule
  const uint64_t glast = d1 & ~uint64_t(15);          // end of full granules
  {  // partial head [d0, hend) and tail [tstart, d1): at most 30 bytes, one per thread
    const uint64_t hend = gfirst < d1 ? gfirst : d1;
    const uint64_t tstart = glast >= gfirst ? glast : d1;
    const uint64_t nh = hend - d0, nt = d1 - tstart;
    if (tid < nh + nt) {
      const uint64_t b = tid < nh ? d0 + tid : tstart + (tid - nh);
      *reinterpret_cast<uint8_t*>(b) = src ? *reinterpret_cast<const uint8_t*>(src + (b - d0)) : 0;
    }
  }
  if (glast <= gfirst) return;
  uint64_t gfirst_rows = gfirst;
  if (ALIGN) {  // granules up to the first ALIGN-byte boundary one per thread (ALIGN <= 16 nthreads):
                // every wave row below is 8 whole 128 B lines
    const uint64_t ga0 = (gfirst + ALIGN - 1) & ~uint64_t(ALIGN - 1);
    const uint64_t ga = ga0 < glast ? ga0 : glast;
    if (tid < (ga - gfirst) / 16) {
      const uint64_t gd = gfirst + 16 * (uint64_t)tid;
      st16<NT>(gd, src ? ld16_unaligned<NT>(src + (gd - d0)) : u32x4{0, 0, 0, 0});
    }
    gfirst_rows = ga;
    if (glast <= ga) return;
  }
  const uint64_t ng = (glast - gfirst_rows) / 16;
  const uint64_t soff = gfirst_rows - d0;  // source offset of the first full granule
  const uint64_t stride = nthreads;
  uint64_t g = tid;
  if (SHFL && src && ((src + soff) & 15)) {  // nthreads is a multiple of 64
    const uint64_t s0 = src + soff;
    g = copy_rows_shfl<U, NT>(gfirst_rows, s0 & ~uint64_t(15), (uint32_t)(s0 & 15), ng, g, stride);
  }
  for (; g + (U - 1) * stride < ng; g += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
      v[k] = src ? ld16_unaligned<NT>(src + soff + (g + k * stride) * 16) : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < U; ++k) st16<NT>(gfirst_rows + (g + k * stride) * 16, v[k]);
  }
  for (; g < ng; g += stride)
    st16<NT>(gfirst_rows + g * 16, src ? ld16_unaligned<NT>(src + soff + g * 16) : u32x4{0, 0, 0, 0});
}

// One task = one piece of an IO's payload copy or gap zero-fill (the list
// prep compacted).  Tasks are handed out by a ticket counter (dynamic
// balance) to 256-thread workgroups, eight per CU, so each CU keeps 32 waves'
// worth of loads in flight.  (A/B: one wave per 64 KiB piece on a 16-wave
// persistent grid ran d3 1.5x slower -- half the loads in flight.)
template <int U, bool NT, bool SHFL, int ALIGN>
__global__ __launch_bounds__(256) void k_update_apply(hf3fs_crc_update_io* __restrict__ ios, uint32_t max_len,
                                                      uint8_t type, UpdateScratch s, uint32_t* __restrict__ queue) {
  __shared__ uint32_t ticket;
  const uint64_t ntasks = *reinterpret_cast<const uint64_t*>(s.max_len + 2);
  uint64_t t = blockIdx.x;
  while (t < ntasks) {
    const uint64_t task = s.tasks[t];
    const uint64_t i = task >> 8;
    const hf3fs_crc_update_io io = ios[i];
    const Eff e = derive(io, max_len, type, HF3FS_UPDATE_MODE_REFERENCE);
    if (!(e.verify && s.pre_out[2 * i] != e.wval)) {  // mismatch: chunk untouched
      const bool gap = task & 0x80u;
      const uint64_t dst = io.chunk + (gap ? e.zero_from : e.off);
      const uint64_t len = gap ? e.zero_to - e.zero_from : e.len;
      const uint64_t ps = piece_bytes(len, s), h = dst & 15, j = task & 0x7fu;
      const uint64_t a = j ? j * ps - h : 0, b0 = (j + 1) * ps - h, b = b0 < len ? b0 : len;
      if (a < b) copy_range<U, NT, SHFL, ALIGN>(dst + a, gap ? 0 : io.payload + a, b - a, threadIdx.x, blockDim.x);
    }
    __syncthreads();
    if (threadIdx.x == 0) ticket = atomicAdd(queue, 1u);
    __syncthreads();
    t = gridDim.x + (uint64_t)ticket;
  }
}

template <uint32_t POLY>
__global__ __launch_bounds__(kThreads) void k_update_fused(hf3fs_crc_update_io* __restrict__ ios, uint64_t n,
                                                           uint32_t max_len, uint8_t type, int mode, UpdateScratch s,
                                                           const PolyTables* __restrict__ T,
                                                           uint32_t* __restrict__ queue) {
  __shared__ uint32_t lds[kLdsWords + kMulcWords];
  __shared__ uint32_t s_part[kWaves];
  __shared__ uint64_t s_chunk, s_pay, s_next;
  __shared__ uint32_t s_job[12];
  fill_lds(lds, T);
  const uint32_t* lj = lds + (threadIdx.x & 31);
  const uint32_t* lc = lds + kLdsWords;
  uint64_t i = blockIdx.x;
  while (i < n) {
    if (threadIdx.x == 0) {
      const Eff e = prep_one(ios, i, max_len, type, mode, s);
      const hf3fs_crc_update_io& io = ios[i];
      s_chunk = io.chunk;
      s_pay = io.payload;
      s_job[0] = e.ok;
      s_job[1] = e.ok && e.hash_payload;
      s_job[2] = e.verify;
      s_job[3] = e.wval;
      s_job[4] = e.off;
      s_job[5] = e.len;
      s_job[6] = !e.te && e.len;  // a payload to write
      // old bytes under the write (delta) or the truncated tail (delta truncate)
      s_job[7] = (uint32_t)s.pre_len[2 * i + 1];
      s_job[8] = e.te;
      s_job[9] = e.zero_from;
      s_job[10] = e.zero_to;
      s_job[11] = e.s1;
    }
    __syncthreads();
    const uint64_t chunk = s_chunk, pay = s_pay;
    const bool ok = s_job[0], hash_payload = s_job[1], verify = s_job[2], write = s_job[6], te = s_job[8];
    const uint32_t wval = s_job[3], off = s_job[4], len = s_job[5], olen = s_job[7];
    const uint32_t zfrom = s_job[9], zto = s_job[10], s1 = s_job[11];
    uint32_t crc_payload = ~0u, lin_old = 0u;  // what k_crc_ranges leaves for empty jobs
    if (hash_payload) crc_payload = wg_hash<POLY>(pay, len, ~0u, lj, lc, T, s_part);
    if (ok && !(verify && crc_payload != wval)) {  // mismatch: chunk untouched
      if (write) {
        if (olen && !te)
          lin_old = wg_write_hash_old<POLY>(chunk + off, pay, len, olen, lj, lc, T, s_part);
        else
          copy_range<4, false, true, 1024>(chunk + off, pay, len, threadIdx.x, blockDim.x);
      }
      if (zto > zfrom) copy_range<4, false, true, 1024>(chunk + zfrom, 0, zto - zfrom, threadIdx.x, blockDim.x);
    }
    if (ok && olen && te) lin_old = wg_hash<POLY>(chunk + s1, olen, 0u, lj, lc, T, s_part);
    if (threadIdx.x == 0) {
      s.pre_out[2 * i] = crc_payload;
      s.pre_out[2 * i + 1] = lin_old;
      s_next = gridDim.x + (uint64_t)atomicAdd(queue, 1u);
    }
    __syncthreads();
    i = s_next;
  }
}

// ---------------------------------------------------------------------------
// Single-read DELTA pipeline.  prep: per IO the W / P / O ranges of DeltaDesc
// and its 64 KiB pieces, listed contiguously per IO (the piece kernel's
// progress argument needs an IO's pieces to be handed out consecutively).
__global__ __launch_bounds__(256) void k_update_delta_prep(hf3fs_crc_update_io* __restrict__ ios, uint64_t n,
                                                           uint32_t max_len, uint8_t type, UpdateScratch s) {
  const uint32_t lane = threadIdx.x & 63;
  unsigned long long* count = reinterpret_cast<unsigned long long*>(s.max_len + 2);
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); i0 < n;
       i0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = i0 + lane;
    uint32_t np = 0;
    if (i < n) {
      const Eff e = prep_one(ios, i, max_len, type, HF3FS_UPDATE_MODE_DELTA, s);
      const hf3fs_crc_update_io& io = ios[i];
      DeltaDesc d{};
      d.chunk = io.chunk;
      d.payload = io.payload;
      if (e.ok) {
        if (!e.te && e.len) {
          d.p0 = e.off;
          d.p1 = e.off + e.len;
        }
        if (!e.te) {  // the write, with the zero-filled gap in front of it (ChunkReplica.cc:281-284)
          d.w0 = e.zero_to > e.zero_from ? e.zero_from : e.off;
          d.w1 = e.off + e.len;
        } else if (e.zero_to > e.zero_from) {  // extend: zeros
          d.w0 = e.zero_from;
          d.w1 = e.zero_to;
        }
        const uint32_t olen = (uint32_t)s.pre_len[2 * i + 1];  // delta old bytes / truncated tail (prep_one)
        if (olen) {
          d.o0 = (uint32_t)(s.pre_addr[2 * i + 1] - io.chunk);
          d.o1 = d.o0 + olen;
        }
        d.verify = e.verify;
        d.hashp = e.hash_payload;
        d.hash = e.hash_payload || olen;
        d.wval = e.wval;
      }
      uint32_t u0 = 0xffffffffu, u1 = 0;
      if (d.w1 > d.w0) { u0 = d.w0; u1 = d.w1; }
      if (d.o1 > d.o0) { u0 = u0 < d.o0 ? u0 : d.o0; u1 = u1 > d.o1 ? u1 : d.o1; }
      if (u1 > 0 && u0 < u1) {
        d.u0 = u0;
        d.u1 = u1;
        d.base = (d.chunk + u0) & ~uint64_t(s.dpiece - 1);
        np = (uint32_t)(((d.chunk + u1 - 1) - d.base) / s.dpiece + 1);
      }
      if (!d.hash) {  // nothing to hash: what an empty payload / old-byte job yields
        s.pre_out[2 * i] = ~0u;
        s.pre_out[2 * i + 1] = 0u;
      }
      d.npieces = np;
      s.dd[i] = d;
    }
    uint32_t incl = np;
#pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
      const uint32_t y = __shfl_up(incl, dd);
      if (lane >= (uint32_t)dd) incl += y;
    }
    const uint32_t total = __shfl(incl, 63);
    unsigned long long base = 0;
    if (lane == 63 && total) base = atomicAdd(count, (unsigned long long)total);
    base = __shfl(base, 63);
    uint64_t at = base + incl - np;
    for (uint32_t j = 0; j < np; ++j) s.tasks[at++] = (i << 16) | j;
  }
}

// Wait until every hash piece of IO i has been folded in (its old bytes are
// read, its payload verified): true when the copy may store.  After ~1 s
// without that, abort the IO (status DEVICE_ERROR; the abort is set only on an
// incomplete word, so no piece of the IO stores) instead of hanging.
__device__ __forceinline__ bool delta_wait_hashed(uint32_t* verdict, hf3fs_crc_update_io* ios, uint64_t i) {
  uint32_t* vp = verdict + i;
  const long long t0 = wall_clock64();
  for (;;) {
    const uint32_t v = __hip_atomic_load(vp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v & kVerdictAborted) return false;
    if ((v & (kVerdictP | kVerdictO)) == (kVerdictP | kVerdictO)) return !(v & kVerdictMismatch);
    if (wall_clock64() - t0 > 100000000ll) {  // 1 s of the 100 MHz wall clock
      if (atomicCAS(vp, v, v | kVerdictAborted) == v) {
        ios[i].status = HF3FS_CRC_DEVICE_ERROR;
        return false;
      }
      continue;  // the word moved on: look again
    }
    __builtin_amdgcn_s_sleep(8);
  }
}

// IO i's payload (P) or old-byte (O) accumulator is complete: lin(P) -> raw(P),
// the verdict and pre_out[2i]; lin(O) -> pre_out[2i + 1] (finalize reads both).
template <uint32_t POLY>
__device__ __attribute__((noinline)) void delta_complete(const DeltaDesc& d, uint64_t i, bool is_o, uint32_t acc,
                                                         const UpdateScratch& s, const PolyTables* __restrict__ T) {
  if (is_o) {
    s.pre_out[2 * i + 1] = acc;
    atomicOr(s.verdict + i, (uint32_t)kVerdictO);
    return;
  }
  const uint32_t plen = d.p1 - d.p0;
  uint32_t rawp = ~0u;
  if (d.hashp && plen) rawp = acc ^ gf_mul(~0u, xpow8_bytes((int64_t)plen, T, POLY), POLY);  // raw = lin ^ ~0 x^(8 len)
  s.pre_out[2 * i] = rawp;
  atomicOr(s.verdict + i, d.verify && rawp != d.wval ? (uint32_t)(kVerdictP | kVerdictMismatch) : (uint32_t)kVerdictP);
}

// A piece's published words come back while the workgroup goes on (the
// returning atomics are not waited for when issued) and are checked at its
// next task: did they complete their IO's arrival mask?
struct DeltaPub {
  uint64_t i;
  bool valid;
  uint64_t ret[2], mine[2];  // payload, old bytes
};

template <uint32_t POLY>
__device__ __forceinline__ void delta_check(const DeltaPub& pub, const UpdateScratch& s,
                                            const PolyTables* __restrict__ T) {
  if (!pub.valid) return;
  const uint32_t np = s.dd[pub.i].npieces;
  const uint32_t full = np >= 32 ? ~0u : ((1u << np) - 1u);
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const uint64_t w = pub.ret[x] ^ pub.mine[x];
    if ((uint32_t)(w >> 32) == full) delta_complete<POLY>(s.dd[pub.i], pub.i, x == 1, (uint32_t)w, s, T);
  }
}

// Ticket t of the fused DELTA kernel -> (copy?, piece).  The 2N tickets of N
// pieces run hash 0 .. L-1, then alternate copy k / hash L + k, then the last
// copies (L = min(lag, N)): piece k is copied L pieces after its hash.
__device__ __forceinline__ uint64_t delta_ticket(uint64_t t, uint64_t np, uint64_t lag, bool& copy) {
  const uint64_t L = np < lag ? np : lag;
  if (t < L) {
    copy = false;
    return t;
  }
  const uint64_t u = t - L, p2 = 2 * (np - L);
  if (u < p2) {
    copy = !(u & 1);
    return copy ? u / 2 : L + u / 2;
  }
  copy = true;
  return (np - L) + (u - p2);
}

// The fused DELTA kernel.  Each piece (the kDeltaPiece-aligned windows of an
// IO's write window, <= 512 KiB) has two tasks in one ticket order.
// HASH: all 16 waves hash the piece's payload bytes (cached loads) and old
// bytes (wg_hash: 4 KiB in flight per wave), each part shifted to its IO
// range's end, and thread 0 publishes them with ONE returning 64-bit atomic
// xor per accumulator that carries the partial CRC and the piece's arrival
// bit, so nothing orders or waits; the value is checked at the workgroup's
// next task, and the piece that completes its IO's mask computes raw(payload),
// lin(old), pre_out and the verdict.
// COPY, L = kCopyLag pieces later in the order: once every hash piece of the
// IO is folded in (its old bytes are read; a mismatching payload leaves the
// chunk untouched, ChunkReplica.cc:193-207), copy the payload into the chunk
// (copy_range, lane-shift realignment) and zero-fill the gap.  The payload was read by the hash ~L pieces (<= 64 MiB of
// payload and old bytes) earlier, so this re-read comes from the 256 MiB
// Infinity Cache rather than HBM.
// Progress: only copies wait, and every hash piece of the awaited IO precedes
// the copy in the ticket order (an IO has < L pieces), was handed out, and is
// published by a workgroup that waits for nothing before publishing (its
// prefetched ticket is later in the order than the wait's copy, and it checks
// its last publish before any wait).  No residency assumption; a wait
// exceeding ~1 s still aborts the IO (DEVICE_ERROR, nothing of it stored).
template <uint32_t POLY>
__global__ __launch_bounds__(kThreads) void k_update_delta(hf3fs_crc_update_io* __restrict__ ios, UpdateScratch s,
                                                           const PolyTables* __restrict__ T,
                                                           uint32_t* __restrict__ queue) {
  __shared__ uint32_t lds[kLdsWords + kMulcWords];
  __shared__ uint32_t s_part[kWaves];
  __shared__ uint64_t s_t;
  __shared__ uint32_t s_v;
  fill_lds(lds, T);
  const uint32_t* lj = lds + (threadIdx.x & 31);
  const uint32_t* lc = lds + kLdsWords;
  const uint64_t np = *reinterpret_cast<const uint64_t*>(s.max_len + 2);
  const uint64_t total = 2 * np;
  DeltaPub pub{};  // thread 0: the last publish, checked at the next task
  uint64_t t = blockIdx.x;
  while (t < total) {
    uint32_t tk = 0;
    if (threadIdx.x == 0) {
      tk = atomicAdd(queue, 1u);  // the next ticket, used at the end of this task
      delta_check<POLY>(pub, s, T);
      pub.valid = false;
    }
    bool copy = false;
    const uint64_t k = delta_ticket(t, np, s.dlag, copy);
    const uint64_t task = s.tasks[k];
    const uint64_t i = task >> 16;
    const uint32_t j = (uint32_t)(task & 0xffffu);
    const DeltaDesc d = s.dd[i];
    // piece window, absolute (it may start before the chunk: base is kDeltaPiece-aligned)
    const uint64_t A0 = d.base + (uint64_t)j * s.dpiece, A1 = A0 + s.dpiece;
    const uint64_t P0 = d.chunk + d.p0, P1 = d.chunk + d.p1;
    if (!copy) {
      if (d.hash) {
        // payload part [a, b) of the piece (absolute), shifted to the payload's end
        const uint64_t a = P0 > A0 ? P0 : A0, b = P1 < A1 ? P1 : A1;
        uint32_t qp = 0, qo = 0;
        if (d.hashp && a < b) qp = wg_hash<POLY>(d.payload + (a - P0), b - a, 0u, lj, lc, T, s_part);
        const uint64_t O0 = d.chunk + d.o0, O1 = d.chunk + d.o1;
        const uint64_t c = O0 > A0 ? O0 : A0, e = O1 < A1 ? O1 : A1;
        if (c < e) qo = wg_hash<POLY>(c, e - c, 0u, lj, lc, T, s_part);
        if (threadIdx.x == 0) {
          if (d.hashp && a < b) qp = gf_mul(qp, xpow8_bytes((int64_t)(P1 - b), T, POLY), POLY);
          if (c < e) qo = gf_mul(qo, xpow8_bytes((int64_t)(O1 - e), T, POLY), POLY);
          uint64_t* sy = s.dsync + i * kSyncWords;
          const uint64_t bit = uint64_t(1) << (32 + j);
          pub.i = i;
          pub.valid = true;
          pub.mine[0] = bit | qp;
          pub.mine[1] = bit | qo;
          pub.ret[0] = __hip_atomic_fetch_xor(sy, pub.mine[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          pub.ret[1] = __hip_atomic_fetch_xor(sy + kSyncO, pub.mine[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    } else if (d.w1 > d.w0 && A0 < d.chunk + d.w1 && A1 > d.chunk + d.w0) {
      // hashed IOs: the old bytes must be read (and the payload verified) before the store
      if (threadIdx.x == 0) s_v = d.hash ? delta_wait_hashed(s.verdict, ios, i) : 1u;
      __syncthreads();
      if (s_v) {
        // zeros: W minus the payload, i.e. [w0, p0) (the gap in front of a write) or all of W (extend)
        const uint64_t Z0 = d.chunk + d.w0, Z1 = d.p1 > d.p0 ? P0 : d.chunk + d.w1;
        const uint64_t g0 = Z0 > A0 ? Z0 : A0, g1 = Z1 < A1 ? Z1 : A1;
        if (g0 < g1) copy_range<4, false, true, 1024>(g0, 0, g1 - g0, threadIdx.x, blockDim.x);
        const uint64_t a = P0 > A0 ? P0 : A0, b = P1 < A1 ? P1 : A1;
        if (a < b) copy_range<4, false, true, 1024>(a, d.payload + (a - P0), b - a, threadIdx.x, blockDim.x);
      }
    }
    if (threadIdx.x == 0) s_t = gridDim.x + (uint64_t)tk;
    __syncthreads();
    t = s_t;
    __syncthreads();  // s_t / s_v are rewritten by the next task
  }
  if (threadIdx.x == 0) delta_check<POLY>(pub, s, T);
}

template <uint32_t POLY>
__global__ void k_update_finalize(hf3fs_crc_update_io* __restrict__ ios, uint64_t n, uint8_t type, int mode,
                                  UpdateScratch s, const PolyTables* __restrict__ T, uint32_t max_len) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    hf3fs_crc_update_io io = ios[i];
    if (io.status != HF3FS_CRC_OK) continue;
    const Eff e = derive(io, max_len, type, mode);
    if (e.verify && s.pre_out[2 * i] != e.wval) {  // ChunkReplica.cc:193-207
      io.status = HF3FS_CRC_CHECKSUM_MISMATCH;
      ios[i] = io;
      continue;
    }
    uint32_t val = 0;
    // engine writes without a CRC32C checksum use the hashed payload (engine.rs:300-303)
    const uint32_t wv = (e.engine && !e.verify && e.len) ? s.pre_out[2 * i] : e.wval;
    switch (e.kase) {
      case 1:
        val = e.engine ? ~0u : 0u;  // replica: size 0 -> 0 (ChunkReplica.cc:334-336); engine: crc32c("") = 0 fin
        break;
      case 2:
        val = wv;
        break;
      case 3:
        val = ck_combine<POLY>(e.cval, wv, e.len, T);
        break;
      default:
        if (e.delta) {
          const uint32_t rawO = e.s0 == 0 ? ~0u : e.cval;
          const uint32_t linO = s.pre_out[2 * i + 1];
          if (e.te) {
            if (e.s1 < e.s0)  // raw(O[:s1]) = (raw(O) ^ lin(O[s1:s0])) * x^-(8 (s0-s1))
              val = gf_mul(rawO ^ linO, xpow8<POLY>(-(int64_t)(e.s0 - e.s1), T), POLY);
            else
              val = gf_mul(rawO, xpow8<POLY>(e.s1 - e.s0, T), POLY);
          } else {
            // raw(N) = raw(O) x^(8(s1-s0)) ^ lin(O_pad[off,off+len) ^ P) x^(8(s1-off-len))
            const uint32_t linP = e.len ? s.pre_out[2 * i] ^ gf_mul(~0u, xpow8<POLY>(e.len, T), POLY) : 0u;
            const uint32_t oldlen = e.off < e.s0 ? ((e.off + e.len < e.s0 ? e.off + e.len : e.s0) - e.off) : 0u;
            const uint32_t linX = gf_mul(linO, xpow8<POLY>(e.len - oldlen, T), POLY) ^ linP;
            val = gf_mul(rawO, xpow8<POLY>(e.s1 - e.s0, T), POLY) ^
                  gf_mul(linX, xpow8<POLY>(e.s1 - e.off - e.len, T), POLY);
          }
        } else {  // prefix.combine(write, len); prefix.combine(suffix, suffix_len)
          const uint32_t suffix_start = e.off + e.len < e.s1 ? e.off + e.len : e.s1;
          val = ck_combine<POLY>(s.post_out[2 * i], wv, e.len, T);
          val = ck_combine<POLY>(val, s.post_out[2 * i + 1], e.s1 - suffix_start, T);
        }
    }
    io.out_size = e.s1;
    io.out_checksum = val;
    io.out_checksum_type = e.wtype;  // meta.checksumType = writeIO.checksum.type (:392)
    ios[i] = io;
  }
}

unsigned grid_for(uint64_t n, unsigned cap) {
  const uint64_t want = (n + 255) / 256;
  return (unsigned)(want < cap ? (want ? want : 1) : cap);
}

// ---------------------------------------------------------------------------
// AioReadJob::setResult (BatchReadJob.cc:24-63): which reads need hashing.
__device__ __forceinline__ bool read_full(const hf3fs_crc_read_io& io) {
  return io.offset == 0 && io.length == io.chunk_len;
}

__global__ void k_read_prep(hf3fs_crc_read_io* __restrict__ ios, uint64_t n, uint8_t type, uint32_t max_len,
                            uint64_t* __restrict__ addr, uint64_t* __restrict__ len, uint32_t* __restrict__ maxl) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    hf3fs_crc_read_io io = ios[i];
    const bool full = read_full(io);
    const bool reuse = io.batch_checksum_type == io.chunk_checksum_type && full;                       // :30-31
    const bool create = io.batch_checksum_type != kTypeNone && !reuse;                                   // :32-35
    const bool recalc = io.recalculate && full && io.chunk_checksum_type != kTypeNone;                   // :43-54
    bool ok = io.length <= max_len && (io.data || io.length == 0);
    if (io.batch_checksum_type != kTypeNone && io.batch_checksum_type != type) ok = false;
    if (io.chunk_checksum_type != kTypeNone && io.chunk_checksum_type != type) ok = false;
    io.status = ok ? HF3FS_CRC_OK : HF3FS_CRC_INVALID_ARG;
    io.out_checksum = 0;
    io.out_checksum_type = kTypeNone;
    ios[i] = io;
    const bool need = ok && (create || recalc);
    addr[i] = need ? io.data : 0;
    len[i] = need ? io.length : 0;
    if (need && io.length) atomicMax(maxl, io.length);
  }
}

__global__ void k_read_finalize(hf3fs_crc_read_io* __restrict__ ios, uint64_t n, const uint32_t* __restrict__ v) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    hf3fs_crc_read_io io = ios[i];
    if (io.status != HF3FS_CRC_OK) continue;
    const bool full = read_full(io);
    if (io.batch_checksum_type == kTypeNone) {
      io.out_checksum_type = kTypeNone;  // "do not return checksum"
      io.out_checksum = 0;
    } else if (io.batch_checksum_type == io.chunk_checksum_type && full) {
      io.out_checksum_type = io.chunk_checksum_type;
      io.out_checksum = io.chunk_checksum;
    } else {
      io.out_checksum_type = io.batch_checksum_type;
      io.out_checksum = v[i];
    }
    if (io.recalculate && full) {  // ChecksumInfo::create(chunk type, localbuf, len) != chunkChecksum
      const uint32_t real = io.chunk_checksum_type == kTypeNone ? 0u : v[i];
      if (real != io.chunk_checksum) io.status = HF3FS_CRC_CHECKSUM_MISMATCH;
    }
    ios[i] = io;
  }
}

}  // namespace

hipError_t launch_read_prep(hf3fs_crc_read_io* ios, uint64_t n, uint8_t type, uint32_t max_len, uint64_t* addr,
                            uint64_t* len, uint32_t* maxl, hipStream_t st) {
  hipLaunchKernelGGL(k_read_prep, dim3(grid_for(n, 4096)), dim3(256), 0, st, ios, n, type, max_len, addr, len, maxl);
  return hipGetLastError();
}

hipError_t launch_read_finalize(hf3fs_crc_read_io* ios, uint64_t n, const uint32_t* v, hipStream_t st) {
  hipLaunchKernelGGL(k_read_finalize, dim3(grid_for(n, 4096)), dim3(256), 0, st, ios, n, v);
  return hipGetLastError();
}

static uint64_t delta_tasks_per_io(uint32_t delta_len) {
  return delta_len ? 34 : 0;  // <= 32 pieces (+ alignment slack)
}

size_t update_scratch_bytes(uint64_t n, uint32_t pieces, uint32_t delta_len) {
  const uint64_t tasks = n * std::max<uint64_t>(2 * (pieces + 1), delta_tasks_per_io(delta_len));
  const uint64_t delta = delta_len ? n * (sizeof(DeltaDesc) + kSyncWords * 8 + 4) + 256 : 0;
  return n * 2 * (8 + 8 + 4 + 4) * 2 + tasks * 8 + delta + 512;
}

void update_scratch_carve(void* base, uint64_t n, uint32_t pieces, uint32_t piece_min, uint32_t delta_len,
                          UpdateScratch* s) {
  uint8_t* p = (uint8_t*)base;
  auto take = [&](size_t bytes) {
    uint8_t* r = p;
    p += (bytes + 15) & ~size_t(15);
    return r;
  };
  s->max_len = (uint32_t*)take(16);
  s->pre_addr = (uint64_t*)take(2 * n * 8);
  s->pre_len = (uint64_t*)take(2 * n * 8);
  s->pre_start = (uint32_t*)take(2 * n * 4);
  s->pre_out = (uint32_t*)take(2 * n * 4);
  s->post_addr = (uint64_t*)take(2 * n * 8);
  s->post_len = (uint64_t*)take(2 * n * 8);
  s->post_start = (uint32_t*)take(2 * n * 4);
  s->post_out = (uint32_t*)take(2 * n * 4);
  s->tasks = (uint64_t*)take(n * std::max<uint64_t>(2 * (pieces + 1), delta_tasks_per_io(delta_len)) * 8);
  s->pieces = pieces;
  s->piece_min = piece_min;
  s->dd = delta_len ? (DeltaDesc*)take(n * sizeof(DeltaDesc)) : nullptr;
  s->dsync = delta_len ? (uint64_t*)take(n * kSyncWords * 8 + 128) : nullptr;
  if (s->dsync) s->dsync = (uint64_t*)(((uintptr_t)s->dsync + 127) & ~uintptr_t(127));  // a line per IO
  s->verdict = delta_len ? (uint32_t*)take(n * 4) : nullptr;
}

hipError_t launch_update_prep(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type, int mode,
                              const UpdateScratch& s, hipStream_t st) {
  hipLaunchKernelGGL(k_update_prep, dim3(grid_for(n, 4096)), dim3(256), 0, st, ios, n, max_len, type, mode, s);
  return hipGetLastError();
}

hipError_t launch_update_delta_prep(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type,
                                    const UpdateScratch& s, hipStream_t st) {
  hipLaunchKernelGGL(k_update_delta_prep, dim3(grid_for(n, 4096)), dim3(256), 0, st, ios, n, max_len, type, s);
  return hipGetLastError();
}

hipError_t launch_update_delta(hf3fs_crc_update_io* ios, uint8_t type, const UpdateScratch& s,
                               const DeviceTables* tabs, uint32_t grid, uint32_t* queue, hipStream_t st) {
  if (type == kTypeCrc32)
    hipLaunchKernelGGL(k_update_delta<kPolyCrc32>, dim3(grid), dim3(kThreads), 0, st, ios, s, &tabs->poly[1], queue);
  else
    hipLaunchKernelGGL(k_update_delta<kPolyCrc32c>, dim3(grid), dim3(kThreads), 0, st, ios, s, &tabs->poly[0], queue);
  return hipGetLastError();
}

hipError_t launch_update_apply(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type,
                               const UpdateScratch& s, uint32_t grid, uint32_t* queue, hipStream_t st) {
  // U = 4 granules in flight per thread, cached loads/stores: U = 8 and non-temporal variants measured
  // slower on d3 (1.96 vs 1.98 / 2.06 / 2.05 ms per batch).  Misaligned sources use one
  // aligned load per granule plus a lane shift (HF3FS_CRC_APPLY_SHFL=0: two loads per granule).
  static const bool shfl = [] {
    const char* v = getenv("HF3FS_CRC_APPLY_SHFL");
    return v ? v[0] == '1' : true;  // A/B d3 DELTA: 1.79 vs 1.81 ms per batch
  }();
  static const int align = [] {
    const char* v = getenv("HF3FS_CRC_APPLY_ALIGN");  // 0, 1 (1 KiB) or 4 (4 KiB)
    return v ? (v[0] == '1' ? 1024 : v[0] == '4' ? 4096 : 0) : 1024;  // A/B d3 DELTA: 1.77 vs 1.81 ms
  }();
  if (shfl && align == 4096)
    hipLaunchKernelGGL((k_update_apply<4, false, true, 4096>), dim3(grid), dim3(256), 0, st, ios, max_len, type, s, queue);
  else if (shfl && align == 1024)
    hipLaunchKernelGGL((k_update_apply<4, false, true, 1024>), dim3(grid), dim3(256), 0, st, ios, max_len, type, s, queue);
  else if (shfl)
    hipLaunchKernelGGL((k_update_apply<4, false, true, 0>), dim3(grid), dim3(256), 0, st, ios, max_len, type, s, queue);
  else if (align)
    hipLaunchKernelGGL((k_update_apply<4, false, false, 1024>), dim3(grid), dim3(256), 0, st, ios, max_len, type, s, queue);
  else
    hipLaunchKernelGGL((k_update_apply<4, false, false, 0>), dim3(grid), dim3(256), 0, st, ios, max_len, type, s, queue);
  return hipGetLastError();
}

hipError_t launch_update_fused(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type, int mode,
                               const UpdateScratch& s, const DeviceTables* tabs, uint32_t grid, uint32_t* queue,
                               hipStream_t st) {
  if (type == kTypeCrc32)
    hipLaunchKernelGGL(k_update_fused<kPolyCrc32>, dim3(grid), dim3(kThreads), 0, st, ios, n, max_len, type, mode, s,
                       &tabs->poly[1], queue);
  else
    hipLaunchKernelGGL(k_update_fused<kPolyCrc32c>, dim3(grid), dim3(kThreads), 0, st, ios, n, max_len, type, mode, s,
                       &tabs->poly[0], queue);
  return hipGetLastError();
}

hipError_t launch_update_finalize(hf3fs_crc_update_io* ios, uint64_t n, uint8_t type, int mode,
                                  const UpdateScratch& s, const DeviceTables* tabs, uint32_t max_len,
                                  hipStream_t st) {
  if (type == kTypeCrc32)
    hipLaunchKernelGGL(k_update_finalize<kPolyCrc32>, dim3(grid_for(n, 4096)), dim3(256), 0, st, ios, n, type, mode,
                       s, &tabs->poly[1], max_len);
  else
    hipLaunchKernelGGL(k_update_finalize<kPolyCrc32c>, dim3(grid_for(n, 4096)), dim3(256), 0, st, ios, n, type, mode,
                       s, &tabs->poly[0], max_len);
  return hipGetLastError();
}

}  // namespace hf3fs_crc
