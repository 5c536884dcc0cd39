// update_kernels.hip -- batched ChunkReplica::update / updateChecksum on HBM-resident chunks.
//
// Pipeline per batch (hf3fs_crc_update_batch):
//   prep      derive each IO's effective sizes / case (ChunkReplica.cc:319-394),
//             emit "pre" hash jobs: payload (verify, :193-207) and, for the
//             delta method, the old bytes about to be overwritten / truncated;
//   ranges    hash the pre jobs (crc_kernels.hip);
//   apply     copy verified payloads into the chunks, zero-fill gaps (:281-292),
//             and finalize every IO that needs no post job;
//   ranges    hash the "post" jobs: prefix [0,off) and suffix [off+len,size)
//             of the written chunk (reference algorithm :356-389);
//   finalize  pick the case and stitch the new chunk checksum with GF(2) shifts
//             (the IOs left: those whose recompute needed the post jobs).
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

// GF(2^32) products and powers x^(8n) for finalize_one, two ways:
// GfGlobal: the bit-serial product over the HBM-resident tables (the apply's inlined finalize);
// GfLds: the carry-less product gf_mul_dw over the x^32 dword tables and the byte-digit power
// tables a workgroup copied to LDS (the finalize launch: one thread per IO is a chain of ~16
// dependent products, 3.5x fewer VALU per product; gf2.h).
template <uint32_t POLY>
struct GfGlobal {
  const PolyTables* T;
  __device__ __forceinline__ uint32_t mul(uint32_t a, uint32_t b) const { return gf_mul(a, b, POLY); }
  __device__ __forceinline__ uint32_t x8(int64_t n) const { return xpow8<POLY>(n, T); }
};
template <uint32_t POLY>
struct GfLds {
  const uint32_t* dw;  // ShortTables::dw (4 x 256)
  const uint32_t* pw;  // PolyTables::pow8b (kPowDigits x 256)
  const uint32_t* iw;  // PolyTables::inv8b
  const PolyTables* T;  // x^(+-2^k) for byte counts >= 2^40
  __device__ __forceinline__ uint32_t mul(uint32_t a, uint32_t b) const { return gf_mul_dw(a, b, dw); }
  __device__ __forceinline__ uint32_t x8(int64_t nbytes) const {  // xpow8_bytes with these tables
    uint64_t m = nbytes < 0 ? (uint64_t)(-nbytes) : (uint64_t)nbytes;
    const bool neg = nbytes < 0;
    const uint32_t* tab = neg ? iw : pw;
    uint32_t x = kOne;
    bool first = true;
    for (int j = 0; j < kPowDigits && m; ++j, m >>= 8) {
      const uint32_t d = (uint32_t)(m & 0xffu);
      if (!d) continue;
      x = first ? tab[256 * j + d] : gf_mul_dw(x, tab[256 * j + d], dw);
      first = false;
    }
    for (int k = 8 * kPowDigits + 3; m; ++k, m >>= 1)
      if (m & 1) x = gf_mul_dw(x, xpow2k(neg ? T->xinv : T->xpow, k, POLY), dw);
    return x;
  }
};

// ChecksumInfo::combine on raw values of one type (Common.h:179-198).
template <uint32_t POLY>
__device__ __forceinline__ uint32_t ck_combine(uint32_t a, uint32_t b, uint32_t len, const PolyTables* T) {
  return len == 0 ? a : gf_mul(~a, xpow8<POLY>(len, T), POLY) ^ b;
}
template <class M>
__device__ __forceinline__ uint32_t ck_combine_m(uint32_t a, uint32_t b, uint32_t len, const M& g) {
  return len == 0 ? a : g.mul(~a, g.x8(len)) ^ b;
}

// The checksum path the reference takes for the IO (hf3fs_crc_update_io.checksum_case):
// the case ChunkReplica::updateChecksum picks (ChunkReplica.cc:334-389; DELTA computes
// case 4 another way but it is the case the reference counts), or for chunk-engine IOs
// the path Chunk::copy_on_write / safe_write takes (chunk.rs:89-281, capacity = max_len).
__device__ __forceinline__ uint8_t ck_case(const hf3fs_crc_update_io& io, const Eff& e) {
  if (!e.engine) return e.kase;
  const uint32_t s0 = io.chunk_size;
  if (e.te) {  // the bridge's truncate / extend: safe_write(no data, offset = target, truncate)
    const uint32_t target = io.length;
    if (io.update_type == HF3FS_UPDATE_TRUNCATE && target < s0) return HF3FS_CKCASE_RECOMPUTE;  // :184-198
    return target > s0 ? HF3FS_CKCASE_COMBINE : HF3FS_CKCASE_NONE;  // zero padding :203-218, :238-277
  }
  if (io.length > 0 && io.offset < s0)  // copy_on_write (engine.rs:383-385): reuse without a read (:110,150-157)
    return io.offset == 0 && io.length >= s0 ? HF3FS_CKCASE_REUSE : HF3FS_CKCASE_RECOMPUTE;
  return (uint64_t)io.offset + io.length > s0 ? HF3FS_CKCASE_COMBINE : HF3FS_CKCASE_NONE;  // safe_write appends
}

// Lengths of IO i's two pre jobs: the payload (verify) and, for the delta method, the old
// bytes under the write or the truncated tail.  Only the IO's input fields and Eff.
__device__ __forceinline__ void pre_lens(const Eff& e, uint64_t& l0, uint64_t& l1) {
  l0 = l1 = 0;
  if (!e.ok) return;
  if (e.hash_payload) l0 = e.len;
  if (e.kase == 4 && e.delta) {
    if (!e.te && e.off < e.s0)
      l1 = (e.off + e.len < e.s0 ? e.off + e.len : e.s0) - e.off;
    else if (e.te && e.s1 < e.s0)
      l1 = e.s0 - e.s1;
  }
}

// k_update_prep for one IO: status and output defaults, the "pre" jobs
// (payload; old bytes for the delta method) and the "post" jobs (prefix +
// suffix after the write, reference algorithm).  Returns the derived IO and the
// longest pre / post job in pre_max / post_max (the caller raises ctl's maxima).
__device__ __forceinline__ Eff prep_one(hf3fs_crc_update_io* __restrict__ ios, uint64_t i, uint32_t max_len,
                                        uint8_t type, int mode, const UpdateScratch& s, uint32_t& pre_max,
                                        uint32_t& post_max) {
  const hf3fs_crc_update_io io = ios[i];
  const Eff e = derive(io, max_len, type, mode);
  // only the output fields are stored: the prep launch's runs workgroup reads the input
  // fields of the same records meanwhile (bal_runs_block), so they are never rewritten
  ios[i].status = e.ok ? HF3FS_CRC_OK : HF3FS_CRC_INVALID_ARG;
  ios[i].out_size = io.chunk_size;
  ios[i].out_checksum = io.chunk_checksum;
  ios[i].out_checksum_type = io.chunk_checksum_type;
  ios[i].checksum_case = 0;
  uint64_t a0 = 0, l0 = 0, a1 = 0, l1 = 0, pa = 0, pl = 0, sa = 0, sl = 0;
  pre_lens(e, l0, l1);
  if (l0) a0 = io.payload;
  if (l1) a1 = io.chunk + (e.te ? e.s1 : e.off);  // old bytes under the write, or the truncated tail
  if (e.ok) {
    if (e.kase == 4 && !e.delta) {  // reference: prefix + suffix after the write
      const uint32_t suffix_start = e.off + e.len < e.s1 ? e.off + e.len : e.s1;
      pa = io.chunk;
      pl = e.off;
      sa = io.chunk + suffix_start;
      sl = e.s1 - suffix_start;
    }
  }
  s.pre_addr[2 * i] = a0;
  s.pre_len[2 * i] = l0;
  s.pre_start[2 * i] = ~0u ^ (s.fault_io == i + 1 ? 1u : 0u);
  s.pre_addr[2 * i + 1] = a1;
  s.pre_len[2 * i + 1] = l1;
  s.pre_start[2 * i + 1] = 0u;
  s.post_addr[2 * i] = pa;
  s.post_len[2 * i] = pl;
  s.post_start[2 * i] = ~0u;
  s.post_addr[2 * i + 1] = sa;
  s.post_len[2 * i + 1] = sl;
  s.post_start[2 * i + 1] = ~0u;
  s.pre_out[2 * i] = 0u;  // the range hashes XOR segment values into these
  s.pre_out[2 * i + 1] = 0u;
  s.post_out[2 * i] = 0u;
  s.post_out[2 * i + 1] = 0u;
  pre_max = (uint32_t)(l0 > l1 ? l0 : l1);
  post_max = (uint32_t)(pl > sl ? pl : sl);
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

// Piece j of a range of len bytes at dst (j < piece_count).
__device__ __forceinline__ void piece_bounds(uint64_t dst, uint64_t len, uint32_t j, const UpdateScratch& s,
                                             uint64_t& a, uint64_t& b) {
  const uint64_t ps = piece_bytes(len, s), h = dst & 15;
  a = j ? (uint64_t)j * ps - h : 0;
  const uint64_t b0 = (uint64_t)(j + 1) * ps - h;
  b = b0 < len ? b0 : len;
}

// One-shot apply pieces of a range: cut at every 2^shift-aligned destination address.
__device__ __forceinline__ uint32_t pieces_of(uint64_t dst, uint64_t len, uint32_t shift) {
  if (!len) return 0;
  const uint64_t m = (uint64_t(1) << shift) - 1;
  return (uint32_t)(((dst & m) + len + m) >> shift);
}

// Byte runs of the 2n pre jobs over nw waves, by ONE extra workgroup of the prep launch
// (k_bal_assign's boff form, crc_kernels.hip): wave k starts at byte X_k = ceil(k T / nw)
// of the jobs laid end to end (T their total), i.e. at byte boff[k] of job bal[k];
// bal[0] = 0, bal[nw] = 2n, and a boundary never points at an empty job (byte_run hashes
// each empty job's start term in the run that contains it).  The job lengths come from the
// IO records' input fields (pre_lens), which prep does not change: this workgroup needs
// nothing the others write and runs beside them.  Thread t owns the kRunIos consecutive IOs
// from t * kRunIos (their 2 kRunIos jobs stay in registers, all records loaded at once); a
// wave scan and one LDS step over the wave totals give every thread its byte prefix.
constexpr uint32_t kRunIos = kPrepRunJobs / 2 / kPrepThreads;
static_assert(kRunIos * 2 * kPrepThreads == kPrepRunJobs, "runs workgroup geometry");
__device__ void bal_runs_block(const hf3fs_crc_update_io* __restrict__ ios, uint32_t n, uint32_t max_len,
                               uint8_t type, int mode, uint32_t nw, uint32_t* __restrict__ bal,
                               uint64_t* __restrict__ boff) {
  __shared__ uint64_t s_wave[kPrepThreads / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nj = 2 * n;
  const uint32_t i0 = tid * kRunIos;
  hf3fs_crc_update_io io[kRunIos];
#pragma unroll
  for (uint32_t u = 0; u < kRunIos; ++u)
    if (i0 + u < n) io[u] = ios[i0 + u];
  uint64_t l[2 * kRunIos];
  uint64_t mine = 0;
#pragma unroll
  for (uint32_t u = 0; u < kRunIos; ++u) {
    l[2 * u] = l[2 * u + 1] = 0;
    if (i0 + u < n) pre_lens(derive(io[u], max_len, type, mode), l[2 * u], l[2 * u + 1]);
    mine += l[2 * u] + l[2 * u + 1];
  }
  uint64_t incl = mine;  // inclusive scan over the wave
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(incl, d);
    if (lane >= (uint32_t)d) incl += y;
  }
  if (lane == 63) s_wave[wv] = incl;
  __syncthreads();
  uint64_t before = 0, total = 0;
#pragma unroll
  for (uint32_t w = 0; w < kPrepThreads / 64; ++w) {
    const uint64_t x = s_wave[w];
    before += w < wv ? x : 0;
    total += x;
  }
  uint64_t P = before + incl - mine;  // bytes before job 2 i0
  if (tid == 0) {
    bal[0] = 0;
    bal[nw] = nj;
    boff[0] = boff[nw] = 0;
  }
  if (total == 0) {  // every job empty: split by count
    for (uint32_t k = tid + 1; k < nw; k += kPrepThreads) {
      bal[k] = (uint32_t)((uint64_t)k * nj / nw);
      boff[k] = 0;
    }
    return;
  }
  // X_k == T (fewer bytes than waves): an empty run at the end, for every k > (T - 1) nw / T
  const uint64_t kend = (total - 1) * nw / total + 1;
  for (uint64_t k = tid + 1; k < nw; k += kPrepThreads)
    if (k >= kend) {
      bal[k] = nj;
      boff[k] = 0;
    }
  if (!mine) return;  // no X_k inside this thread's jobs
  // X_k stepped without a division per boundary: T = q nw + rem, X_k = k q + ceil(k rem / nw)
  const uint64_t q = total / nw, rem = total % nw;
  uint64_t k = P ? (P - 1) * nw / total + 1 : 1;  // first k >= 1 with X_k >= P
  uint64_t acc = (k * rem) % nw;
  uint64_t X = k * q + (k * rem) / nw + (acc ? 1 : 0);
#pragma unroll
  for (uint32_t j = 0; j < 2 * kRunIos; ++j) {
    const uint64_t li = l[j];
    while (k < nw && X < P + li) {  // X_k in [P_j, P_j + len_j): wave k starts inside job 2 i0 + j
      bal[k] = 2 * i0 + j;
      boff[k] = X - P;
      ++k;
      const uint64_t c0 = acc ? 1 : 0;
      acc += rem;
      uint64_t c = 0;
      if (acc >= nw) {
        acc -= nw;
        c = 1;
      }
      X += q + c - c0 + (acc ? 1 : 0);
    }
    P += li;
  }
}

// prep for every IO (one thread each) and the compacted apply task list:
// each wave scans its lanes' piece counts and reserves their slots with one
// atomic.  The loop bound is wave-uniform (blockDim is a multiple of 64).  With
// place_runs one extra workgroup places the pre hash's byte runs meanwhile
// (bal_runs_block): no balance launches between prep and the hash.
__global__ __launch_bounds__(kPrepThreads) void k_update_prep(hf3fs_crc_update_io* __restrict__ ios, uint64_t n,
                                                     uint32_t max_len, uint8_t type, int mode, UpdateScratch s,
                                                     int place_runs) {
  const uint32_t lane = threadIdx.x & 63;
  unsigned long long* count = reinterpret_cast<unsigned long long*>(s.ctl + kCtlTasks);
  unsigned long long* pieces = reinterpret_cast<unsigned long long*>(s.ctl + kCtlPieces);
  // the IOs go to the first kPrepIoThreads threads of each workgroup (4 waves): a launch of
  // n / 256 workgroups spreads the per-IO latency chains over 4x the CUs that 1024 IOs per
  // workgroup used (the 1024-thread size is the runs workgroup's)
  for (uint64_t i0 = (uint64_t)blockIdx.x * kPrepIoThreads + (threadIdx.x & ~63u);
       threadIdx.x < kPrepIoThreads && i0 < n; i0 += (uint64_t)gridDim.x * kPrepIoThreads) {
    const uint64_t i = i0 + lane;
    uint32_t np = 0, ng = 0;
    uint64_t pdst = 0, plen = 0, psrc = 0, gdst = 0, glen = 0;
    uint32_t wval = 0, verify = 0, pre_max = 0, post_max = 0;
    if (i < n) {
      const Eff e = prep_one(ios, i, max_len, type, mode, s, pre_max, post_max);
      if (e.ok) {
        const uint64_t chunk = ios[i].chunk;
        if (!e.te) {
          pdst = chunk + e.off;
          plen = e.len;
          psrc = ios[i].payload;
          np = piece_count(pdst, plen, s);
        }
        if (e.zero_to > e.zero_from) {
          gdst = chunk + e.zero_from;
          glen = e.zero_to - e.zero_from;
          ng = piece_count(gdst, glen, s);
        }
        wval = e.wval;
        verify = e.verify;
      }
    }
    // one-shot pieces of the payload and the gap (the one-shot apply's table; in ticket mode
    // only counted, for the next call's grid)
    const uint32_t pp = pieces_of(pdst, plen, s.piece_shift), pg = pieces_of(gdst, glen, s.piece_shift);
    const uint32_t k = s.one_shot ? pp + pg : np + ng;
    uint32_t incl = k, pinc = pp + pg;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d);
      if (lane >= (uint32_t)d) incl += y;
      // the wave's job maxima: one atomic per wave, not one per IO on the same word
      pre_max = max(pre_max, (uint32_t)__shfl_xor(pre_max, d));
      post_max = max(post_max, (uint32_t)__shfl_xor(post_max, d));
      pinc += __shfl_xor(pinc, d);
    }
    if (lane == 0 && pre_max) atomicMax(&s.ctl[kCtlPreMax], pre_max);
    if (lane == 0 && post_max) atomicMax(&s.ctl[kCtlPostMax], post_max);
    const uint32_t total = __shfl(incl, 63);
    unsigned long long base = 0;
    if (lane == 63 && total) base = atomicAdd(s.one_shot ? pieces : count, (unsigned long long)total);
    if (lane == 0 && pinc && !s.one_shot) atomicAdd(pieces, (unsigned long long)pinc);
    base = __shfl(base, 63);
    uint64_t at = base + incl - k;
    if (s.one_shot) {
      if (i < n) {  // range records at fixed slots, their pieces at `at`
        s.tasks[2 * i] = ApplyTask{pdst, psrc, (uint32_t)plen, (uint32_t)i, wval, (uint32_t)at | (verify << 31)};
        s.tasks[2 * i + 1] = ApplyTask{gdst, 0, (uint32_t)glen, (uint32_t)i, wval, (uint32_t)(at + pp) | (verify << 31)};
      }
      // the piece table, one IO at a time by the whole wave (coalesced rows; a lane writing
      // its own IO's entries hit 64 lines per store and doubled the prep launch)
      // (readlane, not __shfl: an LDS round trip per step made this loop latency-bound)
      for (uint32_t l = 0; l < 64; ++l) {  // wave-uniform
        const uint32_t cnt = __builtin_amdgcn_readlane(pp + pg, l), ppl = __builtin_amdgcn_readlane(pp, l);
        if (!cnt) continue;
        const uint64_t atl = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)at, l) |
                             (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(at >> 32), l) << 32;
        const uint32_t r = (uint32_t)(2 * (i0 + l));
        for (uint32_t j = lane; j < cnt; j += 64) s.ptab[atl + j] = r + (j >= ppl ? 1u : 0u);
      }
      continue;
    }
    for (uint32_t j = 0; j < np; ++j) {
      uint64_t a, b;
      piece_bounds(pdst, plen, j, s, a, b);
      s.tasks[at++] = ApplyTask{pdst + a, psrc + a, (uint32_t)(b - a), (uint32_t)i, wval, verify};
    }
    for (uint32_t j = 0; j < ng; ++j) {
      uint64_t a, b;
      piece_bounds(gdst, glen, j, s, a, b);
      s.tasks[at++] = ApplyTask{gdst + a, 0, (uint32_t)(b - a), (uint32_t)i, wval, verify};
    }
  }
  // the launch's extra workgroup (place_runs): the pre hash's byte runs
  if (place_runs && blockIdx.x == gridDim.x - 1)
    bal_runs_block(ios, (uint32_t)n, max_len, type, mode, s.run_waves, s.run_bal, s.run_boff);
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
template <int U, bool NT, bool NTS = NT>
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
      st16<NTS>(gdst + (gw + lane + k * stride) * 16, funnel16(a[k], lane == 63 ? b[k] : nb, sh));
    }
  }
  return gw + lane;
}

template <int U = 4, bool NT = false, bool SHFL = false, int ALIGN = 0, bool NTS = NT>
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
      st16<NTS>(gd, src ? ld16_unaligned<NT>(src + (gd - d0)) : u32x4{0, 0, 0, 0});
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
    g = copy_rows_shfl<U, NT, NTS>(gfirst_rows, s0 & ~uint64_t(15), (uint32_t)(s0 & 15), ng, g, stride);
  }
  for (; g + (U - 1) * stride < ng; g += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
      v[k] = src ? ld16_unaligned<NT>(src + soff + (g + k * stride) * 16) : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < U; ++k) st16<NTS>(gfirst_rows + (g + k * stride) * 16, v[k]);
  }
  for (; g < ng; g += stride)
    st16<NTS>(gfirst_rows + g * 16, src ? ld16_unaligned<NT>(src + soff + g * 16) : u32x4{0, 0, 0, 0});
}

// The same copy with the source read by unaligned dwordx4 loads (the hardware
// splits a load that crosses a line): one load per destination granule, no lane
// shuffle.  Rows start at a 1 KiB destination boundary as in copy_range; the
// per-wave step count is wave-uniform (a counted loop, no vmcnt(0) at a join).
// In scripts/probe_copy.hip this body moved exactly the algorithmic bytes
// (WRITE_SIZE 1.000x, FETCH_SIZE 1.02-1.03x) where copy_range's lane-shuffle
// rows wrote 1.10x and read 1.11x (profiles/r04_copy_pmc.json).
typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) const u32x4u g_cu32x4u;
template <bool NT>
__device__ __forceinline__ u32x4 ldu16(uint64_t a) {
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<g_cu32x4u*>(a));
  return *reinterpret_cast<g_cu32x4u*>(a);
}

template <int U, bool NTL, bool NTS>
__device__ void copy_range_hw(uint64_t dst, uint64_t src, uint64_t len, uint32_t tid, uint32_t nthreads) {
  const uint64_t d0 = dst, d1 = dst + len;
  const uint64_t gfirst = (d0 + 15) & ~uint64_t(15);
  const uint64_t glast = d1 & ~uint64_t(15);
  {  // partial head and tail granules: at most 30 bytes, one per thread
    const uint64_t hend = gfirst < d1 ? gfirst : d1;
    const uint64_t tstart = glast >= gfirst ? glast : d1;
    const uint64_t nh = hend - d0, nt = d1 - tstart;
    if (tid < nh + nt) {
      const uint64_t b = tid < nh ? d0 + tid : tstart + (tid - nh);
      *reinterpret_cast<uint8_t*>(b) = src ? *reinterpret_cast<const uint8_t*>(src + (b - d0)) : 0;
    }
  }
  if (glast <= gfirst) return;
  const uint64_t ga0 = (gfirst + 1023) & ~uint64_t(1023);
  const uint64_t ga = ga0 < glast ? ga0 : glast;
  if (tid < (ga - gfirst) / 16) {  // granules up to the first 1 KiB boundary, one per thread
    const uint64_t gd = gfirst + 16 * (uint64_t)tid;
    st16<NTS>(gd, src ? ldu16<NTL>(src + (gd - d0)) : u32x4{0, 0, 0, 0});
  }
  if (glast <= ga) return;
  const uint64_t ng = (glast - ga) / 16;
  const uint64_t stride = nthreads;
  const uint64_t wlast = tid | 63;                 // this wave's last thread
  const uint64_t span = wlast + (U - 1) * stride;  // its highest granule of a step
  const uint64_t steps = ng > span ? (ng - 1 - span) / (U * stride) + 1 : 0;
  const uint32_t nsteps = __builtin_amdgcn_readfirstlane((uint32_t)steps);
  uint64_t g = tid;
  if (src) {
    const uint64_t s0 = src + (ga - d0);
    for (uint32_t i = 0; i < nsteps; ++i, g += U * stride) {
      u32x4 v[U];
#pragma unroll
      for (int k = 0; k < U; ++k) v[k] = ldu16<NTL>(s0 + (g + k * stride) * 16);
#pragma unroll
      for (int k = 0; k < U; ++k) st16<NTS>(ga + (g + k * stride) * 16, v[k]);
    }
    for (; g < ng; g += stride) st16<NTS>(ga + g * 16, ldu16<NTL>(s0 + g * 16));
  } else {
    for (; g < ng; g += stride) st16<NTS>(ga + g * 16, u32x4{0, 0, 0, 0});
  }
}

// The new checksum of IO i (and its payload verdict).  which: 0 every IO,
// 1 every verdict and the checksum of IOs that need no post job, 2 only IOs whose
// recompute used the post jobs (REFERENCE prefix + suffix, ChunkReplica.cc:356-389).
// Writes only the output fields: the apply kernel runs this beside copies that never
// read them.
template <class M>
__device__ __forceinline__ void finalize_one(hf3fs_crc_update_io* __restrict__ ios, uint64_t i, uint8_t type,
                                             int mode, const UpdateScratch& s, const M& g, uint32_t max_len,
                                             int which) {
  const hf3fs_crc_update_io io = ios[i];
  if (io.status != HF3FS_CRC_OK) return;
  const Eff e = derive(io, max_len, type, mode);
  const bool post = e.kase == 4 && !e.delta;
  if (which == 2 && !post) return;
  if (e.verify && s.pre_out[2 * i] != e.wval) {  // ChunkReplica.cc:193-207 (the verdict needs no post job)
    ios[i].status = HF3FS_CRC_CHECKSUM_MISMATCH;
    return;
  }
  if (which == 1 && post) return;
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
      val = ck_combine_m(e.cval, wv, e.len, g);
      break;
    default:
      if (e.delta) {
        const uint32_t rawO = e.s0 == 0 ? ~0u : e.cval;
        const uint32_t linO = s.pre_out[2 * i + 1];
        if (e.te) {
          if (e.s1 < e.s0)  // raw(O[:s1]) = (raw(O) ^ lin(O[s1:s0])) * x^-(8 (s0-s1))
            val = g.mul(rawO ^ linO, g.x8(-(int64_t)(e.s0 - e.s1)));
          else
            val = g.mul(rawO, g.x8(e.s1 - e.s0));
        } else {
          // raw(N) = raw(O) x^(8(s1-s0)) ^ lin(O_pad[off,off+len) ^ P) x^(8(s1-off-len))
          const uint32_t linP = e.len ? s.pre_out[2 * i] ^ g.mul(~0u, g.x8(e.len)) : 0u;
          const uint32_t oldlen = e.off < e.s0 ? ((e.off + e.len < e.s0 ? e.off + e.len : e.s0) - e.off) : 0u;
          const uint32_t linX = g.mul(linO, g.x8(e.len - oldlen)) ^ linP;
          val = g.mul(rawO, g.x8(e.s1 - e.s0)) ^ g.mul(linX, g.x8(e.s1 - e.off - e.len));
        }
      } else {  // prefix.combine(write, len); prefix.combine(suffix, suffix_len)
        const uint32_t suffix_start = e.off + e.len < e.s1 ? e.off + e.len : e.s1;
        val = ck_combine_m(s.post_out[2 * i], wv, e.len, g);
        val = ck_combine_m(val, s.post_out[2 * i + 1], e.s1 - suffix_start, g);
      }
  }
  ios[i].out_size = e.s1;
  ios[i].out_checksum = val;
  ios[i].out_checksum_type = e.wtype;  // meta.checksumType = writeIO.checksum.type (:392)
  ios[i].checksum_case = ck_case(io, e);
}

// ---------------------------------------------------------------------------
// Self-check of payload verify mismatches.  An independent re-hash:
// each lane hashes its contiguous slice of the payload serially (dwords through the
// x^32 slicing tables, edge bytes through the x^8 byte table; no code shared with
// the pipeline's 256-stream hash), the slices are shifted to the payload end and
// xor-ed across the wave.
__device__ uint32_t lin_serial(uint64_t a, uint64_t b, const ShortTables* __restrict__ S) {
  uint32_t c = 0;
  for (; a < b && (a & 3); ++a) c = (c >> 8) ^ S->b8[(c ^ *reinterpret_cast<const uint8_t*>(a)) & 0xffu];
  for (; a + 4 <= b; a += 4) {
    c ^= *reinterpret_cast<const uint32_t*>(a);
    c = S->dw[0][c & 0xffu] ^ S->dw[1][(c >> 8) & 0xffu] ^ S->dw[2][(c >> 16) & 0xffu] ^ S->dw[3][c >> 24];
  }
  for (; a < b; ++a) c = (c >> 8) ^ S->b8[(c ^ *reinterpret_cast<const uint8_t*>(a)) & 0xffu];
  return c;
}

// Bytes of pre job j (len L) the byte runs cover (k_crc_ranges byte_run: wave w hashes
// from offset boff[w] of job bal[w] to offset boff[w + 1] of job bal[w + 1]), summed by the wave.
__device__ uint64_t runs_cover(const UpdateScratch& s, uint64_t j, uint64_t L, uint32_t lane) {
  uint64_t covered = 0;
  for (uint32_t w = lane; w < s.run_waves; w += 64) {
    const uint64_t b0 = s.run_bal[w], b1 = s.run_bal[w + 1];
    if (j < b0 || j > b1) continue;
    const uint64_t so = j == b0 ? s.run_boff[w] : 0, eo = j == b1 ? s.run_boff[w + 1] : L;
    if (j == b1 && eo == 0) continue;
    if (eo > so) covered += eo - so;
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) covered += __shfl_xor(covered, d, 64);
  return covered;
}

// IO i was finalized with HF3FS_CRC_CHECKSUM_MISMATCH; the whole wave re-checks it.
template <uint32_t POLY>
__device__ void audit_one(hf3fs_crc_update_io* __restrict__ ios, uint64_t i, uint8_t type, int mode,
                          const UpdateScratch& s, const PolyTables* __restrict__ T,
                          const ShortTables* __restrict__ S, uint32_t max_len, uint32_t lane) {
  const hf3fs_crc_update_io io = ios[i];
  const Eff e = derive(io, max_len, type, mode);
  if (!e.verify) return;  // (a mismatch status comes only from the verify)
  const uint64_t L = e.len, p = io.payload;
  const uint64_t slice = ((L + 63) / 64 + 3) & ~uint64_t(3);
  const uint64_t a = lane * slice < L ? lane * slice : L, b = a + slice < L ? a + slice : L;
  uint32_t v = lin_serial(p + a, p + b, S);
  if (v) v = gf_mul(v, xpow8<POLY>((int64_t)(L - b), T), POLY);
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v ^= __shfl_xor(v, d, 64);
  const uint32_t rehash = gf_mul(~0u, xpow8<POLY>((int64_t)L, T), POLY) ^ v;  // start ~0 (ChecksumInfo::create)
  if (rehash != e.wval) return;  // the client's checksum is wrong: a real mismatch
  const uint32_t got = s.pre_out[2 * i];
  uint32_t kind = HF3FS_ANOMALY_PAYLOAD_HASH;
  if (s.pre_addr[2 * i] != p || s.pre_len[2 * i] != L) kind |= HF3FS_ANOMALY_PRE_JOB;
  if (s.ctl[kCtlPreMax] < L) kind |= HF3FS_ANOMALY_PRE_MAX;  // prep's atomicMax (both pipelines)
  if (got == ~0u) kind |= HF3FS_ANOMALY_START_ONLY;
  if (s.runs_used && runs_cover(s, 2 * i, L, lane) != L) kind |= HF3FS_ANOMALY_RUN_COVER;
  if (lane == 0) {
    ios[i].status = HF3FS_CRC_DEVICE_ERROR;
    hf3fs_crc_anomaly* d = s.diag;
    atomicOr(&d->kinds, kind);
    if (atomicAdd(&d->count, 1u) == 0) {
      d->kind = kind;
      d->pipeline = (s.runs_used ? 0u : 1u) | (uint32_t)mode << 8;
      d->io = i;
      d->pipeline_hash = got;
      d->rehash = rehash;
      d->client_checksum = e.wval;
      d->pre_max = s.ctl[kCtlPreMax];
      d->pre_addr = s.pre_addr[2 * i];
      d->pre_len = s.pre_len[2 * i];
      d->payload = p;
      d->length = L;
    }
  }
}

// The call's piece count and IO count for the next call's one-shot grid (pinned host word;
// a system-scope vector store).
__device__ __forceinline__ void store_hint(uint64_t* hint, uint64_t np, uint64_t n) {
  const uint64_t v = (np < 0xffffffffull ? np : 0xffffffffull) << 32 | (n < 0xffffffffull ? n : 0xffffffffull);
  __hip_atomic_store(hint, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One-shot apply: workgroup b copies piece b -- the bytes of one range record between two
// consecutive 2^PSHIFT-aligned destination addresses -- and exits, so the hardware's in-order
// dispatch keeps the chip's writes inside a narrow moving window of the piece list.  A
// persistent grid of ticketed >= 64 KiB tasks moved the same bytes at 4.6-5.1 TB/s read +
// write, one workgroup per 8 KiB piece at 6.0-6.2 (scripts/probe_copy_ceiling.hip,
// profiles/r06_copy_ceiling*.log; a flat one-granule-per-thread copy reaches 6.2-6.6 there
// and every persistent copy shape 4.3-5.6).
// A workgroup's latency before its first data load decides the rate, so: the table, the
// records, the verdicts and the count are __restrict__ const kernel arguments (scalar loads;
// read through the by-value UpdateScratch they were vector loads, serialised behind each
// other: the kernel ran 20 % slower than the probe's, scripts/probe_apply_inlib.hip); the
// count and the piece's entry are loaded side by side; the payload's first granule and edge
// byte are loaded before the verdict word is looked at.  A failed verify stores nothing.
// More pieces than workgroups (the grid is the previous call's count): each workgroup also
// takes pieces b + grid, b + 2 grid, ...
template <int PSHIFT, bool NTL, bool NTS>
__device__ __forceinline__ void one_shot_piece(uint64_t b, uint32_t r, const ApplyTask* __restrict__ tasks,
                                               const uint32_t* __restrict__ pre_out) {
  constexpr uint64_t P = uint64_t(1) << PSHIFT;
  constexpr int G = 1 << (PSHIFT - 12);  // granules per thread (256 threads x 16 B)
  const uint32_t tid = threadIdx.x;
  const ApplyTask R = tasks[r];
  const uint32_t first = R.verify & 0x7fffffffu;
  const uint64_t cut = (R.dst & ~(P - 1)) + ((b - first) << PSHIFT);
  const uint64_t a = cut > R.dst ? cut : R.dst, e = cut + P < R.dst + R.len ? cut + P : R.dst + R.len;
  const int64_t so = (int64_t)(R.src - R.dst);  // source offset (R.src == 0: zero fill)
  const uint64_t ga = (a + 15) & ~uint64_t(15), ge = e & ~uint64_t(15);
  // edge bytes (at most 30, only in a range's first / last piece), one per thread
  uint64_t bb = 0;
  bool byte = false;
  if (ga >= ge) {
    byte = tid < e - a;
    bb = a + tid;
  } else {
    const uint64_t nh = ga - a, nt = e - ge;
    byte = tid < nh + nt;
    bb = tid < nh ? a + tid : ge + (tid - nh);
  }
  typedef __attribute__((address_space(1))) uint8_t g_u8;  // global, not flat: vmcnt only
  const uint8_t x = byte && R.src ? *reinterpret_cast<const g_u8*>(bb + so) : 0;
  const uint64_t ng = ge > ga ? (ge - ga) >> 4 : 0;
  // the first granule is loaded beside the verdict; each later one after the previous store
  // (load -> store per granule measured faster than all loads first: a wave keeps less in
  // flight, profiles/r06_copy_ceiling*.log one-shot u1 vs u2 / u4)
  u32x4 v = tid < ng && R.src ? ldu16<NTL>(ga + tid * 16 + so) : u32x4{0, 0, 0, 0};
  const uint32_t got = (R.verify >> 31) ? pre_out[2 * (uint64_t)R.io] : R.wval;
  if (got != R.wval) return;  // ChunkReplica.cc:193-207: mismatch, chunk untouched (block-uniform)
  if (byte) *reinterpret_cast<g_u8*>(bb) = x;
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const uint64_t g = tid + k * 256;
    if (k) v = g < ng && R.src ? ldu16<NTL>(ga + g * 16 + so) : u32x4{0, 0, 0, 0};
    if (g < ng) st16<NTS>(ga + g * 16, v);
  }
}

template <int PSHIFT, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_update_apply_one_shot(const ApplyTask* __restrict__ tasks,
                                                               const uint32_t* __restrict__ ptab,
                                                               const uint32_t* __restrict__ pre_out,
                                                               const uint64_t* __restrict__ count, uint64_t n,
                                                               uint64_t ptab_cap, uint64_t* hint) {
  static_assert(PSHIFT >= 12, "a piece is at least one granule per thread");
  // (no finalize here: its GF(2) code took the kernel to 91 VGPRs, 5 waves per SIMD, and a
  // one-shot copy needs every wave slot -- the finalize launch finalizes every IO instead)
  const uint64_t b = blockIdx.x;
  const uint64_t npieces = *count;
  const uint32_t r = b < ptab_cap ? ptab[b] : 0u;  // (entries past the count: never used)
  if (hint && b == 0 && threadIdx.x == 0) store_hint(hint, npieces, n);
  if (b >= npieces) return;
  one_shot_piece<PSHIFT, NTL, NTS>(b, r < 2 * n ? r : 0u, tasks, pre_out);
  for (uint64_t c = b + gridDim.x; c < npieces; c += gridDim.x)  // a grid short of the count
    one_shot_piece<PSHIFT, NTL, NTS>(c, ptab[c], tasks, pre_out);
}

// One task = one piece of an IO's payload copy or gap zero-fill (the list
// prep compacted).  Tasks are handed out by a ticket counter (dynamic
// balance) to 256-thread workgroups, eight per CU, so each CU keeps 32 waves'
// worth of loads in flight.  (A/B: one wave per 64 KiB piece on a 16-wave
// persistent grid ran d3 1.5x slower -- half the loads in flight.)  A task is
// self-describing (ApplyTask): one descriptor load, then the payload verdict.
// With fin, the first workgroups finalize the IOs that need no post job first
// (their inputs -- the pre hashes -- are complete when this kernel starts).
template <uint32_t POLY, bool NTL = false, bool NTS = false, bool HW = false>
__global__ __launch_bounds__(256) void k_update_apply(hf3fs_crc_update_io* __restrict__ ios, uint64_t n,
                                                      uint32_t max_len, uint8_t type, int mode, UpdateScratch s,
                                                      const PolyTables* __restrict__ T, int fin, uint64_t* hint) {
  __shared__ uint32_t ticket;
  // (the self-check audit stays in the finalize launch: inlined here it raised the copy
  // loop's register count and cost 85 us per d3 batch in occupancy)
  if (fin)
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
      finalize_one(ios, i, type, mode, s, GfGlobal<POLY>{T}, max_len, 1);
  const uint64_t ntasks = *reinterpret_cast<const uint64_t*>(s.ctl + kCtlTasks);
  if (hint && blockIdx.x == 0 && threadIdx.x == 0)
    store_hint(hint, *reinterpret_cast<const uint64_t*>(s.ctl + kCtlPieces), n);
  uint64_t t = blockIdx.x;
  while (t < ntasks) {
    const ApplyTask tk = s.tasks[t];  // (the reverse of the pre-hash order measured the same: 1.712 vs 1.710 ms)
    if (!(tk.verify && s.pre_out[2 * (uint64_t)tk.io] != tk.wval))  // mismatch: chunk untouched
    {
      if (HW)
        copy_range_hw<4, NTL, NTS>(tk.dst, tk.src, tk.len, threadIdx.x, blockDim.x);
      else
        copy_range<4, NTL, true, 1024, NTS>(tk.dst, tk.src, tk.len, threadIdx.x, blockDim.x);
    }
    __syncthreads();
    if (threadIdx.x == 0) ticket = atomicAdd(s.ctl + kCtlQueueApply, 1u);
    __syncthreads();
    t = gridDim.x + (uint64_t)ticket;
  }
}

template <uint32_t POLY, bool HWNT = false>
__global__ __launch_bounds__(kThreads) void k_update_fused(hf3fs_crc_update_io* __restrict__ ios, uint64_t n,
                                                           uint32_t max_len, uint8_t type, int mode, UpdateScratch s,
                                                           const PolyTables* __restrict__ T) {
  __shared__ uint32_t lds[kLdsWords + kFoldLdsWords];
  __shared__ uint32_t s_part[kWaves];
  __shared__ uint64_t s_chunk, s_pay, s_next;
  __shared__ uint32_t s_job[12];
  fill_lds_fold<POLY>(lds, T);
  const StepLds lj = step_lds(lds, threadIdx.x & 63);
  const uint32_t* lc = lds + kLdsWords;
  uint64_t i = blockIdx.x;
  while (i < n) {
    if (threadIdx.x == 0) {
      uint32_t pre_max, post_max;
      const Eff e = prep_one(ios, i, max_len, type, mode, s, pre_max, post_max);
      if (pre_max) atomicMax(&s.ctl[kCtlPreMax], pre_max);
      if (post_max) atomicMax(&s.ctl[kCtlPostMax], post_max);
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
    if (hash_payload) crc_payload = wg_hash<POLY>(pay, len, ~0u ^ (s.fault_io == i + 1 ? 1u : 0u), lj, lc, T, s_part);
    if (ok && !(verify && crc_payload != wval)) {  // mismatch: chunk untouched
      if (write) {
        if (olen && !te)
          lin_old = wg_write_hash_old<POLY>(chunk + off, pay, len, olen, lj, lc, T, s_part);
        else if (HWNT)
          copy_range_hw<4, false, true>(chunk + off, pay, len, threadIdx.x, blockDim.x);
        else
          copy_range<4, false, true, 1024>(chunk + off, pay, len, threadIdx.x, blockDim.x);
      }
      if (zto > zfrom) {
        if (HWNT)
          copy_range_hw<4, false, true>(chunk + zfrom, 0, zto - zfrom, threadIdx.x, blockDim.x);
        else
          copy_range<4, false, true, 1024>(chunk + zfrom, 0, zto - zfrom, threadIdx.x, blockDim.x);
      }
    }
    if (ok && olen && te) lin_old = wg_hash<POLY>(chunk + s1, olen, 0u, lj, lc, T, s_part);
    if (threadIdx.x == 0) {
      s.pre_out[2 * i] = crc_payload;
      s.pre_out[2 * i + 1] = lin_old;
      s_next = gridDim.x + (uint64_t)atomicAdd(s.ctl + kCtlQueueFused, 1u);
    }
    __syncthreads();
    i = s_next;
  }
}

// One lane per IO, wave-uniform loop (the audit needs whole waves).
template <uint32_t POLY>
__global__ __launch_bounds__(256) void k_update_finalize(hf3fs_crc_update_io* __restrict__ ios, uint64_t n,
                                                         uint8_t type, int mode, UpdateScratch s,
                                                         const PolyTables* __restrict__ T,
                                                         const ShortTables* __restrict__ S, uint32_t max_len,
                                                         int which, int audit) {
  const uint32_t lane = threadIdx.x & 63;
  // post-only pass (three-pass pipeline: the apply gave every verdict) with no post job in the
  // batch and no audit: nothing to do
  const bool no_post = __builtin_amdgcn_readfirstlane(s.ctl[kCtlPostMax]) == 0;
  if (which == 2 && !audit && no_post) return;
  __shared__ uint32_t l_dw[4 * 256], l_pw[kPowDigits * 256], l_iw[kPowDigits * 256];
  if (!(which == 2 && no_post)) {  // (the audit-only pass multiplies nothing)
    for (uint32_t k = threadIdx.x; k < 4 * 256; k += blockDim.x) l_dw[k] = (&S->dw[0][0])[k];
    for (uint32_t k = threadIdx.x; k < kPowDigits * 256; k += blockDim.x) {
      l_pw[k] = (&T->pow8b[0][0])[k];
      l_iw[k] = (&T->inv8b[0][0])[k];
    }
    __syncthreads();
  }
  const GfLds<POLY> g{l_dw, l_pw, l_iw, T};
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); i0 < n;
       i0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = i0 + lane;
    bool flag = false;
    if (i < n) {
      finalize_one(ios, i, type, mode, s, g, max_len, which);
      flag = audit && ios[i].status == HF3FS_CRC_CHECKSUM_MISMATCH;
    }
    uint64_t m = __ballot(flag);
    while (m) {  // wave-uniform
      const int bit = __ffsll((unsigned long long)m) - 1;
      m &= m - 1;
      audit_one<POLY>(ios, i0 + bit, type, mode, s, T, S, max_len, lane);
    }
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

uint64_t update_piece_cap(uint64_t n, uint32_t max_len, uint32_t piece_shift) {
  // payload + gap of one IO lie in [0, max_len): at most max_len / P + 2 pieces each
  return n * (((uint64_t)max_len >> piece_shift) + 4);
}

size_t update_scratch_bytes(uint64_t n, uint32_t pieces, uint32_t nw, uint64_t ptab_cap) {
  const uint64_t tasks = n * 2 * (uint64_t)(pieces + 1);
  const uint64_t runs = kRunBlocksMax * 8 + (nw + 1) * (4 + 8);
  return n * 2 * (8 + 8 + 4 + 4) * 2 + tasks * sizeof(ApplyTask) + kCtlWords * 4 + runs + ptab_cap * 4 + 1024;
}

void update_scratch_carve(void* base, uint64_t n, uint32_t pieces, uint32_t piece_min, uint32_t nw,
                          uint64_t ptab_cap, UpdateScratch* s) {
  uint8_t* p = (uint8_t*)base;
  auto take = [&](size_t bytes) {
    uint8_t* r = p;
    p += (bytes + 15) & ~size_t(15);
    return r;
  };
  s->ctl = (uint32_t*)take(kCtlWords * 4);
  s->pre_addr = (uint64_t*)take(2 * n * 8);
  s->pre_len = (uint64_t*)take(2 * n * 8);
  s->pre_start = (uint32_t*)take(2 * n * 4);
  s->pre_out = (uint32_t*)take(2 * n * 4);
  s->post_addr = (uint64_t*)take(2 * n * 8);
  s->post_len = (uint64_t*)take(2 * n * 8);
  s->post_start = (uint32_t*)take(2 * n * 4);
  s->post_out = (uint32_t*)take(2 * n * 4);
  s->tasks = (ApplyTask*)take(n * 2 * (uint64_t)(pieces + 1) * sizeof(ApplyTask));
  s->pieces = pieces;
  s->piece_min = piece_min;
  s->ptab = (uint32_t*)take(ptab_cap * 4);
  s->piece_shift = 13;
  s->one_shot = 0;
  s->run_partial = (uint64_t*)take(kRunBlocksMax * 8);
  s->run_bal = (uint32_t*)take((nw + 1) * 4);
  s->run_boff = (uint64_t*)take((nw + 1) * 8);
  s->run_blocks = (uint32_t)std::min<uint64_t>(kRunBlocksMax, std::max<uint64_t>(1, 2 * n / 256));
  s->run_waves = nw;
  s->runs_used = 0;
  s->diag = nullptr;
  s->fault_io = 0;
}

hipError_t launch_update_prep(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type, int mode,
                              const UpdateScratch& s, bool place_runs, hipStream_t st) {
  // place_runs (2n <= kPrepRunJobs, so one pass of the IO loop): one more workgroup for the runs.
  // 1024-thread workgroups: the runs workgroup derives 4 IOs per thread (with 256 threads it
  // took 30 us, the 16 IOs per thread of derive + pre_lens on one wave per SIMD).
  const uint64_t want = (n + kPrepIoThreads - 1) / kPrepIoThreads;
  const unsigned grid = (unsigned)(want < 1024 ? (want ? want : 1) : 1024);
  hipLaunchKernelGGL(k_update_prep, dim3(grid + (place_runs ? 1 : 0)), dim3(kPrepThreads), 0, st, ios, n, max_len,
                     type, mode, s, place_runs ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_update_apply(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type, int mode,
                               const UpdateScratch& s, const DeviceTables* tabs, bool finalize_delta, uint32_t grid,
                               int nt, uint64_t ptab_cap, uint64_t* hint, hipStream_t st) {
  // U = 4 granules in flight per thread, cached loads/stores, one aligned load per misaligned
  // granule + a lane shift, 1 KiB-aligned store rows: the A/Bs of DESIGN.md 3.2 and the copy
  // probe (profiles/r03_probe_copy.log: every copy form measured within 5 % of this one).
  const int fin = finalize_delta ? 1 : 0;
  // nt: bit 0 non-temporal payload loads, bit 1 non-temporal chunk stores, bit 2 the copy_range_hw
  // body (option apply_nt, A/B)
  const PolyTables* T = type == kTypeCrc32 ? &tabs->poly[1] : &tabs->poly[0];
#define HF3FS_APPLY(P, L, S, H)                                                                         \
  hipLaunchKernelGGL((k_update_apply<P, L, S, H>), dim3(grid), dim3(256), 0, st, ios, n, max_len, type, mode, s, \
                     T, fin, hint)
#define HF3FS_APPLY_NT(P)                               \
  switch (nt & 7) {                                     \
    case 1: HF3FS_APPLY(P, true, false, false); break;  \
    case 2: HF3FS_APPLY(P, false, true, false); break;  \
    case 3: HF3FS_APPLY(P, true, true, false); break;   \
    case 4: HF3FS_APPLY(P, false, false, true); break;  \
    case 5: HF3FS_APPLY(P, true, false, true); break;   \
    case 6: HF3FS_APPLY(P, false, true, true); break;   \
    case 7: HF3FS_APPLY(P, true, true, true); break;    \
    default: HF3FS_APPLY(P, false, false, false);       \
  }
  if (s.one_shot) {  // nt bit 0: non-temporal payload loads; stores always non-temporal (the probe's best)
    const uint64_t* count = reinterpret_cast<const uint64_t*>(s.ctl + kCtlPieces);
#define HF3FS_ONE_SHOT(SH)                                                                                     \
  do {                                                                                                         \
    if (nt & 1)                                                                                                \
      hipLaunchKernelGGL((k_update_apply_one_shot<SH, true, true>), dim3(grid), dim3(256), 0, st, s.tasks,      \
                         s.ptab, s.pre_out, count, n, ptab_cap, hint);                                         \
    else                                                                                                       \
      hipLaunchKernelGGL((k_update_apply_one_shot<SH, false, true>), dim3(grid), dim3(256), 0, st, s.tasks,     \
                         s.ptab, s.pre_out, count, n, ptab_cap, hint);                                         \
  } while (0)
    switch (s.piece_shift) {
      case 12: HF3FS_ONE_SHOT(12); break;
      case 14: HF3FS_ONE_SHOT(14); break;
      default: HF3FS_ONE_SHOT(13);
    }
#undef HF3FS_ONE_SHOT
  } else if (type == kTypeCrc32) {
    HF3FS_APPLY_NT(kPolyCrc32)
  } else {
    HF3FS_APPLY_NT(kPolyCrc32c)
  }
#undef HF3FS_APPLY_NT
#undef HF3FS_APPLY
  return hipGetLastError();
}

hipError_t launch_update_fused(hf3fs_crc_update_io* ios, uint64_t n, uint32_t max_len, uint8_t type, int mode,
                               const UpdateScratch& s, const DeviceTables* tabs, uint32_t grid, int nt,
                               hipStream_t st) {
  // (nt & 6) == 6: the copy_range_hw body with non-temporal stores, as in the apply (option apply_nt)
  const bool hwnt = (nt & 6) == 6;
  const PolyTables* T = type == kTypeCrc32 ? &tabs->poly[1] : &tabs->poly[0];
  if (type == kTypeCrc32) {
    if (hwnt)
      hipLaunchKernelGGL((k_update_fused<kPolyCrc32, true>), dim3(grid), dim3(kThreads), 0, st, ios, n, max_len, type,
                         mode, s, T);
    else
      hipLaunchKernelGGL((k_update_fused<kPolyCrc32, false>), dim3(grid), dim3(kThreads), 0, st, ios, n, max_len, type,
                         mode, s, T);
  } else {
    if (hwnt)
      hipLaunchKernelGGL((k_update_fused<kPolyCrc32c, true>), dim3(grid), dim3(kThreads), 0, st, ios, n, max_len, type,
                         mode, s, T);
    else
      hipLaunchKernelGGL((k_update_fused<kPolyCrc32c, false>), dim3(grid), dim3(kThreads), 0, st, ios, n, max_len,
                         type, mode, s, T);
  }
  return hipGetLastError();
}

hipError_t launch_update_finalize(hf3fs_crc_update_io* ios, uint64_t n, uint8_t type, int mode,
                                  const UpdateScratch& s, const DeviceTables* tabs, uint32_t max_len, int which,
                                  bool audit, hipStream_t st) {
  const int au = audit && s.diag ? 1 : 0;
  if (type == kTypeCrc32)
    hipLaunchKernelGGL(k_update_finalize<kPolyCrc32>, dim3(grid_for(n, 4096)), dim3(256), 0, st, ios, n, type, mode,
                       s, &tabs->poly[1], &tabs->sh[1], max_len, which, au);
  else
    hipLaunchKernelGGL(k_update_finalize<kPolyCrc32c>, dim3(grid_for(n, 4096)), dim3(256), 0, st, ios, n, type, mode,
                       s, &tabs->poly[0], &tabs->sh[0], max_len, which, au);
  return hipGetLastError();
}

}  // namespace hf3fs_crc
