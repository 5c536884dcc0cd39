// frame_kernels.hip -- see frame_kernels.h.
#include "crc_device.h"
#include "frame_kernels.h"

namespace hf3fs_crc {
namespace {

constexpr uint32_t kSerdeMagic = 0x86;  // kSerdeMessageMagicNum (MessageHeader.h:14)

unsigned grid_of(uint64_t n) {
  const uint64_t want = (n + 255) / 256;
  return (unsigned)(want < 4096 ? (want ? want : 1) : 4096);
}


// Frames the stream path cannot take: size above max_size, or a payload that
// overlaps or precedes the one before it.
__global__ __launch_bounds__(256) void k_frame_check(const hf3fs_crc_frame* __restrict__ fr, uint64_t n, uint32_t max_size,
                              uint32_t* __restrict__ flags) {
  uint32_t bad = 0;
  uint64_t pay = 0, gap = 0;  // payload bytes, bytes between payloads beyond the 8-byte headers
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t off = fr[i].offset, end = off + fr[i].size;
    bad |= fr[i].size > max_size || end < off;
    pay += fr[i].size;
    if (i + 1 < n) {
      const uint64_t next = fr[i + 1].offset;
      bad |= end > next;
      gap += next > end + kFrameHeaderBytes ? next - end - kFrameHeaderBytes : 0;
    }
  }
  // one atomic per workgroup and word (same-address atomics serialise in L2)
  __shared__ unsigned long long s_pay[4], s_gap[4];
  __shared__ uint32_t s_bad[4];
  const bool any_bad = __ballot(bad) != 0;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    pay += __shfl_xor(pay, d, 64);
    gap += __shfl_xor(gap, d, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_pay[w] = pay;
    s_gap[w] = gap;
    s_bad[w] = any_bad;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long P = 0, G = 0;
    uint32_t B = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
      P += s_pay[k];
      G += s_gap[k];
      B |= s_bad[k];
    }
    unsigned long long* sums = reinterpret_cast<unsigned long long*>(flags + 4);
    if (B) atomicOr(flags + 2, 1u);
    if (P) atomicAdd(sums, P);
    if (G) atomicAdd(sums + 1, G);
  }
}

// Record path for the frames of this thread: job i = (base + offset_i, size_i), v[i] = 0,
// status / computed reset; the longest job -> flags[0] (one atomic per wave).
__device__ void record_prep(const uint8_t* base, hf3fs_crc_frame* __restrict__ frames, uint64_t n,
                            uint32_t max_size, uint64_t* __restrict__ addr, uint64_t* __restrict__ len,
                            uint32_t* __restrict__ v, uint32_t* __restrict__ flags) {
  uint32_t mx = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    hf3fs_crc_frame f = frames[i];
    const bool ok = f.size <= max_size;
    addr[i] = ok ? (uint64_t)(base + f.offset) : 0;
    len[i] = ok ? f.size : 0;
    v[i] = 0;
    f.status = ok ? HF3FS_CRC_OK : HF3FS_CRC_INVALID_ARG;
    f.computed = 0;
    frames[i] = f;
    if (ok && f.size > mx) mx = f.size;
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    const uint32_t o = __shfl_xor(mx, d, 64);
    mx = o > mx ? o : mx;
  }
  if ((threadIdx.x & 63) == 0 && mx) atomicMax(flags, mx);  // one per wave, not per frame
}

// Segment of byte position p: 32-bit division of its 1 KiB block index (spans
// below 4 TiB) instead of a 64-bit division by the segment bytes (a ~100-VALU
// software routine on gfx950).
__device__ __forceinline__ uint64_t seg_of(uint64_t p, uint64_t a0, uint32_t seg_blocks) {
  return (uint32_t)((p - a0) >> 10) / seg_blocks;
}

// Segment grid over the blocks holding [lo, hi] (whole 1 KiB blocks, about
// seg_target segments of equal size) and seg_first[k] = the first frame whose
// payload ends at or after segment k's start (frame i writes the segments after
// the one holding the previous frame's end, up to the one holding its own).
// flags[3] marks payloads spanning more than kFrameHornerSegs segments: the
// finalize takes those from the segment prefix table (k_frame_seg_scan).
// The same launch takes the path decision (every workgroup decides the same way) and, on the
// record path, prepares the record jobs (record_prep): one launch fewer per batch.  It also
// zeroes *count (the finalize's mismatch count), so a batch needs ONE zeroing launch
// (flags[0..15]; flags[8] is the record path's ticket counter).
__global__ void k_frame_map(const uint8_t* base, hf3fs_crc_frame* __restrict__ fr, uint64_t n, uint64_t seg_target,
                            uint64_t waves, uint32_t* __restrict__ flags, FrameStreamParams* __restrict__ prm,
                            uint32_t* __restrict__ seg_first, uint32_t max_size, uint64_t* __restrict__ addr,
                            uint64_t* __restrict__ len, uint32_t* __restrict__ v, uint32_t* __restrict__ count,
                            int try_stream) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *count = 0;  // the finalize adds the mismatches
  const uint64_t b = (uint64_t)base;
  const uint64_t lo = b + fr[0].offset, hi = b + fr[n - 1].offset + fr[n - 1].size;
  const uint64_t a0 = lo & ~uint64_t(kBlockBytes - 1), hib = (hi & ~uint64_t(kBlockBytes - 1)) + kBlockBytes;
  const uint64_t blocks = (hib - a0) / kBlockBytes;
  const uint64_t sb = (blocks + seg_target - 1) / seg_target;  // blocks per segment
  const uint64_t seg = sb * kBlockBytes, nseg = (blocks + sb - 1) / sb;
  // Sparse batches stay on the record path: the stream path reads the whole span, so
  // frames scattered over a large receive buffer (gaps beyond the headers larger than
  // the payload bytes) would cost the gaps too.  A span of 4 TiB or more too (seg_of takes
  // 32-bit block indices), and a wave's byte range must stay below 2^31 (the stream kernel
  // steers by 32-bit offsets in it).
  const unsigned long long* sums = reinterpret_cast<const unsigned long long*>(flags + 4);
  const bool stream = try_stream && !flags[2] && sums[1] <= sums[0] && !(blocks >> 32) &&
                      (nseg + waves - 1) / waves * seg < (1ull << 31);
  if (!stream) {
    record_prep(base, fr, n, max_size, addr, len, v, flags);
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *prm = FrameStreamParams{a0, seg, nseg, lo, hi};
    flags[1] = 1;
  }
  uint32_t lng = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t s0 = b + fr[i].offset;
    const uint64_t k1 = seg_of(s0 + fr[i].size, a0, (uint32_t)sb);
    const uint64_t k0 = i ? seg_of(b + fr[i - 1].offset + fr[i - 1].size, a0, (uint32_t)sb) + 1 : 0;
    for (uint64_t k = k0; k <= k1; ++k) seg_first[k] = (uint32_t)i;
    lng |= k1 - seg_of(s0, a0, (uint32_t)sb) > kFrameHornerSegs;
  }
  if (__ballot(lng) && (threadIdx.x & 63) == 0) atomicOr(flags + 3, 1u);
}

// seg_pre[k] = lin(all segments before k) referenced to segment k's start, for
// payloads spanning many segments.  One workgroup: a Horner run per thread
// over its consecutive segments, an inclusive scan of the runs over the
// workgroup ((v1, c1) then (v2, c2) -> v1 * x^(8 seg c2) ^ v2), then the runs
// again writing the prefixes.  Returns at once unless flags[3].
template <uint32_t POLY>
__global__ __launch_bounds__(1024) void k_frame_seg_scan(const uint32_t* __restrict__ flags,
                                                         const FrameStreamParams* __restrict__ prm,
                                                         const uint32_t* __restrict__ seg_lin,
                                                         uint32_t* __restrict__ seg_pre, const PolyTables* __restrict__ T) {
  __shared__ uint32_t sv[1024], sc[1024];
  if (!flags[1] || !flags[3]) return;
  const uint64_t nseg = prm->nseg, seg = prm->seg;
  const uint32_t t = threadIdx.x;
  const uint64_t per = (nseg + 1023) / 1024;
  const uint64_t k0 = t * per < nseg ? t * per : nseg, k1 = k0 + per < nseg ? k0 + per : nseg;
  const uint32_t xs = xpow8_bytes((int64_t)seg, T, POLY);
  uint32_t v = 0;
  for (uint64_t k = k0; k < k1; ++k) v = gf_mul(v, xs, POLY) ^ seg_lin[k];
  uint32_t c = (uint32_t)(k1 - k0);
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    sv[t] = v;
    sc[t] = c;
    __syncthreads();
    if (t >= d) {
      const uint32_t pv = sv[t - d], pc = sc[t - d];
      v = (pv ? gf_mul(pv, xpow8_bytes((int64_t)(seg * c), T, POLY), POLY) : 0u) ^ v;
      c += pc;
    }
    __syncthreads();
  }
  sv[t] = v;
  __syncthreads();
  uint32_t p = t ? sv[t - 1] : 0u;  // everything before segment k0, referenced to its start
  for (uint64_t k = k0; k < k1; ++k) {
    seg_pre[k] = p;
    p = gf_mul(p, xs, POLY) ^ seg_lin[k];
  }
}

// Boundary math of the stream kernel (the lane-weight fold, crc_device.h):
// branch-free, in-row lane steps are DPP moves, not LDS permutes.
// The block step multiplies every stream by x^8192 and the fold is linear, so
// fold(step(S)) = stride_step(fold(S)): a boundary folds the block's words UNSTEPPED and
// steps the one folded value (one lookup round per lane instead of the four streams'
// sixteen; f4 mix -1..-4 %, 1 KiB frames -8 %, profiles/r06_f4_poststep_ab.log).
// block_prefix_raw: the exclusive lane prefix P_L = sum_{l < L} u_l x^(-128 l) of the
// block's unstepped words, u_l the lane's weighted Horner value.
__device__ __forceinline__ uint32_t block_prefix_raw(const uint4& w, const FoldLds& f, int lane) {
  Streams bs;
  bs.p0 = w.x;
  bs.p1 = w.y;
  bs.p2 = w.z;
  bs.p3 = w.w;
  const uint32_t u = weighted_lw(bs, f);
  const uint32_t v = half_scan(u);
  const uint32_t a = __builtin_amdgcn_readlane(v, 31);
  const uint32_t x = v ^ u;  // exclusive within the half
  const uint32_t hi = a ^ mulc_b(x, f.ch);
  return lane < 32 ? x : hi;
}

template <uint32_t POLY>
__global__ __launch_bounds__(kThreads) void k_frame_stream(const uint8_t* base, const hf3fs_crc_frame* __restrict__ fr,
                                                           uint64_t n, const uint32_t* __restrict__ flags,
                                                           const FrameStreamParams* __restrict__ prm,
                                                           const uint32_t* __restrict__ seg_first,
                                                           uint32_t* __restrict__ seg_lin, uint32_t* __restrict__ ev,
                                                           const PolyTables* __restrict__ T,
                                                           const FoldTables* __restrict__ FT) {
  __shared__ uint32_t lds[kLdsWords + kFoldWords];
  if (!__builtin_amdgcn_readfirstlane(flags[1])) return;  // the record path has the batch
  fill_lds_foldtables(lds, T, FT);
  const FoldLds fl = fold_lds(lds + kLdsWords);
#define HF3FS_FOLD(st_) fold_lw(st_, fl)
#ifndef HF3FS_FRAME_PREFETCH
#define HF3FS_FRAME_PREFETCH 4
#endif
  // blocks in flight per wave (rolling).  Measured in one process
  // (scripts/ab_f4_inproc.py, f4 mix / 16 KiB frames): U = 4, 6, 8 within
  // 2 %; 4 keeps the code and the register count smallest.
  constexpr int U = HF3FS_FRAME_PREFETCH;
  const int lane = threadIdx.x & 63;
  const StepLds lj = step_lds(lds, lane);
  const uint64_t a0 = prm->a0, seg = prm->seg, nseg = prm->nseg, lo = prm->lo, hi = prm->hi;
  const uint64_t lane_off = (uint64_t)lane * 16;
  const bool data = hi > lo;
  const uint64_t glo = lo & ~uint64_t(15), ghi = data ? (hi - 1) & ~uint64_t(15) : glo;
  const uint64_t fb = (uint64_t)base;
  // Every load is unconditional (addresses clamped into valid bytes) and no
  // loaded value merges at a branch join: a conditional load or a join would
  // make the compiler wait for ALL outstanding loads (vmcnt(0)) and collapse
  // the U-deep prefetch.
  auto load = [&](uint64_t blk) -> uint4 {
    uint64_t g = blk + lane_off;
    g = g < glo ? glo : (g > ghi ? ghi : g);
    return gload16s<true>(g);
  };
  // frame f's (offset, size) for the window; f >= n reads frame n - 1 and is
  // turned into the never-reached position ~0 when the window is installed
  auto fetch = [&](uint64_t f, uint64_t& off, uint32_t& size) {
    const hf3fs_crc_frame* p = fr + (f < n ? f : n - 1);
    off = p->offset;
    size = p->size;
  };
  // wave w takes segments [k0, k1): one contiguous byte range, so the block
  // prefetch and the frame window run on across segment boundaries
  const uint64_t nw = (uint64_t)gridDim.x * kWaves;
  const uint64_t per = (nseg + nw - 1) / nw;
  const uint64_t wid = (uint32_t)__builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + (threadIdx.x >> 6));
  const uint64_t k0 = wid * per;
  if (k0 >= nseg) return;  // after fill_lds: no barrier follows
  const uint64_t k1 = k0 + per < nseg ? k0 + per : nseg;
  const uint64_t hib = (hi & ~uint64_t(kBlockBytes - 1)) + kBlockBytes;
  const uint64_t b0 = a0 + k0 * seg, b1e = a0 + k1 * seg, b1 = b1e < hib ? b1e : hib;
  const uint64_t nblk = (b1 - b0) / kBlockBytes;
  const uint64_t blast = b1 - kBlockBytes;  // reloads past the range re-read its last block (cache hits)
  const uint64_t hfull = hi & ~uint64_t(kBlockBytes - 1);  // blocks ending at or before it lie inside the span
  // Control by 32-bit offsets from b0 (the range is < 2^31 bytes, k_frame_map): wave-uniform
  // compares of 64-bit addresses are VALU on gfx950 (no s_cmp_lt_u64), of 32-bit ones SALU.
  // Positions before b0 map to 0, past 2^32 to the maximum.
  auto R = [&](uint64_t x) -> uint32_t {
    return x <= b0 ? 0u : (x - b0 >= 0xffffffffull ? 0xffffffffu : (uint32_t)(x - b0));
  };
  const uint32_t lo_r = R(lo), hi_r = R(hi), blast_r = R(blast), hfull_r = R(hfull);
  uint64_t fw = (uint32_t)__builtin_amdgcn_readfirstlane(seg_first[k0]);
  uint64_t c_off, n_off;
  uint32_t c_sz, n_sz;
  fetch(fw + lane, c_off, c_sz);
  fetch(fw + 64 + lane, n_off, n_sz);
  uint64_t prev_e = 0;  // payload end of frame fw - 1
  if (fw > 0) prev_e = fb + fr[fw - 1].offset + fr[fw - 1].size;
  uint4 c[U];
#pragma unroll
  for (int q = 0; q < U; ++q) {
    const uint64_t blk = b0 + q * kBlockBytes;
    c[q] = load(blk < blast ? blk : blast);
  }
  // The window: lane i holds frame fw + i's payload [s_i, e_i) as 32-bit
  // offsets r(p) = p - b0 + 1 into this wave's range (0 before it, saturated
  // past it).  Every end is a boundary; a start is one only for the first
  // frame or after a gap of more than kFrameGapMax bytes (the finalize derives
  // the others from the end before them and the header bytes in between).
  auto rel = [&](uint64_t p) -> uint32_t {
    return p < b0 ? 0u : (p - b0 >= 0xffffffffull ? 0xffffffffu : (uint32_t)(p - b0 + 1));
  };
  uint32_t s_i, e_i;
  bool sev_i;
  auto install = [&](uint64_t f, uint64_t off, uint32_t size) {
    const bool ok = f < n;
    const uint64_t s = fb + off, e = s + size;
    const uint32_t pl = __shfl_up((uint32_t)e, 1, 64), ph = __shfl_up((uint32_t)(e >> 32), 1, 64);
    const uint64_t ep = lane ? ((uint64_t)ph << 32) | pl : prev_e;
    sev_i = ok && (f == 0 || s - ep > kFrameGapMax);
    s_i = ok ? rel(s) : 0xffffffffu;
    e_i = ok ? rel(e) : 0xffffffffu;
  };
  install(fw + lane, c_off, c_sz);
  // first boundary at or after X in the window (sorted: s_i <= e_i <= s_{i+1})
  auto first_at = [&](uint32_t X) -> uint32_t {
    const uint64_t me = __ballot(e_i >= X);
    if (!me) return 0xffffffffu;
    const uint64_t ms = __ballot(sev_i && s_i >= X);
    const int ie = __builtin_ctzll(me);
    if (ms) {
      const int is = __builtin_ctzll(ms);
      if (is <= ie) return __builtin_amdgcn_readlane(s_i, is);
    }
    return __builtin_amdgcn_readlane(e_i, ie);
  };
  uint32_t next = first_at(1);
  // this lane's frame boundaries found so far in the window, stored when the
  // window moves on; the drain after the stores keeps them from turning every
  // later wait in the loop into a full one (loads and stores share vmcnt)
  uint32_t vs_ = 0, ve_ = 0;
  bool fs_ = false, fe_ = false;
  auto flush = [&]() {
    if (fs_) ev[2 * (fw + lane)] = vs_;
    if (fe_) ev[2 * (fw + lane) + 1] = ve_;
    fs_ = fe_ = false;
  };
  uint64_t kc = k0;
  uint32_t send_r = (uint32_t)seg;  // current segment and its end (offset from b0)
  const uint32_t nblk32 = (uint32_t)nblk;
  Streams st;
  for (uint32_t j = 0; j < nblk32; j += U) {
    {  // a group of U blocks without a boundary, a segment end or a span edge: the short path
      const uint32_t g = j * kBlockBytes, ge = g + U * kBlockBytes;
      const uint64_t Ge = b0 + ge;
      if (j + U <= nblk32 && send_r >= ge && next >= ge + 1 && g >= lo_r && ge <= hi_r) {
        if (ge + U * kBlockBytes <= blast_r && ge + U * kBlockBytes <= hfull_r) {
          // the U blocks refilled are whole blocks of the span: no clamping
#pragma unroll
          for (int q = 0; q < U; ++q) {
            const uint4 w = c[q];
            c[q] = gload16s<true>(Ge + q * kBlockBytes + lane_off);
            st.step(w, lj);
          }
        } else {
#pragma unroll
          for (int q = 0; q < U; ++q) {
            const uint4 w = c[q];
            const uint32_t nb_r = g + (q + U) * kBlockBytes;
            c[q] = load(b0 + (nb_r < blast_r ? nb_r : blast_r));
            st.step(w, lj);
          }
        }
        continue;
      }
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      if (j + q >= nblk32) break;  // wave-uniform
      const uint32_t B_r = (j + q) * kBlockBytes, Bn_r = B_r + kBlockBytes;
      const uint64_t B = b0 + B_r;
      const uint4 w0 = c[q];
      const uint32_t nb_r = B_r + U * kBlockBytes;
      if (nb_r + kBlockBytes <= hfull_r && nb_r <= blast_r) {  // interior refill: no per-lane clamp
        c[q] = gload16s<true>(b0 + nb_r + lane_off);
      } else {
        asm volatile("" ::: "memory");  // keeps this a branch (no if-conversion into both address forms)
        c[q] = load(b0 + (nb_r < blast_r ? nb_r : blast_r));
      }
      if (B_r == send_r) {  // segment boundary: its value, fresh streams for the next
        const uint32_t L = HF3FS_FOLD(st);
        if (lane == 0) seg_lin[kc] = L;
        st = Streams();
        ++kc;
        send_r += (uint32_t)seg;
      }
      // span edges: byte masks from addresses only (no branch on loaded data)
      uint32_t m0 = ~0u, m1 = ~0u, m2 = ~0u, m3 = ~0u;
      if (B_r < lo_r || Bn_r > hi_r) {
        const uint64_t g = B + lane_off;
        const uint64_t x0 = lo > g ? lo : g, x1 = hi < g + 16 ? hi : g + 16;
        const int sb = x0 < x1 ? (int)(x0 - g) : 0, eb = x0 < x1 ? (int)(x1 - g) : 0;
        m0 = dword_mask(sb, eb, 0);
        m1 = dword_mask(sb, eb, 1);
        m2 = dword_mask(sb, eb, 2);
        m3 = dword_mask(sb, eb, 3);
      }
      const uint4 w = make_uint4(w0.x & m0, w0.y & m1, w0.z & m2, w0.w & m3);
      const uint32_t rB = B_r + 1, rBn = rB + kBlockBytes;  // r() of B and Bn
      if (next < rBn) {  // wave-uniform: boundaries in this block
        const bool hs = sev_i && s_i >= rB && s_i < rBn, he = e_i >= rB && e_i < rBn;
        const uint64_t bs_ = __ballot(hs), be_ = __ballot(he);
        const bool more = __builtin_amdgcn_readlane(e_i, 63) < rBn && fw + 64 < n;  // the next window has some too
        if (!more && __popcll(bs_) + __popcll(be_) <= (int)kFrameSparse) {
          // few boundaries: each from the streams with the block's words below its
          // granule added, folded, then stepped (stride_step of the folded value)
          uint64_t ms = bs_, me = be_;
          while (ms | me) {
            const bool is_s = ms != 0;
            const int t = __builtin_ctzll(is_s ? ms : me);
            const uint32_t pr = __builtin_amdgcn_readlane(is_s ? s_i : e_i, t);
            const int L = (int)((pr - rB) >> 4);
            const uint32_t m = lane < L ? ~0u : 0u;
            Streams u;
            u.p0 = __builtin_amdgcn_bitop3_b32(st.p0, st.t0, w.x & m, 0x96);
            u.p1 = __builtin_amdgcn_bitop3_b32(st.p1, st.t1, w.y & m, 0x96);
            u.p2 = __builtin_amdgcn_bitop3_b32(st.p2, st.t2, w.z & m, 0x96);
            u.p3 = __builtin_amdgcn_bitop3_b32(st.p3, st.t3, w.w & m, 0x96);
            const uint32_t E = __builtin_amdgcn_readfirstlane(stride_step(HF3FS_FOLD(u), lj));
            if (lane == t) {
              if (is_s) {
                vs_ = E;
                fs_ = true;
              } else {
                ve_ = E;
                fe_ = true;
              }
            }
            if (is_s)
              ms &= ms - 1;
            else
              me &= me - 1;
          }
        } else {  // many: fold once, lane prefix of the block
          // P_L = stride_step(fold(st) ^ prefix_L): the boundary value at granule L
          const uint32_t P = stride_step(HF3FS_FOLD(st) ^ block_prefix_raw(w, fl, lane), lj);
          for (;;) {
            const bool hs2 = sev_i && s_i >= rB && s_i < rBn, he2 = e_i >= rB && e_i < rBn;
            const int ls = hs2 ? (int)((s_i - rB) >> 4) : lane;
            const int le = he2 ? (int)((e_i - rB) >> 4) : lane;
            const uint32_t ps = __shfl(P, ls, 64), pe = __shfl(P, le, 64);
            if (hs2) {
              vs_ = ps;
              fs_ = true;
            }
            if (he2) {
              ve_ = pe;
              fe_ = true;
            }
            const uint32_t last = __builtin_amdgcn_readlane(e_i, 63);
            if (last < rBn && fw + 64 < n) {  // window used up inside this block
              flush();
              __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0): drain the stores (gfx9 encoding)
              prev_e = b0 + last - 1;  // frame fw + 63's end (inside the range: last < rBn)
              fw += 64;
              install(fw + lane, n_off, n_sz);
              fetch(fw + 64 + lane, n_off, n_sz);
              continue;
            }
            break;
          }
        }
        next = first_at(rBn);
      }
      st.step(w, lj);
    }
  }
  flush();
  const uint32_t L = HF3FS_FOLD(st);
  if (lane == 0) seg_lin[kc] = L;  // referenced to min(b1, its end): only frames that end later read it
#undef HF3FS_FOLD
}

// LDS image of the finalize tables: ShortTables (dw, b8, xs8: contiguous) then the first two
// byte digits of PolyTables::pow8b.
constexpr int kShortWords = 5 * 256 + kXs8Neg + kXs8Pos;
constexpr int kShXs8 = 5 * 256 + kXs8Neg;  // sh[kShXs8 + n] = x^(8n)
constexpr int kShPow = kShortWords;        // sh[kShPow + 256 j + d] = x^(8 d 256^j), j < 2
constexpr int kShLds = kShPow + 2 * 256;

// lin(bytes [a, b)) for a <= b <= (a & ~15) + 32, any alignment, from at most
// two granules: whole dwords through the x^32 slices (4 independent lookups),
// the edge bytes through the x^8 byte table.
__device__ __forceinline__ uint32_t lin_t(uint64_t a, uint64_t b, const uint32_t* sh) {
  if (a >= b) return 0u;
  const uint64_t g = a & ~uint64_t(15);
  const uint4 w0 = gload16(g);
  const uint4 w1 = b > g + 16 ? gload16(g + 16) : make_uint4(0, 0, 0, 0);
  const uint32_t w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
  const int ja = (int)(a - g), jb = (int)(b - g);
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int lo = ja > 4 * k ? ja : 4 * k, hi = jb < 4 * k + 4 ? jb : 4 * k + 4;
    if (hi - lo == 4) {
      c ^= w[k];
      c = sh[c & 0xffu] ^ sh[256 + ((c >> 8) & 0xffu)] ^ sh[512 + ((c >> 16) & 0xffu)] ^ sh[768 + (c >> 24)];
    } else {
      for (int t = lo - 4 * k; t < hi - 4 * k; ++t) c = (c >> 8) ^ sh[1024 + ((c ^ (w[k] >> (8 * t))) & 0xffu)];
    }
  }
  return c;
}

// v * x^(8 n): small signed n from the direct table, n < 2^16 from two byte digits, others
// from xpow8_bytes; every product through gf_mul_dw on the LDS dword tables.
template <uint32_t POLY>
__device__ __forceinline__ uint32_t mul_x8(uint32_t v, int64_t n, const PolyTables* T, const uint32_t* sh) {
  if (!v) return 0u;
  uint32_t f;
  if (n >= -kXs8Neg && n < kXs8Pos) {
    f = sh[kShXs8 + n];
  } else if (n > 0 && n < 65536) {
    const uint32_t d0 = (uint32_t)n & 0xffu, d1 = (uint32_t)n >> 8;
    f = d1 ? sh[kShPow + 256 + d1] : kOne;
    if (d0) f = d1 ? gf_mul_dw(f, sh[kShPow + d0], sh) : sh[kShPow + d0];
  } else {
    f = xpow8_bytes(n, T, POLY);
  }
  return gf_mul_dw(v, f, sh);
}

// lin(bytes of the segment before p), referenced at p, from its boundary value
// E = lin(segment bytes before the granule of p) referenced at the end of p's
// block: E * x^(8 (p - block end)) ^ lin(granule of p .. p).
// With the previous payload end ep <= p <= ep + 16 in the same segment, E of
// ep serves p directly: the bytes from ep's granule to p are at most 31.
template <uint32_t POLY>
__device__ __forceinline__ uint32_t seg_lin_at(uint32_t E, uint64_t q, uint64_t p, uint64_t lo, const PolyTables* T,
                                               const uint32_t* sh) {
  const uint64_t bend = (q & ~uint64_t(kBlockBytes - 1)) + kBlockBytes;
  const uint64_t g = q & ~uint64_t(15);
  return mul_x8<POLY>(E, (int64_t)p - (int64_t)bend, T, sh) ^ lin_t(g > lo ? g : lo, p, sh);
}

// Processor::unpackSerdeMsg (Processor.h:111-120): the compressed bit comes
// from the received header, calcSerde(data, size, compressed) must equal it.
template <uint32_t POLY>
__global__ __launch_bounds__(256) void k_frame_finalize(const uint8_t* base, hf3fs_crc_frame* __restrict__ frames, uint64_t n,
                                 const uint32_t* __restrict__ v, const uint32_t* __restrict__ flags,
                                 const FrameStreamParams* __restrict__ prm, const uint32_t* __restrict__ ev,
                                 const uint32_t* __restrict__ seg_lin, const uint32_t* __restrict__ seg_pre,
                                 uint32_t* __restrict__ count, const PolyTables* __restrict__ T,
                                 const ShortTables* __restrict__ S) {
  const bool stream = flags[1] != 0;
  __shared__ uint32_t sh[kShLds];
  if (stream) {
    for (int k = threadIdx.x; k < kShortWords; k += blockDim.x) sh[k] = (&S->dw[0][0])[k];  // dw, b8, xs8
    for (int k = threadIdx.x; k < 2 * 256; k += blockDim.x) sh[kShPow + k] = (&T->pow8b[0][0])[k];
    __syncthreads();
  }
  uint32_t bad = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    hf3fs_crc_frame f = frames[i];
    uint32_t val;
    if (stream) {
      const uint64_t a0 = prm->a0, seg = prm->seg, lo = prm->lo;
      const uint64_t s = (uint64_t)base + f.offset, e = s + f.size;
      const uint32_t sbk = (uint32_t)(seg >> 10);
      const uint64_t ks = seg_of(s, a0, sbk), ke = seg_of(e, a0, sbk);
      uint32_t qs;  // lin(segment ks before s), referenced at s
      const uint64_t ep = i ? (uint64_t)base + frames[i - 1].offset + frames[i - 1].size : 0;
      if (i && s - ep <= kFrameGapMax) {  // start derived from the end before it
        qs = seg_of(ep, a0, sbk) == ks ? seg_lin_at<POLY>(ev[2 * i - 1], ep, s, lo, T, sh)
                                   : lin_t(a0 + ks * seg, s, sh);  // a segment starts in between
      } else {
        qs = seg_lin_at<POLY>(ev[2 * i], s, s, lo, T, sh);
      }
      const uint32_t qe = seg_lin_at<POLY>(ev[2 * i + 1], e, e, lo, T, sh);
      if (ks == ke) {
        val = qe ^ mul_x8<POLY>(qs, (int64_t)f.size, T, sh);
      } else {
        // the head: s to the end of segment ks, referenced there
        const uint64_t h = a0 + (ks + 1) * seg, t0 = a0 + ke * seg;
        uint32_t acc = seg_lin[ks] ^ mul_x8<POLY>(qs, (int64_t)(h - s), T, sh);
        if (ke - ks <= kFrameHornerSegs) {  // Horner over the whole segments in between
          const uint32_t xs = xpow8_bytes((int64_t)seg, T, POLY);
          for (uint64_t k = ks + 1; k < ke; ++k) acc = gf_mul_dw(acc, xs, sh) ^ seg_lin[k];
        } else {  // segments ks+1 .. ke-1 from the prefix table: pre[ke] ^ pre[ks+1] * x^(8 (t0 - h))
          acc = mul_x8<POLY>(acc ^ seg_pre[ks + 1], (int64_t)(t0 - h), T, sh) ^ seg_pre[ke];
        }
        val = mul_x8<POLY>(acc, (int64_t)(e - t0), T, sh) ^ qe;
      }
      f.status = HF3FS_CRC_OK;  // calcSerde starts from 0: raw == lin
    } else {
      if (f.status != HF3FS_CRC_OK) {
        ++bad;
        continue;
      }
      val = v[i];
    }
    f.computed = (val & ~0xffu) | kSerdeMagic | (f.checksum & 1u);
    if (f.computed != f.checksum) {
      f.status = HF3FS_CRC_CHECKSUM_MISMATCH;
      ++bad;
    }
    // only the outputs: the thread of frame i + 1 reads this frame's offset and size
    frames[i].computed = f.computed;
    frames[i].status = f.status;
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) bad += __shfl_xor(bad, d, 64);
  __shared__ uint32_t s_bad[4];
  if ((threadIdx.x & 63) == 0) s_bad[threadIdx.x >> 6] = bad;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t b = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) b += s_bad[k];
    if (b) atomicAdd(count, b);
  }
}

}  // namespace

hipError_t launch_frame_check(const hf3fs_crc_frame* frames, uint64_t n, uint32_t max_size, uint32_t* flags,
                              hipStream_t st) {
  const unsigned g = grid_of(n);  // <= 512 workgroups: at most 1536 atomics on flags
  hipLaunchKernelGGL(k_frame_check, dim3(g < 512 ? g : 512), dim3(256), 0, st, frames, n, max_size, flags);
  return hipGetLastError();
}
hipError_t launch_frame_map(const uint8_t* base, hf3fs_crc_frame* frames, uint64_t n, uint64_t seg_target,
                            uint64_t waves, uint32_t* flags, FrameStreamParams* prm, uint32_t* seg_first,
                            uint32_t max_size, uint64_t* addr, uint64_t* len, uint32_t* v, uint32_t* count,
                            bool try_stream, hipStream_t st) {
  hipLaunchKernelGGL(k_frame_map, dim3(grid_of(n)), dim3(256), 0, st, base, frames, n, seg_target, waves, flags, prm,
                     seg_first, max_size, addr, len, v, count, try_stream ? 1 : 0);
  return hipGetLastError();
}
hipError_t launch_frame_stream(const uint8_t* base, const hf3fs_crc_frame* frames, uint64_t n,
                               const uint32_t* flags, const FrameStreamParams* prm, const uint32_t* seg_first,
                               uint32_t* seg_lin, uint32_t* ev, uint32_t workgroups, const DeviceTables* tabs,
                               hipStream_t st) {
  hipLaunchKernelGGL(k_frame_stream<kPolyCrc32c>, dim3(workgroups), dim3(kThreads), 0, st, base, frames, n, flags,
                     prm, seg_first, seg_lin, ev, &tabs->poly[0], &tabs->fold[0]);
  return hipGetLastError();
}
hipError_t launch_frame_seg_scan(const uint32_t* flags, const FrameStreamParams* prm, const uint32_t* seg_lin,
                                 uint32_t* seg_pre, const DeviceTables* tabs, hipStream_t st) {
  hipLaunchKernelGGL(k_frame_seg_scan<kPolyCrc32c>, dim3(1), dim3(1024), 0, st, flags, prm, seg_lin, seg_pre,
                     &tabs->poly[0]);
  return hipGetLastError();
}
hipError_t launch_frame_finalize(const uint8_t* base, hf3fs_crc_frame* frames, uint64_t n, const uint32_t* v,
                                 const uint32_t* flags, const FrameStreamParams* prm, const uint32_t* ev,
                                 const uint32_t* seg_lin, const uint32_t* seg_pre, uint32_t* count,
                                 const DeviceTables* tabs, hipStream_t st) {
  // <= 1024 workgroups (4 per CU): each loads the 11 KiB of LDS tables once for 4 frames per
  // thread (1 M frames: 256 B frames -7 %, the mix -1..-3 % against 4096 workgroups, 512 and
  // 256 workgroups slower; profiles/r05_f4_clmul_ab.log)
  constexpr unsigned kFinWorkgroups = 1024;
  const unsigned g = grid_of(n);
  hipLaunchKernelGGL(k_frame_finalize<kPolyCrc32c>, dim3(g < kFinWorkgroups ? g : kFinWorkgroups), dim3(256), 0, st, base, frames, n, v, flags,
                     prm, ev, seg_lin, seg_pre, count, &tabs->poly[0], &tabs->sh[0]);
  return hipGetLastError();
}

}  // namespace hf3fs_crc
