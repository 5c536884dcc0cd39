// crc_kernels.hip -- CDNA4 kernels of the chunk-integrity engine (see crc_kernels.h).
#include "crc_device.h"
#include "options.h"

namespace hf3fs_crc {
// Diagnostic builds only (-DHF3FS_CRC_WAVE_STAMPS, scripts/probe_wave_stamps.py): every wave of
// k_crc_ranges writes its wall clock at entry, after the LDS tables, and at exit.
#ifdef HF3FS_CRC_WAVE_STAMPS
__device__ uint64_t g_wave_stamps[4 * 65536];
#define HF3FS_STAMP(k)                                                                            \
  do {                                                                                            \
    if ((threadIdx.x & 63) == 0) g_wave_stamps[4 * (blockIdx.x * kWaves + (threadIdx.x >> 6)) + (k)] = wall_clock64(); \
  } while (0)
#else
#define HF3FS_STAMP(k) \
  do {                 \
  } while (0)
#endif
namespace {

// Bytes of granule w (at 16-aligned g) outside [lo, hi) cleared.
__device__ __forceinline__ uint4 mask16(uint4 w, uint64_t g, uint64_t lo, uint64_t hi) {
  const uint64_t a = lo > g ? lo : g;
  const uint64_t b = hi < g + 16 ? hi : g + 16;
  if (a >= b) return make_uint4(0, 0, 0, 0);
  const int s = (int)(a - g), e = (int)(b - g);
  w.x &= dword_mask(s, e, 0);
  w.y &= dword_mask(s, e, 1);
  w.z &= dword_mask(s, e, 2);
  w.w &= dword_mask(s, e, 3);
  return w;
}

// Whole-buffer geometry of one range: block grid aligned to its END (16 B
// granule), nb blocks from vs.
struct DirectRange {
  uint64_t a0, len, vs, nb;
  __device__ __forceinline__ void set(uint64_t addr, uint64_t l) {
    a0 = addr;
    len = l;
    const uint64_t vend = (a0 + len + 15) & ~uint64_t(15);
    nb = len ? (vend - (a0 & ~uint64_t(15)) + kBlockBytes - 1) / kBlockBytes : 0;
    vs = vend - nb * kBlockBytes;
  }
};

// Whole-buffer tasks on a static stride, software-pipelined ACROSS tasks: the
// next task's descriptor is loaded while this one hashes, and its first U
// blocks (bytes outside the range are masked when they are consumed) while
// this one folds, so a wave of small ranges (KV blocks, serde frames) keeps
// loads in flight through the fold instead of draining at every range.
// Same algebra as the whole-buffer branch of k_crc_ranges.
template <uint32_t POLY, bool NT, class Src>
__device__ __forceinline__ void direct_pipe(const Src& src, uint32_t t, uint32_t ntasks, uint32_t nwaves,
                                            uint32_t* __restrict__ out, const PolyTables* __restrict__ T,
                                            const StepLds& lj, const uint32_t* lc, int lane) {
  constexpr int U = kHashPrefetch;
  const uint64_t lane_off = (uint64_t)lane * 16;
  DirectRange cur;
  uint4 pre[U];
  if (t < ntasks) {
    cur.set(src.addr(t), src.length(t));
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t g = cur.vs + k * kBlockBytes + lane_off;
      pre[k] = k < cur.nb && g < cur.a0 + cur.len && g + 16 > cur.a0 ? gload16s<NT>(g) : make_uint4(0, 0, 0, 0);
    }
  }
  while (t < ntasks) {
    const uint32_t tn = t + nwaves;
    uint64_t naddr = 0, nlen = 0;
    if (tn < ntasks) {
      naddr = src.addr(tn);
      nlen = src.length(tn);
    }
    const uint32_t start = src.start_of(t);
    const uint64_t a0 = cur.a0, len = cur.len, vs = cur.vs, nb = cur.nb, a1 = a0 + len;
    const uint32_t pad = (uint32_t)(((a1 + 15) & ~uint64_t(15)) - a1);
    const bool spill = len && a0 - vs > (uint64_t)(kBlockBytes - 4);
    const bool init = len >= 4 && !spill;
    uint32_t col = 0;
    Streams st;
    if (len) {
      col = lane < 32 ? T->xneg8_cols[pad][lane] : 0u;
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if ((uint64_t)k < nb) {  // wave-uniform
          uint4 w = pre[k];
          const uint64_t g = vs + k * kBlockBytes + lane_off;
          if (k == 0 || (uint64_t)k + 1 == nb) w = mask16(w, g, a0, a1);
          if (k == 0 && init) {  // start xor-ed into data bytes a0..a0+3
            const int o = (int)(a0 - vs) - 16 * lane;
#define HF3FS_INIT_XOR(F, D)                                                             \
  {                                                                                      \
    const int sh = o - 4 * (D);                                                          \
    if (sh > -4 && sh < 4) w.F ^= sh >= 0 ? start << (8 * sh) : start >> (-8 * sh);      \
  }
            HF3FS_INIT_XOR(x, 0)
            HF3FS_INIT_XOR(y, 1)
            HF3FS_INIT_XOR(z, 2)
            HF3FS_INIT_XOR(w, 3)
#undef HF3FS_INIT_XOR
          }
          st.step(w, lj);
        }
      }
      if (nb > (uint64_t)U) st = hash_grid<false, NT>(vs + U * kBlockBytes, nb - U, a0, a1, 0u, lj, lane, st);
    }
    // the next task's head: in flight during this task's fold
    if (tn < ntasks) {
      cur.set(naddr, nlen);
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t g = cur.vs + k * kBlockBytes + lane_off;
        pre[k] = k < cur.nb && g < cur.a0 + cur.len && g + 16 > cur.a0 ? gload16s<NT>(g) : make_uint4(0, 0, 0, 0);
      }
    }
    uint32_t r = start;  // create(type, buf, 0, start) == {type, start}
    if (len) {
      r = __builtin_amdgcn_readfirstlane(fold_streams(st, lc, lane));
      if (pad) {  // r * x^(-8 pad), lane-parallel as in k_crc_ranges
        uint32_t v = ((r >> (31 - (lane & 31))) & 1u) ? col : 0u;
#pragma unroll
        for (int d = 16; d > 0; d >>= 1) v ^= __shfl_xor(v, d, 64);
        r = __builtin_amdgcn_readfirstlane(v);
      }
      if (len < 4) {
        r ^= gf_mul(start, T->xpos8[len], POLY);
      } else if (spill) {
        const uint32_t f = xpow_pair<POLY>(8 * (int64_t)len, 8 * (int64_t)len, lane, T);
        r ^= gf_mul(start, __builtin_amdgcn_readlane(f, 0), POLY);
      }
    }
    if (lane == 0) out[t] = r;
    t = tn;
  }
}

// Whole-range tasks [t, tend) of one wave (byte-balanced runs, k_bal_assign) as ONE
// block stream: a producer walks the tasks' end-aligned block grids (the same grids as
// the whole-buffer branch of k_crc_ranges) and keeps U blocks in flight, across task
// ends; a consumer U blocks behind steps the streams and, at each task's last block,
// folds them and writes the task's value while the next task's blocks are already in
// flight -- no drain at every task end (KV blocks of 4-64 KiB).  Both
// walk the same task sequence, so no per-block metadata travels with the data.
// Loads are unconditional (edge-block addresses clamped into the range's granules) and
// edge blocks are byte-masked when consumed.
struct RangeGeo {
  uint64_t a0, a1, vs;
  uint32_t nb, i;
};
template <class Src>
__device__ __forceinline__ bool range_geo(const Src& src, uint32_t i, RangeGeo& g) {
  const uint64_t len = src.length(i);
  if (!len) return false;
  g.a0 = src.addr(i);
  g.a1 = g.a0 + len;
  const uint64_t vend = (g.a1 + 15) & ~uint64_t(15);
  g.nb = (uint32_t)((vend - (g.a0 & ~uint64_t(15)) + kBlockBytes - 1) / kBlockBytes);
  g.vs = vend - (uint64_t)g.nb * kBlockBytes;
  g.i = i;
  return true;
}

template <uint32_t POLY, bool NT, class Src>
__global__ __launch_bounds__(kThreads) void k_crc_range_stream(Src src, uint32_t* __restrict__ out,
                                                               const PolyTables* __restrict__ T,
                                                               const uint32_t* __restrict__ bal) {
  __shared__ uint32_t lds[kLdsWords + kFoldLdsWords];
  fill_lds_fold<POLY>(lds, T);
  constexpr int U = kHashPrefetch;
  const int lane = threadIdx.x & 63;
  const StepLds lj = step_lds(lds, lane);
  const uint32_t* lc = lds + kLdsWords;
  const uint64_t lane_off = (uint64_t)lane * 16;
  const uint32_t w = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t t0 = __builtin_amdgcn_readfirstlane(bal[w]), tend = __builtin_amdgcn_readfirstlane(bal[w + 1]);
  // producer: the next block to load; empty tasks it passes get their value here
  uint32_t pi = t0, pk = 0;
  RangeGeo pg{}, last{};
  bool pdone = true;
  for (; pi < tend; ++pi) {
    if (range_geo(src, pi, pg)) {
      pdone = false;
      break;
    }
    if (lane == 0) out[pi] = src.start_of(pi);  // create(type, buf, 0, start) == {type, start}
  }
  if (pdone) return;  // no bytes in this wave's run (after fill_lds: no barrier follows)
  // Always one load (past the run's end: the last task's first granules again, never
  // consumed): no branch around a load, whose join would wait for every load in flight.
  auto produce = [&]() -> uint4 {
    const uint64_t glo = pg.a0 & ~uint64_t(15), ghi = (pg.a1 - 1) & ~uint64_t(15);
    uint64_t g = pg.vs + (uint64_t)pk * kBlockBytes + lane_off;
    g = g < glo ? glo : (g > ghi ? ghi : g);  // edge blocks: granules outside the range re-read a valid one
    const uint4 v = gload16s<NT>(g);
    if (pdone) return v;
    if (++pk == pg.nb) {  // next non-empty task
      pk = 0;
      last = pg;
      pdone = true;
      for (++pi; pi < tend; ++pi) {
        if (range_geo(src, pi, pg)) {
          pdone = false;
          break;
        }
        if (lane == 0) out[pi] = src.start_of(pi);
      }
    }
    if (pdone) pg = last;  // keep a valid address for the loads past the end
    return v;
  };
  // consumer: the task being hashed
  uint32_t ck = 0;
  RangeGeo cg{};
  bool cdone = true;
  for (uint32_t i = t0; i < tend; ++i)
    if (range_geo(src, i, cg)) {
      cdone = false;
      break;
    }
  uint32_t cstart = 0, cpad = 0, ccol = 0;
  bool cinit = false, cspill = false;
  auto begin_task = [&]() {
    const uint64_t len = cg.a1 - cg.a0, vend = cg.vs + (uint64_t)cg.nb * kBlockBytes;
    cstart = src.start_of(cg.i);
    cpad = (uint32_t)(vend - cg.a1);
    cspill = cg.a0 - cg.vs > (uint64_t)(kBlockBytes - 4);
    cinit = len >= 4 && !cspill;
    ccol = cpad && lane < 32 ? T->xneg8_cols[cpad][lane] : 0u;
  };
  if (!cdone) begin_task();
  Streams st;
  uint4 c[U];
#pragma unroll
  for (int q = 0; q < U; ++q) c[q] = produce();
  while (!cdone) {  // wave-uniform
    uint4 nx[U];
#pragma unroll
    for (int q = 0; q < U; ++q) nx[q] = produce();
#pragma unroll
    for (int q = 0; q < U; ++q) {
      if (cdone) break;  // wave-uniform
      uint4 wv = c[q];
      const bool first = ck == 0, last = ck + 1 == cg.nb;
      if (first || last) {
        const uint64_t g = cg.vs + (uint64_t)ck * kBlockBytes + lane_off;
        wv = mask16(wv, g, cg.a0, cg.a1);
        if (first && cinit) {  // start xor-ed into data bytes a0..a0+3
          const int o = (int)(cg.a0 - cg.vs) - 16 * lane;
#define HF3FS_INIT_XOR(F, D)                                                            \
  {                                                                                     \
    const int sh = o - 4 * (D);                                                         \
    if (sh > -4 && sh < 4) wv.F ^= sh >= 0 ? cstart << (8 * sh) : cstart >> (-8 * sh); \
  }
          HF3FS_INIT_XOR(x, 0)
          HF3FS_INIT_XOR(y, 1)
          HF3FS_INIT_XOR(z, 2)
          HF3FS_INIT_XOR(w, 3)
#undef HF3FS_INIT_XOR
        }
      }
      st.step(wv, lj);
      if (!last) {
        ++ck;
        continue;
      }
      // the task's last block: its value (the next task's blocks are in flight)
      const uint64_t len = cg.a1 - cg.a0;
      uint32_t r = __builtin_amdgcn_readfirstlane(fold_streams(st, lc, lane));
      if (cpad) {  // r * x^(-8 pad), lane-parallel
        uint32_t v = ((r >> (31 - (lane & 31))) & 1u) ? ccol : 0u;
#pragma unroll
        for (int d = 16; d > 0; d >>= 1) v ^= __shfl_xor(v, d, 64);
        r = __builtin_amdgcn_readfirstlane(v);
      }
      if (len < 4) {
        r ^= gf_mul(cstart, T->xpos8[len], POLY);
      } else if (cspill) {
        const uint32_t f = xpow_pair<POLY>(8 * (int64_t)len, 8 * (int64_t)len, lane, T);
        r ^= gf_mul(cstart, __builtin_amdgcn_readlane(f, 0), POLY);
      }
      if (lane == 0) out[cg.i] = r;
      st = Streams();
      ck = 0;
      cdone = true;
      for (uint32_t i = cg.i + 1; i < tend; ++i)
        if (range_geo(src, i, cg)) {
          cdone = false;
          break;
        }
      if (!cdone) begin_task();
    }
#pragma unroll
    for (int q = 0; q < U; ++q) c[q] = nx[q];
  }
}

// Start-aligned block grids (segments, byte-run parts) begin at the part's start rounded
// down to kGridAlign bytes; the bytes in front of the part are masked to zero.  128: every
// 1 KiB block of a part covers 8 whole cache lines instead of straddling a 9th (in one
// process, the d3 pre-hash job list as byte runs: 0.6684 ms at 128 vs 0.6826 at 16 and
// 0.6725 at 1024, d2 unchanged; profiles/r04_grid_align_ab.log).
#ifndef HF3FS_CRC_GRID_ALIGN
#define HF3FS_CRC_GRID_ALIGN 128
#endif
constexpr uint64_t kGridAlign = HF3FS_CRC_GRID_ALIGN;
static_assert(kGridAlign >= 16 && kGridAlign <= kBlockBytes && (kGridAlign & (kGridAlign - 1)) == 0, "grid alignment");

// Bytes [so, eo) of range i (start-aligned block grid), shifted to the range's
// end and xor-ed into out[i]; with so == 0 the start term start * x^(8 len)
// too: raw(buf, start) = start * x^(8 len) ^ xor of the parts.
template <uint32_t POLY, bool NT, class Src>
__device__ __forceinline__ void hash_part(const Src& src, uint32_t i, uint64_t len, uint64_t so, uint64_t eo,
                                          uint32_t* __restrict__ out, const PolyTables* __restrict__ T,
                                          const StepLds& lj, const uint32_t* lc, int lane) {
  const uint64_t base = src.addr(i);
  const uint64_t a0 = base + so, a1 = base + eo;
  const uint64_t vs = a0 & ~uint64_t(kGridAlign - 1);  // bytes before a0 are masked to zero (lin ignores them)
  const uint64_t nb = (a1 - vs + kBlockBytes - 1) / kBlockBytes;
  const uint64_t vend = vs + nb * kBlockBytes;
  const Streams st = hash_grid<false, NT>(vs, nb, a0, a1, 0u, lj, lane);
  const uint32_t v = fold_streams(st, lc, lane);  // lin(part) * x^(8(vend - a1))
  const int64_t ebits = 8 * (int64_t)(base + len - vend);
  const uint32_t f = xpow_pair<POLY>(ebits, 8 * (int64_t)len, lane, T);
  const uint32_t pa = __builtin_amdgcn_readlane(f, 0);
  const uint32_t pb = __builtin_amdgcn_readlane(f, 32);
  const uint32_t vv = __builtin_amdgcn_readfirstlane(v);
  uint32_t val = gf_mul(vv, pa, POLY);
  if (so == 0) val ^= gf_mul(src.start_of(i), pb, POLY);
  if (lane == 0) atomicXor(out + i, val);
}

// (readfirstlane returns int: each half goes through uint32_t, or a low word with bit 31
// set would sign-extend over the high word -- a byte-run offset >= 2 GiB faulted that way)
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32);
}

// Wave w's byte run: from byte boff[w] of range bal[w] up to byte boff[w + 1]
// of range bal[w + 1].  bal[] points at non-empty ranges (or n), so each empty
// range lies in exactly one run, whose wave adds its start term; a non-empty
// range's parts partition it, and the part at offset 0 adds the start term.
template <uint32_t POLY, bool NT, class Src>
__device__ __forceinline__ void byte_run(const Src& src, uint32_t w, const uint32_t* __restrict__ bal,
                                         const uint64_t* __restrict__ boff, uint32_t* __restrict__ out,
                                         const PolyTables* __restrict__ T, const StepLds& lj, const uint32_t* lc,
                                         int lane) {
  const uint32_t n = (uint32_t)src.n;
  const uint32_t iend = __builtin_amdgcn_readfirstlane(bal[w + 1]);
  const uint64_t eo_last = rfl64(boff[w + 1]);
  uint64_t so = rfl64(boff[w]);
  for (uint32_t i = __builtin_amdgcn_readfirstlane(bal[w]); i <= iend && i < n; ++i, so = 0) {
    const uint64_t len = src.length(i);
    const uint64_t eo = i == iend ? eo_last : len;
    if (i == iend && eo == 0) break;  // the next run's range
    if (len == 0) {  // create(type, buf, 0, start) == {type, start}
      if (lane == 0) atomicXor(out + i, src.start_of(i));
      continue;
    }
    if (so < eo) hash_part<POLY, NT>(src, i, len, so, eo, out, T, lj, lc, lane);
  }
}

// Persistent kernel over the (segment, range) task grid, segment-major
// (task t -> range t % n, segment t / n) so that empty trailing segments of
// short ranges cluster at the end.  Wave w starts with task w; further tasks
// come from a per-launch ticket counter (`queue`, zeroed before the launch)
// so ragged batches balance dynamically; with queue == nullptr the grid is
// strided statically.  A task hashes its segment and xors
//   lin(segment) * x^(8 * bytes after it)  [ ^ start * x^(8 len) for seg 0 ]
// into out[i]  (raw(buf, start) = start * x^(8 len) ^ lin(buf)).
template <uint32_t POLY, bool DIRECT, bool NT, class Src>
__global__ __launch_bounds__(kThreads) void k_crc_ranges(Src src, uint32_t segs, uint64_t seg_bytes,
                                                         uint32_t* __restrict__ out,
                                                         const PolyTables* __restrict__ T,
                                                         uint32_t* __restrict__ queue,
                                                         const uint32_t* __restrict__ dyn_max, uint64_t pipe_max,
                                                         const uint32_t* __restrict__ skip,
                                                         const uint32_t* __restrict__ bal,
                                                         const uint64_t* __restrict__ boff, uint32_t run_rep) {
  __shared__ uint32_t lds[kLdsWords + kFoldLdsWords];
  // another path took the batch (serde frames on the stream path)
  if (skip && __builtin_amdgcn_readfirstlane(*skip)) return;
  HF3FS_STAMP(0);
  const int lane = threadIdx.x & 63;
  const StepLds lj = step_lds(lds, lane);
  const uint32_t* lc = lds + kLdsWords;
  const uint32_t n = (uint32_t)src.n;
  uint64_t len_bound = seg_bytes;  // every range fits one task when segs == 1
  if (dyn_max) {  // longest range known only on the device (update jobs): no empty segments
    const uint32_t m = __builtin_amdgcn_readfirstlane(*dyn_max);
    len_bound = m;
    if (m == 0) {  // every range is empty: create(type, buf, 0, start) == start, nothing to hash
      for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        atomicXor(out + i, src.start_of(i));
      return;
    }
    segs = m > seg_bytes ? (uint32_t)((m + seg_bytes - 1) / seg_bytes) : 1u;
  }
  if (boff) {  // byte runs (k_bal_assign): ranges split at exact byte shares of the batch
    fill_lds_fold<POLY>(lds, T);
    const uint32_t w0 = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t k = 0; k < run_rep; ++k)  // runs w, w + W, ...: the waves sweep the batch in windows
      byte_run<POLY, NT>(src, w0 + k * gridDim.x * kWaves, bal, boff, out, T, lj, lc, lane);
    return;
  }
  // Whole-buffer tasks also when the device-side length bound leaves one
  // segment per range (record jobs of small frames / reads / blocks): no
  // x^(8e) butterfly and no atomic per range.
  const bool direct = DIRECT || segs == 1;
  fill_lds_fold<POLY>(lds, T);
  HF3FS_STAMP(1);
  const uint32_t ntasks = n * segs;
  const uint32_t nwaves = gridDim.x * kWaves;
  // Tickets only pay for ragged, moderately sized task sets: one counter word
  // serves ~88 dequeues/us (MI355X_MICROARCH.md "dequeue"), so with >16 tasks
  // per wave a static stride balances by averaging instead.
  if (ntasks <= nwaves || ntasks > 16u * nwaves) queue = nullptr;
  uint32_t t = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // byte-balanced static assignment (k_bal_assign): wave w takes the contiguous
  // tasks [bal[w], bal[w + 1]) instead of the stride w, w + nwaves, ...
  uint32_t tend = ntasks, tstep = nwaves;
  if (bal && !queue) {
    const uint32_t w = t;
    t = __builtin_amdgcn_readfirstlane(bal[w]);
    tend = __builtin_amdgcn_readfirstlane(bal[w + 1]);
    tstep = 1;
  } else if (direct && !queue && len_bound <= pipe_max) {  // segs == 1: task t is range t
    direct_pipe<POLY, NT>(src, t, ntasks, nwaves, out, T, lj, lc, lane);
    HF3FS_STAMP(2);
    return;
  }
  while (t < tend) {
    const uint32_t seg = segs == 1 ? 0u : t / n;
    const uint32_t i = t - seg * n;
    const uint64_t len = src.length(i);
    const uint64_t addr_i = src.addr(i);  // with the length: one round trip for the descriptor, not two
    const uint64_t tb = (uint64_t)seg * seg_bytes;
    if (seg == 0 || tb < len) {
      if (len == 0) {  // create(type, buf, 0, start) == {type, start}
        if (lane == 0) {
          if (direct)
            out[i] = src.start_of(i);
          else
            atomicXor(out + i, src.start_of(i));
        }
      } else if (direct) {
        // whole buffer in one task: block grid aligned to the buffer END (16 B
        // granule), so an aligned buffer needs neither masking nor a final
        // shift; the start value is xor-ed into the first four data bytes.
        const uint64_t a0 = addr_i, a1 = a0 + len;
        const uint64_t vend = (a1 + 15) & ~uint64_t(15);
        const uint64_t nb = (vend - (a0 & ~uint64_t(15)) + kBlockBytes - 1) / kBlockBytes;
        const uint64_t vs = vend - nb * kBlockBytes;
        const uint32_t start = src.start_of(i);
        // The start xor needs data bytes a0..a0+3 inside block 0; when they
        // straddle into block 1 (a0 in the block's last 3 bytes) the start
        // term start * x^(8 len) is added explicitly instead.
        const bool spill = a0 - vs > (uint64_t)(kBlockBytes - 4);
        // lin * x^(-8 pad) for an unaligned end, lane-parallel: lane i < 32
        // holds x^(-8 pad) * x^i, loaded now and used after the hash
        const uint32_t pad = (uint32_t)(vend - a1);
        uint32_t col = 0;  // no load per task for buffers ending on a granule (KV blocks)
        if (pad) col = lane < 32 ? T->xneg8_cols[pad][lane] : 0u;
        const Streams st = len >= 4 && !spill ? hash_grid<true, NT>(vs, nb, a0, a1, start, lj, lane)
                                              : hash_grid<false, NT>(vs, nb, a0, a1, start, lj, lane);
        uint32_t r = __builtin_amdgcn_readfirstlane(fold_streams(st, lc, lane));
        if (pad) {  // r * x^(-8 pad) = xor of x^(-8 pad) x^i over the bits (31 - i) of r
          uint32_t v = ((r >> (31 - (lane & 31))) & 1u) ? col : 0u;
#pragma unroll
          for (int d = 16; d > 0; d >>= 1) v ^= __shfl_xor(v, d, 64);
          r = __builtin_amdgcn_readfirstlane(v);
        }
        if (len < 4) {
          r ^= gf_mul(start, T->xpos8[len], POLY);
        } else if (spill) {  // wave-uniform branch: the butterfly needs every lane
          const uint32_t f = xpow_pair<POLY>(8 * (int64_t)len, 8 * (int64_t)len, lane, T);
          r ^= gf_mul(start, __builtin_amdgcn_readlane(f, 0), POLY);
        }
        if (lane == 0) out[i] = r;
      } else {
        const uint64_t te = len < tb + seg_bytes ? len : tb + seg_bytes;
        const uint64_t base = addr_i;
        const uint64_t a0 = base + tb, a1 = base + te;
        const uint64_t vs = a0 & ~uint64_t(kGridAlign - 1);
        const uint64_t nb = (a1 - vs + kBlockBytes - 1) / kBlockBytes;
        const uint64_t vend = vs + nb * kBlockBytes;
        const Streams st = hash_grid<false, NT>(vs, nb, a0, a1, 0u, lj, lane);
        const uint32_t v = fold_streams(st, lc, lane);  // lin(segment) * x^(8(vend - a1))
        const int64_t ebits = 8 * (int64_t)(base + len - vend);
        const uint32_t f = xpow_pair<POLY>(ebits, 8 * (int64_t)len, lane, T);
        const uint32_t pa = __builtin_amdgcn_readlane(f, 0);
        const uint32_t pb = __builtin_amdgcn_readlane(f, 32);
        const uint32_t vv = __builtin_amdgcn_readfirstlane(v);
        uint32_t val = gf_mul(vv, pa, POLY);
        if (seg == 0) val ^= gf_mul(src.start_of(i), pb, POLY);
        if (lane == 0) atomicXor(out + i, val);
      }
    }
    if (queue) {
      uint32_t ticket = 0;
      if (lane == 0) ticket = atomicAdd(queue, 1u);
      t = nwaves + __builtin_amdgcn_readfirstlane(ticket);
    } else {
      t += tstep;
    }
  }
  HF3FS_STAMP(2);
}

template <uint32_t POLY, bool DIRECT, bool NT, class Src>
void launch_one(const Src& src, const Plan& p, uint32_t* out, const PolyTables* T, hipStream_t s) {
  hipLaunchKernelGGL((k_crc_ranges<POLY, DIRECT, NT, Src>), dim3(p.grid), dim3(kThreads), 0, s, src,
                     (uint32_t)p.segs, p.seg_bytes, out, T, p.queue, p.dyn_max, p.pipe_max, p.skip, p.bal, p.boff,
                     p.run_rep);
}

template <uint32_t POLY, class Src>
void launch_poly(const Src& src, const Plan& p, uint32_t* out, const PolyTables* T, hipStream_t s) {
  // byte-balanced whole-range tasks as one block stream per wave (option range_stream)
  if (p.range_stream && p.bal && !p.boff && !p.queue && p.segs == 1 && !p.dyn_max) {
    if (p.nt)
      hipLaunchKernelGGL((k_crc_range_stream<POLY, true, Src>), dim3(p.grid), dim3(kThreads), 0, s, src, out, T, p.bal);
    else
      hipLaunchKernelGGL((k_crc_range_stream<POLY, false, Src>), dim3(p.grid), dim3(kThreads), 0, s, src, out, T, p.bal);
    return;
  }
  // One segment per range on the host's length bound: whole-buffer tasks.  With a
  // device-side bound (record jobs) too, since it never exceeds the host's
  // (option record_direct = 0: the runtime-direct instantiation, A/B).
  const bool rec_direct = options().record_direct.load() != 0;
  const bool direct = p.segs == 1 && (!p.dyn_max || rec_direct);
  if (direct)
    p.nt ? launch_one<POLY, true, true>(src, p, out, T, s) : launch_one<POLY, true, false>(src, p, out, T, s);
  else
    p.nt ? launch_one<POLY, false, true>(src, p, out, T, s) : launch_one<POLY, false, false>(src, p, out, T, s);
}

template <class Src>
hipError_t launch_ranges(uint8_t type, const Src& src, const Plan& p, uint32_t* out, const DeviceTables* tabs,
                         hipStream_t s) {
  if (type == kTypeCrc32)
    launch_poly<kPolyCrc32>(src, p, out, &tabs->poly[1], s);
  else
    launch_poly<kPolyCrc32c>(src, p, out, &tabs->poly[0], s);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Persistent request service.  Workgroup w serves tickets w, w + W, w + 2W
// ... (W = gridDim.x): wave 0 polls the slot of its next ticket until the
// host publishes it (system-scope acquire of the slot's seq), the request is
// split over the 16 waves in 1 KiB aligned segments (start-aligned grids,
// shifted to the request end by x^(8e)), the partial values are xor-ed in
// LDS and thread 0 publishes value + done with a system-scope release.
// Every wave leaves through the same barrier-broadcast command, on `stop` or
// after idle_ticks of wall clock without a request, so the grid always
// drains; the next ticket of each workgroup persists in device memory for
// the relaunch.
template <uint32_t POLY>
__global__ __launch_bounds__(kThreads) void k_crc_service(ServiceArgs a, const PolyTables* __restrict__ T) {
  __shared__ uint32_t lds[kLdsWords + kFoldLdsWords];
  __shared__ uint64_t s_addr, s_len;
  __shared__ uint32_t s_start, s_cmd;
  __shared__ uint32_t s_part[kWaves];
  fill_lds_fold<POLY>(lds, T);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const StepLds lj = step_lds(lds, lane);
  const uint32_t* lc = lds + kLdsWords;
  const uint32_t mask = a.ring - 1;
  uint32_t ticket = __builtin_amdgcn_readfirstlane(a.next[blockIdx.x]);
  for (;;) {
    // Wave 0 polls with wave-uniform control flow (readfirstlane broadcasts
    // lane-uniform loads): a loop that only thread 0 ran, in front of the
    // barrier, would let the compiler's structurizer send wave 0's other
    // lanes through the barrier loop without lane 0 and desynchronise the
    // workgroup's barriers.
    if (wave == 0) {
      uint32_t cmd = 2;
      const long long idle_from = wall_clock64();
      uint32_t backoff = 1;
      uint32_t seq = 0;
      const ServiceReq* r = a.req + (ticket & mask);
      for (;;) {
        seq = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&r->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM));
        if (seq == ticket + 1) {  // published
          if (lane == 0) {
            s_addr = __hip_atomic_load(&r->addr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            s_len = __hip_atomic_load(&r->len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            s_start = __hip_atomic_load(&r->start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
          cmd = 1;
          break;
        }
        if (__builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&a.ctrl->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))) {
          cmd = 3;
          break;
        }
        if ((uint64_t)(wall_clock64() - idle_from) > a.idle_ticks) break;
        // back off while idle (polls cross PCIe), capped at ~4 us of sleep
        for (uint32_t k = 0; k < backoff; ++k) __builtin_amdgcn_s_sleep(16);
        if (backoff < 8) backoff <<= 1;
      }
      if (lane == 0) {
        if (cmd != 1) {
          a.next[blockIdx.x] = ticket;  // resume here after a relaunch
          // diagnostics for the host (coalescer service_dump)
          __hip_atomic_store(&a.ctrl->dbg_seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(&a.ctrl->dbg_ticket, ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(&a.ctrl->dbg_exit, cmd, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        s_cmd = cmd;
      }
    }
    __syncthreads();
    if (s_cmd != 1) break;
    const uint32_t r = wg_hash<POLY>(s_addr, s_len, s_start, lj, lc, T, s_part);
    if (threadIdx.x == 0) {
      ServiceResp* o = a.resp + (ticket & mask);
      __hip_atomic_store(&o->value, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&o->done, ticket + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    ticket += gridDim.x;
  }
}

// ---------------------------------------------------------------------------
__global__ void k_compare(const uint32_t* __restrict__ computed, const uint32_t* __restrict__ expected,
                          uint8_t* __restrict__ mismatch, uint32_t* __restrict__ count, uint64_t n) {
  uint32_t local = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t bad = computed[i] != expected[i];
    mismatch[i] = bad;
    local += bad;
  }
  // wave-aggregate then one atomic per wave
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) local += __shfl_xor(local, d, 64);
  if ((threadIdx.x & 63) == 0 && local) atomicAdd(count, local);
}

// ChecksumInfo::combine element-wise: acc = (~acc) * x^(8 len2) ^ crc2.  x^(8 len2) from the
// byte-digit power tables and every product through gf_mul_dw, both table sets in LDS
// (9 KiB per workgroup, <= 2048 workgroups).
template <uint32_t POLY>
__global__ __launch_bounds__(256) void k_combine(uint32_t* __restrict__ acc, const uint32_t* __restrict__ crc2,
                                                 const uint64_t* __restrict__ len2, uint64_t n,
                                                 const PolyTables* __restrict__ T, const ShortTables* __restrict__ S) {
  __shared__ uint32_t dw[4 * 256], pw[kPowDigits * 256];
  for (int k = threadIdx.x; k < 4 * 256; k += blockDim.x) dw[k] = (&S->dw[0][0])[k];
  for (int k = threadIdx.x; k < kPowDigits * 256; k += blockDim.x) pw[k] = (&T->pow8b[0][0])[k];
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t m = len2[i];
    if (m == 0) continue;
    uint32_t x = kOne;
    bool first = true;
    for (int j = 0; j < kPowDigits && m; ++j, m >>= 8) {  // as xpow8_bytes, n > 0
      const uint32_t d = (uint32_t)(m & 0xffu);
      if (!d) continue;
      x = first ? pw[256 * j + d] : gf_mul_dw(x, pw[256 * j + d], dw);
      first = false;
    }
    for (int k = 8 * kPowDigits + 3; m; ++k, m >>= 1)  // (lengths >= 2^61 square x^(2^63) on)
      if (m & 1) x = gf_mul_dw(x, xpow2k(T->xpow, k, POLY), dw);
    acc[i] = gf_mul_dw(~acc[i], x, dw) ^ crc2[i];
  }
}

// Byte-balanced static assignment of whole-range tasks (segs == 1) to waves:
// bal[k] = the first task i whose byte prefix P_i = sum_{j<i} len_j reaches
// X_k = ceil(k * total / nw), bal[0] = 0, bal[nw] = n.  Two passes: chunk sums,
// then a block scan of each chunk that places the boundaries falling in it.
constexpr int kBalThreads = 256;

template <class Src>
__global__ __launch_bounds__(kBalThreads) void k_bal_sums(Src src, uint64_t n, uint64_t chunk,
                                                        uint64_t* __restrict__ partial) {
  __shared__ uint64_t red[kBalThreads / 64];
  const uint64_t c0 = (uint64_t)blockIdx.x * chunk, c1 = c0 + chunk < n ? c0 + chunk : n;
  uint64_t v = 0;
  for (uint64_t i = c0 + threadIdx.x; i < c1; i += kBalThreads) v += src.length(i);
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < kBalThreads / 64; ++w) t += red[w];
    partial[blockIdx.x] = t;
  }
}

template <class Src>
__global__ __launch_bounds__(kBalThreads) void k_bal_assign(Src src, uint64_t n, uint64_t chunk, uint32_t nblocks,
                                                          const uint64_t* __restrict__ partial, uint32_t nw,
                                                          uint32_t* __restrict__ bal, uint64_t* __restrict__ boff) {
  __shared__ uint64_t sa[kBalThreads], sb[kBalThreads];
  const uint32_t tid = threadIdx.x;
  uint64_t before = 0, total = 0;  // bytes of the chunks before this one, of all chunks
  for (uint32_t b = tid; b < nblocks; b += kBalThreads) {
    const uint64_t v = partial[b];
    total += v;
    if (b < blockIdx.x) before += v;
  }
  sa[tid] = before;
  sb[tid] = total;
  __syncthreads();
  for (uint32_t d = kBalThreads / 2; d > 0; d >>= 1) {
    if (tid < d) {
      sa[tid] += sa[tid + d];
      sb[tid] += sb[tid + d];
    }
    __syncthreads();
  }
  before = sa[0];
  total = sb[0];
  __syncthreads();
  if (blockIdx.x == 0 && tid == 0) {
    bal[0] = 0;
    bal[nw] = (uint32_t)n;
    if (boff) boff[0] = boff[nw] = 0;
  }
  if (total == 0) {  // every range empty: split by count
    for (uint64_t k = (uint64_t)blockIdx.x * kBalThreads + tid + 1; k < nw; k += (uint64_t)gridDim.x * kBalThreads) {
      bal[k] = (uint32_t)(k * n / nw);
      if (boff) boff[k] = 0;
    }
    return;
  }
  // this thread's run of the chunk and its bytes; exclusive scan over the block
  const uint64_t c0 = (uint64_t)blockIdx.x * chunk, c1 = c0 + chunk < n ? c0 + chunk : n;
  const uint64_t sub = (chunk + kBalThreads - 1) / kBalThreads;
  const uint64_t r0 = c0 + tid * sub < c1 ? c0 + tid * sub : c1, r1 = r0 + sub < c1 ? r0 + sub : c1;
  uint64_t mine = 0;
  for (uint64_t i = r0; i < r1; ++i) mine += src.length(i);
  sa[tid] = mine;
  __syncthreads();
  for (uint32_t d = 1; d < kBalThreads; d <<= 1) {  // inclusive Hillis-Steele scan
    const uint64_t add = tid >= d ? sa[tid - d] : 0;
    __syncthreads();
    sa[tid] += add;
    __syncthreads();
  }
  uint64_t P = before + sa[tid] - mine;  // bytes before task r0
  // X_k = ceil(k T / nw) stepped without a division per boundary (a 64-bit division is a
  // ~100-instruction routine; one thread placing thousands of boundaries in one long range
  // spent 0.9 ms on them): T = q nw + rem, X_k = k q + ceil(k rem / nw), acc = k rem mod nw.
  const uint64_t q = total / nw, rem = total % nw;
  uint64_t acc = 0, X = 0;
  auto seek = [&](uint64_t k) {
    acc = (k * rem) % nw;
    X = k * q + (k * rem) / nw + (acc ? 1 : 0);
  };
  auto next = [&]() {  // k -> k + 1
    const uint64_t c0 = acc ? 1 : 0;
    acc += rem;
    uint64_t c = 0;
    if (acc >= nw) {
      acc -= nw;
      c = 1;
    }
    X += q + c - c0 + (acc ? 1 : 0);
  };
  if (boff) {  // byte runs: X_k in [P_i, P_i + len_i) -> wave k starts at byte X_k - P_i of range i
    if (blockIdx.x == 0)  // X_k == total (fewer bytes than waves): an empty run at the end
      for (uint64_t k = tid + 1; k < nw; k += kBalThreads)
        if ((k * total + nw - 1) / nw >= total) {
          bal[k] = (uint32_t)n;
          boff[k] = 0;
        }
    // first boundary k >= 1 with X_k >= P: ceil(k T / nw) >= P  <=>  k > (P - 1) nw / T
    uint64_t k = P ? (P - 1) * nw / total + 1 : 1;
    seek(k);
    for (uint64_t i = r0; i < r1 && k < nw; ++i) {
      const uint64_t li = src.length(i);
      while (k < nw && X < P + li) {
        bal[k] = (uint32_t)i;
        boff[k] = X - P;
        ++k;
        next();
      }
      P += li;
    }
    return;
  }
  // first boundary k >= 1 with X_k > P
  uint64_t k = P * nw / total + 1;
  seek(k);
  for (uint64_t i = r0; i < r1 && k < nw; ++i) {
    P += src.length(i);
    while (k < nw && X <= P) {  // X_k in (P_i, P_{i+1}]: wave k starts after task i
      bal[k] = (uint32_t)(i + 1);
      ++k;
      next();
    }
  }
}

__global__ void k_fill_words(uint32_t* __restrict__ p, uint64_t n, uint32_t v) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_fill_synth(uint8_t* __restrict__ dst, uint64_t stride, uint64_t chunk_len, uint64_t n_chunks,
                             uint64_t seed, uint64_t first_chunk_id) {
  const uint64_t wpc = (chunk_len + 7) / 8;
  const uint64_t total = wpc * n_chunks;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t c = t / wpc, w = t - c * wpc;
    const uint64_t v = splitmix64(seed ^ ((first_chunk_id + c) << 32) ^ w);
    uint8_t* p = dst + c * stride + w * 8;
    if (w * 8 + 8 <= chunk_len) {
      *reinterpret_cast<uint64_t*>(p) = v;
    } else {
      for (uint64_t k = 0; w * 8 + k < chunk_len; ++k) p[k] = (uint8_t)(v >> (8 * k));
    }
  }
}

}  // namespace

hipError_t launch_ranges_strided(uint8_t type, const StridedSource& src, const Plan& p, uint32_t* out,
                                 const DeviceTables* tabs, hipStream_t s) {
  return launch_ranges(type, src, p, out, tabs, s);
}
hipError_t launch_ranges_list(uint8_t type, const ListSource& src, const Plan& p, uint32_t* out,
                              const DeviceTables* tabs, hipStream_t s) {
  return launch_ranges(type, src, p, out, tabs, s);
}
hipError_t launch_ranges_arena(uint8_t type, const ArenaSource& src, const Plan& p, uint32_t* out,
                               const DeviceTables* tabs, hipStream_t s) {
  return launch_ranges(type, src, p, out, tabs, s);
}

template <class Src>
hipError_t launch_balance_t(const Src& src, uint64_t n, uint32_t nw, uint64_t* partial, uint32_t nblocks,
                            uint32_t* bal, hipStream_t s, uint64_t* boff) {
  const uint64_t chunk = (n + nblocks - 1) / nblocks;
  hipLaunchKernelGGL(k_bal_sums<Src>, dim3(nblocks), dim3(kBalThreads), 0, s, src, n, chunk, partial);
  hipLaunchKernelGGL(k_bal_assign<Src>, dim3(nblocks), dim3(kBalThreads), 0, s, src, n, chunk, nblocks, partial, nw,
                     bal, boff);
  return hipGetLastError();
}
hipError_t launch_balance(const ArenaSource& src, uint64_t n, uint32_t nw, uint64_t* partial, uint32_t nblocks,
                          uint32_t* bal, hipStream_t s, uint64_t* boff) {
  return launch_balance_t(src, n, nw, partial, nblocks, bal, s, boff);
}
hipError_t launch_balance(const ListSource& src, uint64_t n, uint32_t nw, uint64_t* partial, uint32_t nblocks,
                          uint32_t* bal, hipStream_t s, uint64_t* boff) {
  return launch_balance_t(src, n, nw, partial, nblocks, bal, s, boff);
}

// Byte runs of n equal ranges of len > 0 bytes over nw waves, in closed form (k_bal_assign's
// boff form for uniform lengths): X_k = ceil(k n len / nw), bal[k] = X_k / len, boff[k] =
// X_k % len; X_k == n len (fewer bytes than waves) is the empty run at the end.
__global__ void k_runs_uniform(uint64_t n, uint64_t len, uint32_t nw, uint32_t* __restrict__ bal,
                               uint64_t* __restrict__ boff) {
  const uint64_t T = n * len;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k <= nw; k += gridDim.x * blockDim.x) {
    const uint64_t X = ((uint64_t)k * T + nw - 1) / nw;
    const bool end = k == nw || X >= T;
    bal[k] = end ? (uint32_t)n : (uint32_t)(X / len);
    boff[k] = end ? 0 : X % len;
  }
}

hipError_t launch_runs_uniform(uint64_t n, uint64_t len, uint32_t nw, uint32_t* bal, uint64_t* boff, hipStream_t s) {
  hipLaunchKernelGGL(k_runs_uniform, dim3((nw + 256) / 256), dim3(256), 0, s, n, len, nw, bal, boff);
  return hipGetLastError();
}

hipError_t launch_service(const ServiceArgs& a, uint32_t workgroups, const DeviceTables* tabs, hipStream_t s) {
  hipLaunchKernelGGL(k_crc_service<kPolyCrc32c>, dim3(workgroups), dim3(kThreads), 0, s, a, &tabs->poly[0]);
  return hipGetLastError();
}

hipError_t launch_compare(const uint32_t* computed, const uint32_t* expected, uint8_t* mismatch, uint32_t* count,
                          uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t want = (n + 255) / 256;
  const unsigned grid = (unsigned)(want < 4096 ? want : 4096);
  hipLaunchKernelGGL(k_compare, dim3(grid), dim3(256), 0, s, computed, expected, mismatch, count, n);
  return hipGetLastError();
}

hipError_t launch_combine(uint8_t type, uint32_t* acc, const uint32_t* crc2, const uint64_t* len2, uint64_t n,
                          const DeviceTables* tabs, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t want = (n + 255) / 256;
  const unsigned grid = (unsigned)(want < 2048 ? want : 2048);
  if (type == kTypeCrc32)
    hipLaunchKernelGGL(k_combine<kPolyCrc32>, dim3(grid), dim3(256), 0, s, acc, crc2, len2, n, &tabs->poly[1],
                       &tabs->sh[1]);
  else
    hipLaunchKernelGGL(k_combine<kPolyCrc32c>, dim3(grid), dim3(256), 0, s, acc, crc2, len2, n, &tabs->poly[0],
                       &tabs->sh[0]);
  return hipGetLastError();
}

hipError_t launch_fill_words(void* p, uint64_t n_words, uint32_t v, hipStream_t s) {
  if (n_words == 0) return hipSuccess;
  const uint64_t want = (n_words + 255) / 256;
  const unsigned grid = (unsigned)(want < 4096 ? want : 4096);
  hipLaunchKernelGGL(k_fill_words, dim3(grid), dim3(256), 0, s, (uint32_t*)p, n_words, v);
  return hipGetLastError();
}

hipError_t launch_fill_synth(uint8_t* dst, uint64_t stride, uint64_t chunk_len, uint64_t n_chunks, uint64_t seed,
                             uint64_t first_chunk_id, hipStream_t s) {
  const uint64_t total = (chunk_len + 7) / 8 * n_chunks;
  if (total == 0) return hipSuccess;
  const uint64_t want = (total + 255) / 256;
  const unsigned grid = (unsigned)(want < 16384 ? want : 16384);
  hipLaunchKernelGGL(k_fill_synth, dim3(grid), dim3(256), 0, s, dst, stride, chunk_len, n_chunks, seed,
                     first_chunk_id);
  return hipGetLastError();
}

}  // namespace hf3fs_crc

#ifdef HF3FS_CRC_WAVE_STAMPS
extern "C" int hf3fs_crc_debug_wave_stamps(uint64_t* host, uint64_t n, int* khz) {
  if (hipDeviceGetAttribute(khz, hipDeviceAttributeWallClockRate, 0) != hipSuccess) return -1;
  if (n > 4 * 65536) n = 4 * 65536;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(hf3fs_crc::g_wave_stamps), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -1;
}
#endif
