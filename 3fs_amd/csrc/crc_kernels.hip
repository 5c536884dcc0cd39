// crc_kernels.hip -- CDNA4 kernels of the chunk-integrity engine (see crc_kernels.h).
#include "crc_kernels.h"

namespace hf3fs_crc {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;

// global_load_dwordx4 (address space 1, not flat: flat loads would also count
// on lgkmcnt and serialise against the LDS table reads).
__device__ __forceinline__ uint4 gload16(uint64_t addr) {
  const u32x4 v = *reinterpret_cast<g_u32x4*>(addr);
  return make_uint4(v.x, v.y, v.z, v.w);
}
// The streamed body of a range: optionally non-temporal (read-once data).
template <bool NT>
__device__ __forceinline__ uint4 gload16s(uint64_t addr) {
  if (NT) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<g_u32x4*>(addr));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return gload16(addr);
}

// Bytes [lo, hi) of dword `d` (byte positions 4d..4d+3 of a granule) kept.
__device__ __forceinline__ uint32_t dword_mask(int s, int e, int d) {
  int lo = s - 4 * d, hi = e - 4 * d;
  lo = lo < 0 ? 0 : lo;
  hi = hi > 4 ? 4 : hi;
  if (hi <= lo) return 0u;
  uint32_t m = hi == 4 ? 0xffffffffu : ((1u << (8 * hi)) - 1u);
  return m & ~((1u << (8 * lo)) - 1u);
}

// 16-byte granule at g (16-aligned) with only bytes inside [lo, hi) kept.
// The aligned granule never crosses a page, so touching it is safe whenever
// at least one of its bytes belongs to the buffer; fully outside -> no load.
__device__ __forceinline__ uint4 gload16_masked(uint64_t g, uint64_t lo, uint64_t hi) {
  uint64_t a = lo > g ? lo : g;
  uint64_t b = hi < g + 16 ? hi : g + 16;
  if (a >= b) return make_uint4(0, 0, 0, 0);
  uint4 w = gload16(g);
  int s = (int)(a - g), e = (int)(b - g);
  w.x &= dword_mask(s, e, 0);
  w.y &= dword_mask(s, e, 1);
  w.z &= dword_mask(s, e, 2);
  w.w &= dword_mask(s, e, 3);
  return w;
}

// One stream update: (s ^ w) * x^8192 via the lane's private LDS table copy.
__device__ __forceinline__ uint32_t stride_step(uint32_t x, const uint32_t* lj) {
  return lj[(x & 0xffu) << 5] ^ lj[8192 + (((x >> 8) & 0xffu) << 5)] ^ lj[16384 + (((x >> 16) & 0xffu) << 5)] ^
         lj[24576 + ((x >> 24) << 5)];
}

struct Streams {
  uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  __device__ __forceinline__ void step(const uint4& w, const uint32_t* lj) {
    s0 = stride_step(s0 ^ w.x, lj);
    s1 = stride_step(s1 ^ w.y, lj);
    s2 = stride_step(s2 ^ w.z, lj);
    s3 = stride_step(s3 ^ w.w, lj);
  }
};

// LDS image: [0, kLdsWords) the 4 x 256 step table, 32 replicas per entry
// (entry e at words [32e, 32e+32)): lane l reads replica l % 32 -> bank l % 32,
// so the hot loop is bank-conflict free.  [kLdsWords, +kMulcWords) the seven
// constant-multiply tables of the fold (read rarely; not replicated).
__device__ __forceinline__ void fill_lds(uint32_t* lds, const PolyTables* T) {
  const uint32_t* step = &T->step[0][0];
  for (int e = threadIdx.x; e < 1024; e += blockDim.x) {
    const uint32_t v = step[e];
    const uint4 v4 = make_uint4(v, v, v, v);
    uint4* dst = reinterpret_cast<uint4*>(lds + e * kCopies);
#pragma unroll
    for (int c = 0; c < kCopies / 4; ++c) dst[c] = v4;
  }
  const uint4* msrc = reinterpret_cast<const uint4*>(&T->mulc[0][0][0]);
  uint4* mdst = reinterpret_cast<uint4*>(lds + kLdsWords);
  for (int e = threadIdx.x; e < kMulcWords / 4; e += blockDim.x) mdst[e] = msrc[e];
  __syncthreads();
}

// a * C_k with the byte tables of constant C_k (lc = LDS base of table k).
__device__ __forceinline__ uint32_t mulc(uint32_t a, const uint32_t* lc) {
  return lc[a & 0xffu] ^ lc[256 + ((a >> 8) & 0xffu)] ^ lc[512 + ((a >> 16) & 0xffu)] ^ lc[768 + (a >> 24)];
}

// Fold the 256 stream registers of a wave into one value in lane 0:
//   R = sum_{l,d} s_{l,d} * x^(-32 (4l + d))
// (in-lane Horner with C_0 = x^-32, then a shuffle tree with C_{k+1} = x^(-128*2^k)
// applied to the LATER lane of each pair).  Stream (l,d) carries an extra
// x^(32(4l+d)) relative to the block grid's end, so R = lin(grid bytes) exactly.
__device__ __forceinline__ uint32_t fold_streams(const Streams& st, const uint32_t* lc, int lane) {
  uint32_t u = mulc(st.s3, lc) ^ st.s2;
  u = mulc(u, lc) ^ st.s1;
  u = mulc(u, lc) ^ st.s0;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const uint32_t o = __shfl_down(u, 1 << k, 64);
    const uint32_t m = mulc(o, lc + (k + 1) * 1024);
    if ((lane & ((2 << k) - 1)) == 0) u ^= m;
  }
  return u;
}

// Stream nb 1 KiB blocks starting at vs (16-aligned) through the lane
// registers; bytes outside [a0, a1) read as zero (an aligned 16 B granule never
// crosses a page, and fully-outside granules are not loaded).  Block 0 holds a0.
// INIT: xor `start` into data bytes a0..a0+3 (raw(D, s) = lin(D with its first
// 4 bytes ^ s) for |D| >= 4), which replaces the start * x^(8 len) term.
template <bool INIT, bool NT>
__device__ __forceinline__ Streams hash_grid(uint64_t vs, uint64_t nb, uint64_t a0, uint64_t a1, uint32_t start,
                                             const uint32_t* lj, int lane) {
  constexpr int U = 4;
  const uint64_t lane_off = (uint64_t)lane * 16;
  const uint64_t lb = (a1 - vs) / kBlockBytes;  // blocks ending at or before a1
  Streams st;
  uint64_t b = 0;
  const bool head_full = vs >= a0 && lb >= 1;
  if (!head_full || INIT) {
    uint4 w = head_full ? gload16(vs + lane_off) : gload16_masked(vs + lane_off, a0, a1);
    if (INIT) {
      const int o = (int)(a0 - vs) - 16 * lane;  // start's byte offset within this lane's granule
#define HF3FS_INIT_XOR(F, D)                                           \
  {                                                                    \
    const int sh = o - 4 * (D);                                        \
    if (sh > -4 && sh < 4) w.F ^= sh >= 0 ? start << (8 * sh) : start >> (-8 * sh); \
  }
      HF3FS_INIT_XOR(x, 0)
      HF3FS_INIT_XOR(y, 1)
      HF3FS_INIT_XOR(z, 2)
      HF3FS_INIT_XOR(w, 3)
#undef HF3FS_INIT_XOR
    }
    st.step(w, lj);
    b = 1;
  }
  const uint64_t nfull = lb > b ? lb - b : 0;
  const uint64_t gbase = vs + b * kBlockBytes + lane_off;
  uint64_t g = 0;
  if (nfull >= U) {
    uint4 c0 = gload16s<NT>(gbase), c1 = gload16s<NT>(gbase + 1024), c2 = gload16s<NT>(gbase + 2048),
          c3 = gload16s<NT>(gbase + 3072);
    for (g = U; g + U <= nfull; g += U) {
      const uint64_t q = gbase + g * kBlockBytes;
      uint4 n0 = gload16s<NT>(q), n1 = gload16s<NT>(q + 1024), n2 = gload16s<NT>(q + 2048),
            n3 = gload16s<NT>(q + 3072);
      st.step(c0, lj);
      st.step(c1, lj);
      st.step(c2, lj);
      st.step(c3, lj);
      c0 = n0;
      c1 = n1;
      c2 = n2;
      c3 = n3;
    }
    st.step(c0, lj);
    st.step(c1, lj);
    st.step(c2, lj);
    st.step(c3, lj);
  }
  for (; g < nfull; ++g) st.step(gload16s<NT>(gbase + g * kBlockBytes), lj);
  if (lb < nb && lb >= b) st.step(gload16_masked(vs + lb * kBlockBytes + lane_off, a0, a1), lj);
  return st;
}

// x^(e) for a signed bit count e; every lane of each 32-lane half computes the
// same exponent (lanes 0-31: eA, lanes 32-63: eB) in 5 butterfly rounds.
template <uint32_t POLY>
__device__ __forceinline__ uint32_t xpow_pair(int64_t eA, int64_t eB, int lane, const PolyTables* T) {
  const int64_t e = lane < 32 ? eA : eB;
  const int k = lane & 31;
  const uint64_t m = e < 0 ? (uint64_t)(-e) : (uint64_t)e;
  const uint32_t* tab = e < 0 ? T->xinv : T->xpow;
  uint32_t f = ((m >> k) & 1u) ? tab[k] : kOne;
  if (m >> 32) {
    const uint32_t h = ((m >> (k + 32)) & 1u) ? tab[k + 32] : kOne;
    f = gf_mul(f, h, POLY);
  }
#pragma unroll
  for (int d = 1; d < 32; d <<= 1) f = gf_mul(f, __shfl_xor(f, d, 64), POLY);
  return f;
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
                                                         const uint32_t* __restrict__ dyn_max) {
  __shared__ uint32_t lds[kLdsWords + kMulcWords];
  fill_lds(lds, T);
  const int lane = threadIdx.x & 63;
  const uint32_t* lj = lds + (lane & 31);
  const uint32_t* lc = lds + kLdsWords;
  const uint32_t n = (uint32_t)src.n;
  if (dyn_max) {  // longest range known only on the device (update jobs): no empty segments
    const uint32_t m = __builtin_amdgcn_readfirstlane(*dyn_max);
    segs = m > seg_bytes ? (uint32_t)((m + seg_bytes - 1) / seg_bytes) : 1u;
  }
  const uint32_t ntasks = n * segs;
  const uint32_t nwaves = gridDim.x * kWaves;
  // Tickets only pay for ragged, moderately sized task sets: one counter word
  // serves ~88 dequeues/us (MI355X_MICROARCH.md "dequeue"), so with >16 tasks
  // per wave a static stride balances by averaging instead.
  if (ntasks <= nwaves || ntasks > 16u * nwaves) queue = nullptr;
  uint32_t t = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  while (t < ntasks) {
    const uint32_t seg = segs == 1 ? 0u : t / n;
    const uint32_t i = t - seg * n;
    const uint64_t len = src.length(i);
    const uint64_t tb = (uint64_t)seg * seg_bytes;
    if (seg == 0 || tb < len) {
      if (len == 0) {  // create(type, buf, 0, start) == {type, start}
        if (lane == 0) {
          if (DIRECT)
            out[i] = src.start_of(i);
          else
            atomicXor(out + i, src.start_of(i));
        }
      } else if (DIRECT) {
        // whole buffer in one task: block grid aligned to the buffer END (16 B
        // granule), so an aligned buffer needs neither masking nor a final
        // shift; the start value is xor-ed into the first four data bytes.
        const uint64_t a0 = src.addr(i), a1 = a0 + len;
        const uint64_t vend = (a1 + 15) & ~uint64_t(15);
        const uint64_t nb = (vend - (a0 & ~uint64_t(15)) + kBlockBytes - 1) / kBlockBytes;
        const uint64_t vs = vend - nb * kBlockBytes;
        const uint32_t start = src.start_of(i);
        // The start xor needs data bytes a0..a0+3 inside block 0; when they
        // straddle into block 1 (a0 in the block's last 3 bytes) the start
        // term start * x^(8 len) is added explicitly instead.
        const bool spill = a0 - vs > (uint64_t)(kBlockBytes - 4);
        const Streams st = len >= 4 && !spill ? hash_grid<true, NT>(vs, nb, a0, a1, start, lj, lane)
                                              : hash_grid<false, NT>(vs, nb, a0, a1, start, lj, lane);
        uint32_t r = __builtin_amdgcn_readfirstlane(fold_streams(st, lc, lane));
        const uint32_t pad = (uint32_t)(vend - a1);  // lin * x^(8 pad) -> lin
        if (pad) r = gf_mul(r, T->xneg8[pad], POLY);
        if (len < 4) {
          r ^= gf_mul(start, T->xpos8[len], POLY);
        } else if (spill) {  // wave-uniform branch: the butterfly needs every lane
          const uint32_t f = xpow_pair<POLY>(8 * (int64_t)len, 8 * (int64_t)len, lane, T);
          r ^= gf_mul(start, __builtin_amdgcn_readlane(f, 0), POLY);
        }
        if (lane == 0) out[i] = r;
      } else {
        const uint64_t te = len < tb + seg_bytes ? len : tb + seg_bytes;
        const uint64_t base = src.addr(i);
        const uint64_t a0 = base + tb, a1 = base + te;
        const uint64_t vs = a0 & ~uint64_t(15);
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
      t += nwaves;
    }
  }
}

template <uint32_t POLY, bool DIRECT, bool NT, class Src>
void launch_one(const Src& src, const Plan& p, uint32_t* out, const PolyTables* T, hipStream_t s) {
  hipLaunchKernelGGL((k_crc_ranges<POLY, DIRECT, NT, Src>), dim3(p.grid), dim3(kThreads), 0, s, src,
                     (uint32_t)p.segs, p.seg_bytes, out, T, p.queue, p.dyn_max);
}

template <uint32_t POLY, class Src>
void launch_poly(const Src& src, const Plan& p, uint32_t* out, const PolyTables* T, hipStream_t s) {
  const bool direct = p.segs == 1 && !p.dyn_max;
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
  __shared__ uint32_t lds[kLdsWords + kMulcWords];
  __shared__ uint64_t s_addr, s_len;
  __shared__ uint32_t s_ticket, s_start, s_cmd;
  __shared__ uint32_t s_part[kWaves];
  fill_lds(lds, T);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const uint32_t* lj = lds + (lane & 31);
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
            s_ticket = ticket;
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
    const uint64_t base = s_addr, len = s_len;
    const uint32_t start = s_start;
    // wave w hashes [w*seg, (w+1)*seg) of the request
    const uint64_t seg = ((len + kWaves - 1) / kWaves + kBlockBytes - 1) / kBlockBytes * kBlockBytes;
    const uint64_t tb = (uint64_t)wave * seg;
    uint32_t val = 0;
    if (tb < len) {
      const uint64_t te = len < tb + seg ? len : tb + seg;
      const uint64_t a0 = base + tb, a1 = base + te;
      const uint64_t vs = a0 & ~uint64_t(15);
      const uint64_t nb = (a1 - vs + kBlockBytes - 1) / kBlockBytes;
      const uint64_t vend = vs + nb * kBlockBytes;
      const Streams st = hash_grid<false, false>(vs, nb, a0, a1, 0u, lj, lane);
      const uint32_t v = fold_streams(st, lc, lane);
      const uint32_t f = xpow_pair<POLY>(8 * (int64_t)(base + len - vend), 8 * (int64_t)len, lane, T);
      val = gf_mul(__builtin_amdgcn_readfirstlane(v), __builtin_amdgcn_readlane(f, 0), POLY);
      if (wave == 0) val ^= gf_mul(start, __builtin_amdgcn_readlane(f, 32), POLY);
    }
    if (lane == 0) s_part[wave] = val;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t r = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) r ^= s_part[w];
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

// ChecksumInfo::combine element-wise: acc = (~acc) * x^(8 len2) ^ crc2.
template <uint32_t POLY>
__global__ void k_combine(uint32_t* __restrict__ acc, const uint32_t* __restrict__ crc2,
                          const uint64_t* __restrict__ len2, uint64_t n, const PolyTables* __restrict__ T) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t l = len2[i];
    if (l == 0) continue;
    uint64_t m = 8 * l;
    uint32_t x = kOne;
    for (int k = 0; m; ++k, m >>= 1)
      if (m & 1) x = gf_mul(x, T->xpow[k], POLY);
    acc[i] = gf_mul(~acc[i], x, POLY) ^ crc2[i];
  }
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
  const unsigned grid = (unsigned)(want < 8192 ? want : 8192);
  if (type == kTypeCrc32)
    hipLaunchKernelGGL(k_combine<kPolyCrc32>, dim3(grid), dim3(256), 0, s, acc, crc2, len2, n, &tabs->poly[1]);
  else
    hipLaunchKernelGGL(k_combine<kPolyCrc32c>, dim3(grid), dim3(256), 0, s, acc, crc2, len2, n, &tabs->poly[0]);
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
