// crc_kernels.h -- CDNA4 (gfx950) kernels of the chunk-integrity engine.
//
// Algorithm: a wave hashes a contiguous byte range in 1 KiB
// "blocks".  Lane l loads the 16 B granule at block + 16 l with one coalesced
// global_load_dwordx4 (a wave-instruction moves the whole 1 KiB), and keeps
// FOUR independent CRC streams, one per dword d of its granule.  Stream (l, d)
// therefore sees one dword every 1024 bytes, so its register update is
//     s <- (s ^ w) * x^(8*1024)  mod P,
// a 32-bit linear map evaluated with four 256-entry byte tables (slicing-by-4
// whose tables already include the 1020-byte stride).  The tables live in LDS
// replicated 32 times so that lane l always reads copy (l % 32): every
// ds_read_b32 is bank-conflict free whatever the data bytes are (random
// indices into one shared table would cost ~3.5x in bank conflicts).
// After the range, the 256 stream registers are folded with compile-time
// shift constants (x^32 inside a lane, x^(128*2^k) across lanes via a shuffle
// tree) into the range's linear CRC, which is shifted to the end of its buffer
// by x^(8 e) (lane-parallel power from a table of x^(2^k)) and xor-ed into the
// buffer's output word.  No MFMA: CRC is GF(2) arithmetic, not a contraction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf2.h"

namespace hf3fs_crc {

constexpr int kWaves = 16;               // waves per workgroup (one workgroup per CU)
constexpr int kThreads = kWaves * 64;    // 1024
constexpr int kBlockBytes = 1024;        // bytes one wave hashes per step
constexpr int kCopies = 32;              // LDS replicas: one per ds_read_b32 bank
constexpr int kLdsWords = 4 * 256 * kCopies;  // 128 KiB, replicated step tables
constexpr int kMulcTables = 7;                 // fold constants x^-32, x^(-128*2^k) k=0..5
constexpr int kMulcWords = kMulcTables * 1024; // 28 KiB (LDS total 156 KiB of 160)
constexpr int kPowDigits = 5;
constexpr int kXs8Neg = 1024, kXs8Pos = 32;      // direct table of x^(8n) for small signed n                  // byte-digit power tables cover |n| < 2^40 bytes

// Per-polynomial constant tables (built on the host, resident in HBM).
struct PolyTables {
  uint32_t step[4][256];                // step[k][b] = (b << 8k) * x^(8*1024) mod P
  uint32_t mulc[kMulcTables][4][256];   // mulc[t][k][b] = (b << 8k) * C_t, C_0 = x^-32, C_t = x^(-128*2^(t-1))
  uint32_t xpow[64];                    // x^(2^k)
  uint32_t xinv[64];                    // x^(-2^k)
  uint32_t xneg8[16];                   // x^(-8p)
  uint32_t xneg8_cols[16][32];          // xneg8_cols[p][i] = x^(-8p) * x^i: lane-parallel multiply by x^(-8p)
  uint32_t xpos8[4];                    // x^(8p)
  uint32_t pow8b[kPowDigits][256];      // pow8b[j][d] = x^(8 d 256^j): x^(8n) = product over the bytes of n
  uint32_t inv8b[kPowDigits][256];      // the same powers of x^-1
};
// Short-range tables of the serde-frame finalize (frame_kernels.hip), kept out
// of PolyTables: growing that struct changed the frame stream kernel's code
// generation (41.0 -> 38.8 KB, 7 % slower on 16 KiB frames, same source).
struct ShortTables {
  uint32_t dw[4][256];              // dw[k][b] = (b << 8k) * x^32: one dword of data per step
  uint32_t b8[256];                 // b8[b] = b * x^8: one byte of data per step
  uint32_t xs8[kXs8Neg + kXs8Pos];  // xs8[kXs8Neg + n] = x^(8n), -kXs8Neg <= n < kXs8Pos
};
// Tables of the lane-weight fold (crc_device.h fold_lw, every kernel):
//   w[j][n][c]  = (n << 4j) * x^(-128 c), c = lane % 32: lane c reads column c, i.e.
//                 always its own bank -- the per-lane weight of the fold (nibble tables:
//                 16 entries x 32 columns stay conflict-free at 16 KiB)
//   c0[k][b]    = (b << 8k) * x^-32 (the in-lane Horner over the 4 streams)
//   ch[k][b]    = (b << 8k) * x^-4096 (lanes 32..63 relative to lanes 0..31)
// c0 and ch are byte tables: one VALU op per lookup (the byte extract; the table base is the
// ds_read offset) against two for a nibble; their lookups may collide in banks, and the
// fold is VALU-bound, not LDS-bound.
constexpr int kFoldWords = 8 * 16 * 32 + 2 * 4 * 256;  // 24 KiB
struct FoldTables {
  uint32_t w[8][16][32];
  uint32_t c0[4][256];
  uint32_t ch[4][256];
};
static_assert(sizeof(FoldTables) == 4 * kFoldWords, "FoldTables is its LDS image");
struct DeviceTables {
  PolyTables poly[2];   // [0] CRC32C, [1] CRC32
  ShortTables sh[2];
  FoldTables fold[2];
};

// x^(8 n) for a signed byte count n: one table entry per non-zero byte of |n|
// (4 multiplies for n < 4 GiB instead of one per bit), bits from 2^40 on from
// the x^(2^k) table.
// tab[k] = x^(+-2^k) for k < 64; exponent bits 64.. (byte counts >= 2^61) square tab[63]
__device__ __forceinline__ uint32_t xpow2k(const uint32_t* tab, int k, uint32_t poly) {
  uint32_t f = tab[k < 64 ? k : 63];
  for (int j = 63; j < k; ++j) f = gf_mul(f, f, poly);
  return f;
}

__device__ __forceinline__ uint32_t xpow8_bytes(int64_t nbytes, const PolyTables* T, uint32_t poly) {
  uint64_t m = nbytes < 0 ? (uint64_t)(-nbytes) : (uint64_t)nbytes;
  const bool neg = nbytes < 0;
  uint32_t x = kOne;
  bool first = true;
  for (int j = 0; j < kPowDigits && m; ++j, m >>= 8) {
    const uint32_t d = (uint32_t)(m & 0xffu);
    if (!d) continue;
    const uint32_t f = neg ? T->inv8b[j][d] : T->pow8b[j][d];
    x = first ? f : gf_mul(x, f, poly);
    first = false;
  }
  for (int k = 8 * kPowDigits + 3; m; ++k, m >>= 1)  // byte bit b -> exponent bit b + 3
    if (m & 1) x = gf_mul(x, xpow2k(neg ? T->xinv : T->xpow, k, poly), poly);
  return x;
}

// -------- job sources: where range i lives ---------------------------------
// Each source answers: how many ranges, address and length of range i, and
// the register value the range starts from (ChecksumInfo startingChecksum).
struct StridedSource {
  uint64_t base, stride, len, n;
  uint32_t start;
  __device__ uint64_t addr(uint64_t i) const { return base + i * stride; }
  __device__ uint64_t length(uint64_t) const { return len; }
  __device__ uint32_t start_of(uint64_t) const { return start; }
};

struct ListSource {
  const uint64_t* addrs;
  const uint64_t* lens;
  const uint32_t* starts;  // nullable: ~0U
  uint64_t n;
  uint32_t default_start;
  __device__ uint64_t addr(uint64_t i) const { return addrs[i]; }
  __device__ uint64_t length(uint64_t i) const { return lens[i]; }
  __device__ uint32_t start_of(uint64_t i) const { return starts ? starts[i] : default_start; }
};

struct ArenaSource {  // KVCache blocks addressed by offset into one arena
  uint64_t base;
  const uint64_t* offsets;
  const uint32_t* lens;
  uint64_t n;
  __device__ uint64_t addr(uint64_t i) const { return base + offsets[i]; }
  __device__ uint64_t length(uint64_t i) const { return lens[i]; }
  __device__ uint32_t start_of(uint64_t) const { return ~0u; }
};

// -------- launch plan -------------------------------------------------------
struct Plan {
  uint64_t segs;       // tasks per range (>= 1)
  uint64_t seg_bytes;  // bytes per task, multiple of kBlockBytes
  uint32_t grid;       // workgroups
  uint32_t* queue;     // per-launch ticket counter (zeroed on the stream) or nullptr (static stride)
  const uint32_t* dyn_max;  // device word: longest range (segs computed in-kernel), or nullptr
  const uint32_t* skip;     // device word: nonzero = another path took the batch (frame stream), or nullptr
  const uint32_t* bal;      // byte-balanced task boundaries per wave (launch_balance), or nullptr
  const uint64_t* boff;     // with bal: byte runs -- wave w hashes the bytes from offset boff[w] of range
                            // bal[w] up to offset boff[w + 1] of range bal[w + 1] (ranges split anywhere)
  bool nt;                  // non-temporal loads for the streamed body of each range
  uint64_t pipe_max;        // whole-buffer tasks on a static stride whose ranges are all <= pipe_max
                            // bytes load the next task's head during the fold
  bool range_stream = false;  // with bal (whole-range tasks): one block stream per wave (k_crc_range_stream)
  uint32_t run_rep = 1;       // with boff: runs per wave -- bal / boff place run_rep x W runs and wave w
                              // hashes runs w, w + W, ... (W = the launch's waves), so the chip's reads
                              // sweep the batch in run_rep windows of W runs
};

// -------- persistent request service (coalescer service mode) -------------
// A request ring in pinned, coherent host memory, served by resident
// workgroups that poll it (no launch per request).  Tickets are 32-bit and
// wrap; the ring size is a power of two.  Each slot is published on its own
// (seq = ticket + 1, stored last), so submitters never wait for each other.
// Ticket t is served by workgroup t % workgroups: no claim protocol, no
// shared counter, one PCIe poll per request per workgroup.
struct ServiceReq {  // written by the host, seq last
  uint64_t addr;     // device-accessible address of the bytes
  uint64_t len;
  uint32_t start;
  uint32_t seq;      // ticket + 1 once the slot holds that ticket's request
  uint32_t pad[2];
};
struct ServiceResp {  // written by the device: value, then done = ticket + 1
  uint32_t value;
  uint32_t done;
};
struct ServiceCtrl {  // host memory
  uint32_t stop;      // host asks the service to exit
  // diagnostics, written by the device when a workgroup exits
  uint32_t dbg_exit;  // 2 idle timeout, 3 stop
  uint32_t dbg_seq;   // the ticket it waited for and the seq of its slot
  uint32_t dbg_ticket;
  uint32_t pad[12];
};
struct ServiceArgs {
  const ServiceReq* req;
  ServiceResp* resp;
  ServiceCtrl* ctrl;
  uint32_t* next;        // device, one word per workgroup: its next ticket (persists across launches)
  uint32_t ring;         // power of two
  uint64_t idle_ticks;   // exit after this many wall-clock ticks without a request
};

// Launchers (defined in crc_kernels.hip).  `direct` = segs == 1 (plain store
// of the result); otherwise results are xor-accumulated and out must be
// zeroed beforehand.
hipError_t launch_ranges_strided(uint8_t type, const StridedSource& src, const Plan& p, uint32_t* out,
                                 const DeviceTables* tabs, hipStream_t s);
hipError_t launch_ranges_list(uint8_t type, const ListSource& src, const Plan& p, uint32_t* out,
                              const DeviceTables* tabs, hipStream_t s);
hipError_t launch_ranges_arena(uint8_t type, const ArenaSource& src, const Plan& p, uint32_t* out,
                               const DeviceTables* tabs, hipStream_t s);
// bal[0..nw] = byte-balanced contiguous task ranges of nw waves over n
// whole-range tasks (scratch: partial[nblocks]); nw = the launch's waves.
// With boff (nw + 1 words): byte runs instead -- wave w starts at byte
// boff[w] of range bal[w], exactly ceil(w * total / nw) bytes into the batch.
hipError_t launch_balance(const ArenaSource& src, uint64_t n, uint32_t nw, uint64_t* partial, uint32_t nblocks,
                          uint32_t* bal, hipStream_t s, uint64_t* boff = nullptr);
hipError_t launch_balance(const ListSource& src, uint64_t n, uint32_t nw, uint64_t* partial, uint32_t nblocks,
                          uint32_t* bal, hipStream_t s, uint64_t* boff = nullptr);
// Byte runs of n equal ranges of len > 0 bytes (bal[0..nw], boff[0..nw]) without a balance pass.
hipError_t launch_runs_uniform(uint64_t n, uint64_t len, uint32_t nw, uint32_t* bal, uint64_t* boff, hipStream_t s);
hipError_t launch_service(const ServiceArgs& a, uint32_t workgroups, const DeviceTables* tabs, hipStream_t s);
hipError_t launch_compare(const uint32_t* computed, const uint32_t* expected, uint8_t* mismatch, uint32_t* count,
                          uint64_t n, hipStream_t s);
hipError_t launch_combine(uint8_t type, uint32_t* acc, const uint32_t* crc2, const uint64_t* len2, uint64_t n,
                          const DeviceTables* tabs, hipStream_t s);
// Zero n words with a kernel.  Every device-API path zeroes this way instead of
// hipMemsetAsync: captured into a hipGraph, small memset nodes replayed stale
// byte patterns (0x30303030 into a mismatch count) once other work had run in
// the process; kernel nodes replay exactly.
hipError_t launch_fill_words(void* p, uint64_t n_words, uint32_t v, hipStream_t s);
inline hipError_t launch_zero_words(void* p, uint64_t n_words, hipStream_t s) { return launch_fill_words(p, n_words, 0u, s); }
inline hipError_t launch_zero_counter(uint32_t* q, hipStream_t s) { return launch_zero_words(q, 4, s); }
hipError_t launch_fill_synth(uint8_t* dst, uint64_t stride, uint64_t chunk_len, uint64_t n_chunks, uint64_t seed,
                             uint64_t first_chunk_id, hipStream_t s);

}  // namespace hf3fs_crc
