// hf3fs_crc_api.hip -- C ABI of libhf3fs_crc.so (declared in include/hf3fs_crc.h).
//
// Host side of the boundary: per-device contexts (constant tables in HBM),
// launch planning and argument validation.  All byte hashing happens in the
// HIP kernels of crc_kernels.hip; the host only does O(log n) scalar algebra
// (combine/shift of 32-bit values), exactly like ChecksumInfo::combine does on
// the reference's host (Common.h:179-198).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hf3fs_crc.h"
#include "aux_kernels.h"
#include "frame_kernels.h"
#include "crc_kernels.h"
#include "digest_kernels.h"
#include "internal.h"
#include "options.h"
#include "update_kernels.h"

static_assert(sizeof(hf3fs_crc_update_io) == 56, "hf3fs_crc_update_io ABI layout");
static_assert(sizeof(hf3fs_crc_read_io) == 48, "hf3fs_crc_read_io ABI layout");
static_assert(sizeof(hf3fs_crc_block_digest) == 24, "hf3fs_crc_block_digest ABI layout");
static_assert(sizeof(hf3fs_crc_file_digest) == 24, "hf3fs_crc_file_digest ABI layout");
static_assert(sizeof(hf3fs_crc_scrub_io) == 32, "hf3fs_crc_scrub_io ABI layout");
static_assert(sizeof(hf3fs_crc_frame) == 24, "hf3fs_crc_frame ABI layout");
static_assert(sizeof(hf3fs_crc_engine_meta) == 120, "hf3fs_crc_engine_meta ABI layout");
static_assert(sizeof(hf3fs_crc_anomaly) == 72, "hf3fs_crc_anomaly ABI layout");

using namespace hf3fs_crc;

namespace {

#define HIP_OR_FAIL(expr)                                                                                    \
  do {                                                                                                       \
    hipError_t _e = (expr);                                                                                  \
    if (_e != hipSuccess) return fail(HF3FS_CRC_DEVICE_ERROR, "%s: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                                      __FILE__, __LINE__);                                                   \
  } while (0)

bool valid_type(uint8_t t) { return t == kTypeNone || t == kTypeCrc32c || t == kTypeCrc32; }

void build_short_tables(ShortTables& T, uint32_t poly) {
  const uint32_t x32 = xpow_bits(32, poly), x8 = xpow_bits(8, poly);
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) T.dw[k][b] = gf_mul(b << (8 * k), x32, poly);
  for (uint32_t b = 0; b < 256; ++b) T.b8[b] = gf_mul(b, x8, poly);
  for (int n = -kXs8Neg; n < kXs8Pos; ++n) T.xs8[kXs8Neg + n] = xpow_signed_bits(8ll * n, poly);
}

void build_fold_tables(FoldTables& T, uint32_t poly) {
  const uint32_t c0 = xpow_neg_bits(32, poly), ch = xpow_neg_bits(4096, poly);
  for (int j = 0; j < 8; ++j)
    for (uint32_t n = 0; n < 16; ++n) {
      const uint32_t a = n << (4 * j);
      for (int c = 0; c < 32; ++c) T.w[j][n][c] = gf_mul(a, xpow_neg_bits(128ull * c, poly), poly);
    }
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) {
      T.c0[k][b] = gf_mul(b << (8 * k), c0, poly);
      T.ch[k][b] = gf_mul(b << (8 * k), ch, poly);
    }
}

void build_poly_tables(PolyTables& T, uint32_t poly) {
  const uint32_t k = xpow_bits(8ull * kBlockBytes, poly);
  for (int b = 0; b < 4; ++b)
    for (uint32_t i = 0; i < 256; ++i) T.step[b][i] = gf_mul(i << (8 * b), k, poly);
  T.xpow[0] = kOne >> 1;
  T.xinv[0] = x_inverse(poly);
  for (int i = 1; i < 64; ++i) {
    T.xpow[i] = gf_mul(T.xpow[i - 1], T.xpow[i - 1], poly);
    T.xinv[i] = gf_mul(T.xinv[i - 1], T.xinv[i - 1], poly);
  }
  for (int t = 0; t < kMulcTables; ++t) {
    const uint32_t c = xpow_neg_bits(t == 0 ? 32 : (128ull << (t - 1)), poly);
    for (int b = 0; b < 4; ++b)
      for (uint32_t i = 0; i < 256; ++i) T.mulc[t][b][i] = gf_mul(i << (8 * b), c, poly);
  }
  for (int p = 0; p < 16; ++p) T.xneg8[p] = xpow_neg_bits(8ull * p, poly);
  for (int p = 0; p < 16; ++p)
    for (int i = 0; i < 32; ++i) T.xneg8_cols[p][i] = gf_mul(T.xneg8[p], xpow_bits((uint64_t)i, poly), poly);
  for (int p = 0; p < 4; ++p) T.xpos8[p] = xpow_bits(8ull * p, poly);

  for (int j = 0; j < kPowDigits; ++j) {  // pow8b[j][d] = (x^(8 * 256^j))^d
    const uint32_t base = xpow_bits(8ull << (8 * j), poly), ibase = xpow_neg_bits(8ull << (8 * j), poly);
    T.pow8b[j][0] = T.inv8b[j][0] = kOne;
    for (int d = 1; d < 256; ++d) {
      T.pow8b[j][d] = gf_mul(T.pow8b[j][d - 1], base, poly);
      T.inv8b[j][d] = gf_mul(T.inv8b[j][d - 1], ibase, poly);
    }
  }
}

// Work queued by one thread on one stream is ordered, so per-(stream, thread)
// state is reused safely by that pair; no two pairs ever share it (two threads
// on the null stream, or on one stream handle, interleave their launches).
using StreamKey = std::pair<hipStream_t, std::thread::id>;
inline StreamKey stream_key(hipStream_t s) { return {s, std::this_thread::get_id()}; }

// Device memory the library owns, from hipMalloc also while the calling thread's
// stream is being captured: the thread switches to relaxed capture mode for the
// call (hipThreadExchangeStreamCaptureMode), so the allocation is no graph node
// and invalidates no capture.  Library scratch never comes from the stream-ordered
// pool.
hipError_t owned_malloc(void** p, size_t bytes, bool capturing) {
  if (!capturing) return hipMalloc(p, bytes);
  hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
  hipError_t e = hipThreadExchangeStreamCaptureMode(&m);
  if (e != hipSuccess) return e;
  e = hipMalloc(p, bytes);
  (void)hipThreadExchangeStreamCaptureMode(&m);  // back to the caller's mode
  return e;
}

// ---- Scratch of calls captured into graphs ------------------------------------------
// Every captured call gets device memory of its own (ticket counter, balance region,
// verify values, batch scratch), owned by the graph it was captured into.  One owner
// record per capture sequence (keyed by the capture id): one hipUserObject whose
// reference the graph holds -- and every executable graph instantiated from it -- and
// the capture's buffers: requests of <= kCapSmall bytes are carved from kCapSlab-byte
// slabs of the capture, larger ones get buffers of their own.  When the last reference
// goes, the destructor moves the buffers to the dead list.  A destructor may not call
// HIP, so dead buffers are freed by hf3fs_crc_release_graph_scratch, release_stream,
// shutdown, or by an uncaptured call once the dead list holds >= kCapReapBytes (never
// in every call: hipFree waits for the whole device).  That device-wide wait of hipFree
// is also what makes the free safe for an executable graph destroyed while a replay
// is still in flight (HIP may release user objects at hipGraphExecDestroy without
// waiting for pending launches).  A capture whose graph could not take the reference
// (orphan) keeps its buffers until release_graph_scratch or shutdown.  The registry is
// process-wide (a graph may outlive hf3fs_crc_shutdown) and a heap object that is never
// destroyed, so a late destructor callback from the HIP runtime's own teardown after
// this library's static destructors still finds a live mutex and map.  Owners are keyed
// by a never-reused id (the user object's payload), not by address.
struct CapturedBuf {
  void* ptr;
  int device;
  size_t bytes;
};
struct CaptureOwner {
  std::vector<CapturedBuf> bufs;
  unsigned long long cap_id = 0;  // the capture sequence (by_capture key), 0 = none
  bool orphan = true;
  uint8_t* slab = nullptr;  // the current slab and its fill
  size_t slab_used = 0;
};
constexpr size_t kCapSmall = 64 << 10, kCapSlab = 256 << 10, kCapReapBytes = 64ull << 20;
struct CapRegistry {
  std::mutex mu;
  std::map<uint64_t, CaptureOwner> live;                  // owner id -> owner
  std::map<unsigned long long, uint64_t> by_capture;      // capture id -> owner id (capture in progress)
  std::vector<CapturedBuf> dead;
  std::atomic<size_t> dead_n{0}, dead_bytes{0};
  uint64_t next_id = 1;
};
CapRegistry& cap_reg() {
  static CapRegistry* r = new CapRegistry;  // intentionally leaked (late destructor callbacks)
  return *r;
}

void captured_graph_gone(void* id) {
  CapRegistry& R = cap_reg();
  std::lock_guard<std::mutex> lk(R.mu);
  auto it = R.live.find((uint64_t)(uintptr_t)id);
  if (it == R.live.end() || it->second.orphan) return;  // freed already (shutdown), or no graph owns it
  for (const CapturedBuf& b : it->second.bufs) {
    R.dead.push_back(b);
    R.dead_bytes.fetch_add(b.bytes);
  }
  auto bc = R.by_capture.find(it->second.cap_id);
  if (bc != R.by_capture.end() && bc->second == it->first) R.by_capture.erase(bc);
  R.live.erase(it);
  R.dead_n.store(R.dead.size());
}

// hipFree the buffers of destroyed graphs.  Relaxed capture mode for the frees, so that
// another thread's global-mode capture neither fails this call nor is invalidated by it.
void free_captured(std::vector<CapturedBuf>& dead) {
  if (dead.empty()) return;
  int prev = 0;
  (void)hipGetDevice(&prev);
  hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
  (void)hipThreadExchangeStreamCaptureMode(&m);
  for (const CapturedBuf& b : dead) {
    (void)hipSetDevice(b.device);
    (void)hipFree(b.ptr);
  }
  (void)hipThreadExchangeStreamCaptureMode(&m);
  (void)hipSetDevice(prev);
}

// Free the dead list (force), or from an uncaptured call only once it holds kCapReapBytes.
void reap_captured(bool force = false) {
  CapRegistry& R = cap_reg();
  if (R.dead_n.load(std::memory_order_relaxed) == 0) return;
  if (!force && R.dead_bytes.load(std::memory_order_relaxed) < kCapReapBytes) return;
  std::vector<CapturedBuf> dead;
  {
    std::lock_guard<std::mutex> lk(R.mu);
    dead.swap(R.dead);
    R.dead_n.store(0);
    R.dead_bytes.store(0);
  }
  free_captured(dead);
}

// `bytes` of device memory for the call being captured on s, owned by the capture's graph.
hipError_t capture_malloc(int device, hipStream_t s, size_t bytes, void** out) {
  CapRegistry& R = cap_reg();
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long cap_id = 0;
  hipGraph_t graph = nullptr;
  const bool info = hipStreamGetCaptureInfo_v2(s, &st, &cap_id, &graph, nullptr, nullptr) == hipSuccess && graph &&
                    st == hipStreamCaptureStatusActive;
  uint64_t id = 0;
  bool fresh = false;
  {
    std::lock_guard<std::mutex> lk(R.mu);
    auto bc = info ? R.by_capture.find(cap_id) : R.by_capture.end();
    auto ow = bc != R.by_capture.end() ? R.live.find(bc->second) : R.live.end();
    if (ow == R.live.end() || ow->second.bufs.empty() || ow->second.bufs.front().device != device) {
      id = R.next_id++;
      R.live[id].cap_id = info ? cap_id : 0;  // an orphan until its graph holds the reference
      if (info) R.by_capture[cap_id] = id;
      fresh = true;
    } else {
      id = ow->first;
    }
  }
  if (fresh && info) {  // the owner's user object, retained by the graph
    hipUserObject_t obj = nullptr;
    if (hipUserObjectCreate(&obj, (void*)(uintptr_t)id, captured_graph_gone, 1, hipUserObjectNoDestructorSync) ==
        hipSuccess) {
      {  // owned before the graph holds the reference: the destructor may run as soon as it does
        std::lock_guard<std::mutex> lk(R.mu);
        R.live[id].orphan = false;
      }
      if (hipGraphRetainUserObject(graph, obj, 1, hipGraphUserObjectMove) != hipSuccess) {
        {
          std::lock_guard<std::mutex> lk(R.mu);
          R.live[id].orphan = true;  // the release below then frees nothing
        }
        (void)hipUserObjectRelease(obj, 1);
      }
    }
  }
  std::lock_guard<std::mutex> lk(R.mu);
  auto it = R.live.find(id);
  if (it == R.live.end()) return hipErrorInvalidValue;  // (the graph died during this call)
  CaptureOwner& o = it->second;
  const size_t need = (bytes + 255) & ~size_t(255);
  if (need <= kCapSmall) {
    if (!o.slab || o.slab_used + need > kCapSlab) {
      void* p = nullptr;
      hipError_t e = owned_malloc(&p, kCapSlab, true);
      if (e != hipSuccess) return e;
      o.bufs.push_back(CapturedBuf{p, device, kCapSlab});
      o.slab = (uint8_t*)p;
      o.slab_used = 0;
    }
    *out = o.slab + o.slab_used;
    o.slab_used += need;
    return hipSuccess;
  }
  void* p = nullptr;
  hipError_t e = owned_malloc(&p, bytes, true);
  if (e != hipSuccess) return e;
  o.bufs.push_back(CapturedBuf{p, device, bytes});
  *out = p;
  return hipSuccess;
}

struct Context {
  int device = -1;
  int cus = 0;
  DeviceTables* tables = nullptr;  // device
  hf3fs_crc_anomaly* diag = nullptr;  // device: the self-check's record (hf3fs_crc_anomalies)
  std::mutex mu;                   // guards everything below
  // verify scratch (d_computed == NULL), per (stream, calling thread)
  struct Scratch {
    uint32_t* ptr = nullptr;
    size_t words = 0;
  };
  std::map<StreamKey, Scratch> scratch;
  // scratch of update / record / frame / digest batches, per (stream, calling thread)
  std::map<StreamKey, Scratch> call;
  // Ticket counters of the dynamic task queues (16 B each, zeroed on the launch
  // stream right before the launch).  A (stream, thread) pair owns one counter
  // for all its launches (they are stream-ordered), a slot of a slab.  A launch
  // captured into a graph gets a counter of its own, owned by the graph
  // (capture_malloc), since the graph may be replayed on any stream.
  static constexpr uint32_t kSlabSlots = 16384;
  std::vector<uint32_t*> slabs;
  uint32_t slab_used = kSlabSlots;
  std::map<StreamKey, uint32_t*> counters;
  int queue_counter(hipStream_t s, uint32_t** out) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIP_OR_FAIL(hipStreamIsCapturing(s, &cs));
    if (cs != hipStreamCaptureStatusNone) {
      HIP_OR_FAIL(capture_malloc(device, s, 16, (void**)out));
      return HF3FS_CRC_OK;
    }
    reap_captured();
    std::lock_guard<std::mutex> lk(mu);
    uint32_t*& q = counters[stream_key(s)];
    if (!q) {
      if (slab_used == kSlabSlots) {
        uint32_t* slab = nullptr;
        HIP_OR_FAIL(hipMalloc(&slab, kSlabSlots * 16));
        slabs.push_back(slab);
        slab_used = 0;
      }
      q = slabs.back() + 4 * slab_used++;
    }
    *out = q;
    return HF3FS_CRC_OK;
  }
  // Byte-balance scratch of whole-range launches (partial sums + per-wave task
  // boundaries, bal_words words): one per (stream, thread) pair, and for a
  // launch captured into a graph a region owned by the graph (capture_malloc).
  static constexpr uint32_t kBalBlocksMax = 1024;
  std::map<StreamKey, uint32_t*> bal_scratch;
  size_t bal_words() const { return (2 * kBalBlocksMax + (size_t)cus * kWaves + 1 + 63) / 64 * 64; }
  int balance_scratch(hipStream_t s, uint32_t** out) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIP_OR_FAIL(hipStreamIsCapturing(s, &cs));
    *out = nullptr;
    if (cs != hipStreamCaptureStatusNone) {
      HIP_OR_FAIL(capture_malloc(device, s, bal_words() * 4, (void**)out));
      return HF3FS_CRC_OK;
    }
    reap_captured();
    std::lock_guard<std::mutex> lk(mu);
    uint32_t*& q = bal_scratch[stream_key(s)];
    if (!q) HIP_OR_FAIL(hipMalloc(&q, bal_words() * 4));
    *out = q;
    return HF3FS_CRC_OK;
  }
  // One-shot apply grid hints (update_batch): a pinned word per (stream, thread) pair where the
  // apply kernel leaves (pieces << 32 | n) of its call; the pair's next call sizes its one-shot
  // grid from it.  One slab for the process's pairs (a word of a captured call's graph stays
  // valid until shutdown); more pairs than slots share words (only the grid's fit suffers).
  // release_stream returns the stream's slots to a free list.
  static constexpr uint32_t kHintSlots = 4096;
  uint64_t* hint_host = nullptr;
  uint64_t* hint_dev = nullptr;
  std::map<StreamKey, uint32_t> hint_slot;
  std::vector<uint32_t> hint_free;
  uint32_t hint_next = 0;
  int hint_word(hipStream_t s, uint64_t** host, uint64_t** dev) {
    std::lock_guard<std::mutex> lk(mu);
    if (!hint_host) {
      HIP_OR_FAIL(hipHostMalloc((void**)&hint_host, kHintSlots * 8, hipHostMallocMapped | hipHostMallocCoherent));
      memset(hint_host, 0, kHintSlots * 8);
      HIP_OR_FAIL(hipHostGetDevicePointer((void**)&hint_dev, hint_host, 0));
    }
    auto it = hint_slot.find(stream_key(s));
    if (it == hint_slot.end()) {
      uint32_t slot;
      if (!hint_free.empty()) {
        slot = hint_free.back();
        hint_free.pop_back();
      } else {
        slot = hint_next++ % kHintSlots;
      }
      it = hint_slot.emplace(stream_key(s), slot).first;
    }
    *host = hint_host + it->second;
    *dev = hint_dev + it->second;
    return HF3FS_CRC_OK;
  }
  // A side stream per (stream, thread) pair with a fork and a join event: the update batch's
  // one-shot apply runs beside the finalize of every verdict.  Per pair, so
  // that two threads capturing graphs never fork into one stream; created in relaxed capture
  // mode (a call may be captured), destroyed by release_stream and shutdown.
  struct Side {
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
  };
  std::map<StreamKey, Side> sides;
  int side_of(hipStream_t s, Side* out) {
    {
      std::lock_guard<std::mutex> lk(mu);
      auto it = sides.find(stream_key(s));
      if (it != sides.end()) {
        *out = it->second;
        return HF3FS_CRC_OK;
      }
    }
    Side n;
    hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
    HIP_OR_FAIL(hipThreadExchangeStreamCaptureMode(&m));
    hipError_t e = hipStreamCreateWithFlags(&n.side, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&n.fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&n.join, hipEventDisableTiming);
    (void)hipThreadExchangeStreamCaptureMode(&m);
    if (e != hipSuccess) {
      if (n.join) (void)hipEventDestroy(n.join);
      if (n.fork) (void)hipEventDestroy(n.fork);
      if (n.side) (void)hipStreamDestroy(n.side);
      return fail(HF3FS_CRC_DEVICE_ERROR, "side stream: %s", hipGetErrorString(e));
    }
    std::lock_guard<std::mutex> lk(mu);
    sides[stream_key(s)] = n;
    *out = n;
    return HF3FS_CRC_OK;
  }
  static void destroy_side(const Side& x) {
    (void)hipStreamSynchronize(x.side);
    (void)hipEventDestroy(x.fork);
    (void)hipEventDestroy(x.join);
    (void)hipStreamDestroy(x.side);
  }
  // host staging (hf3fs_crc_create_host), one caller at a time
  std::mutex stage_mu;
  static constexpr size_t kStage = 32ull << 20;
  uint8_t* pinned[2] = {nullptr, nullptr};
  uint8_t* dstage[2] = {nullptr, nullptr};
  uint64_t* pdesc[2] = {nullptr, nullptr};  // pinned descriptors (addr, len pairs) + out
  uint64_t* ddesc[2] = {nullptr, nullptr};
  hipStream_t streams[2] = {nullptr, nullptr};
};

std::mutex g_ctx_mu;
std::vector<std::unique_ptr<Context>> g_ctx;

int get_context(Context** out) {
  int dev = 0;
  HIP_OR_FAIL(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  if ((int)g_ctx.size() <= dev) g_ctx.resize(dev + 1);
  if (!g_ctx[dev]) {
    auto c = std::make_unique<Context>();
    c->device = dev;
    HIP_OR_FAIL(hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, dev));
    auto host = std::make_unique<DeviceTables>();
    build_poly_tables(host->poly[0], kPolyCrc32c);
    build_poly_tables(host->poly[1], kPolyCrc32);
    build_short_tables(host->sh[0], kPolyCrc32c);
    build_short_tables(host->sh[1], kPolyCrc32);
    build_fold_tables(host->fold[0], kPolyCrc32c);
    build_fold_tables(host->fold[1], kPolyCrc32);
    HIP_OR_FAIL(hipMalloc(&c->tables, sizeof(DeviceTables)));
    HIP_OR_FAIL(hipMemcpy(c->tables, host.get(), sizeof(DeviceTables), hipMemcpyHostToDevice));
    HIP_OR_FAIL(hipMalloc(&c->diag, sizeof(hf3fs_crc_anomaly)));
    const hf3fs_crc_anomaly none{};
    HIP_OR_FAIL(hipMemcpy(c->diag, &none, sizeof(none), hipMemcpyHostToDevice));
    (void)options();  // the environment snapshot, once per process
    g_ctx[dev] = std::move(c);
  }
  *out = g_ctx[dev].get();
  return HF3FS_CRC_OK;
}

// Cross-task head prefetch for whole-buffer tasks on a static stride (DESIGN.md
// §3.1), by default only for batches whose longest range (the kernel's bound:
// the device-side maximum of record jobs, else the task size) fits the
// prefetched head four times over (A/B profiles/r01_ab_pipe.jsonl: f4 frames <= 16 KiB
// +3.5 %, d5 KV blocks <= 64 KiB -3 %, d2 4 MiB flat).
constexpr uint64_t kPipeMaxLen = 16 << 10;  // 4 x the prefetched head (kHashPrefetch = 4 blocks of 1 KiB)

// Tasks of seg_bytes each; as large as possible while leaving >= ~4 tasks per
// resident wave for balance (or seg_hint when the caller knows better).
// Option seg_kib overrides (tuning).
Plan make_plan(const Context* c, uint64_t n, uint64_t max_len, uint64_t seg_hint = 0) {
  Plan p;
  const Options& o = options();
  const uint64_t waves = (uint64_t)c->cus * kWaves;
  const uint64_t max_seg = std::max<uint64_t>(kBlockBytes, (max_len + kBlockBytes - 1) / kBlockBytes * kBlockBytes);
  uint64_t seg = max_seg;
  const uint64_t total = n * max_len;
  if (const uint32_t kib = o.seg_kib.load()) {
    seg = (uint64_t)kib * 1024;
  } else if (seg_hint) {
    seg = seg_hint;
  } else if (total / waves < 4 * seg) {
    uint64_t target = std::max<uint64_t>(total / (4 * waves), 64 << 10);
    uint64_t pow2 = 64 << 10;
    while (pow2 < target) pow2 <<= 1;
    seg = pow2;
  }
  seg = std::min(seg, max_seg);
  p.seg_bytes = seg;
  p.segs = std::max<uint64_t>(1, (max_len + seg - 1) / seg);
  const uint64_t tasks = n * p.segs;
  const uint64_t want = (tasks + kWaves - 1) / kWaves;
  p.grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)c->cus));
  p.queue = nullptr;
  p.dyn_max = nullptr;
  p.skip = nullptr;
  p.bal = nullptr;
  p.boff = nullptr;
  p.nt = o.nt.load() != 0;  // non-temporal streamed loads (A/B: profiles/r01_ab_bulk.json)
  const int pipe = o.pipe.load();
  p.pipe_max = pipe < 0 ? kPipeMaxLen : pipe ? ~uint64_t(0) : 0;
  p.range_stream = o.range_stream.load() != 0;
  return p;
}

// Ticket queues for ragged task sets, unless the static stride is forced (option static).
inline bool tickets_allowed() { return options().static_stride.load() == 0; }

// Zero what the launch accumulates into and hand it a freshly zeroed ticket
// counter (the kernel decides whether tickets pay for its task count).
int launch_prepare(Context* c, Plan& p, uint64_t n, uint32_t* out, hipStream_t s) {
  const uint64_t tasks = n * p.segs;
  if (tasks >= (1ull << 32)) return fail(HF3FS_CRC_INVALID_ARG, "too many tasks (%llu)", (unsigned long long)tasks);
  if (p.segs > 1 || p.dyn_max) HIP_OR_FAIL(launch_zero_words(out, n, s));
  p.queue = nullptr;
  if ((tasks > (uint64_t)p.grid * kWaves || p.dyn_max) && tickets_allowed()) {
    if (int rc = c->queue_counter(s, &p.queue)) return rc;
    HIP_OR_FAIL(launch_zero_counter(p.queue, s));
  }
  return HF3FS_CRC_OK;
}

// Whole-range tasks on a static stride (more than 16 per wave, too long for
// the cross-task prefetch) get byte-balanced contiguous task ranges per wave:
// the stride leaves the slowest waves' summed lengths several sigma above the
// mean for ragged sizes (KVCache blocks of 4-64 KiB).  Option balance = 0: off.
template <class Src>
int plan_balance(Context* c, Plan& p, const Src& src, uint64_t n, uint64_t max_len, hipStream_t s) {
  const bool on = options().balance.load() != 0;
  const uint64_t nw = (uint64_t)p.grid * kWaves;
  // (the kernel drops its ticket queue for more than 16 tasks per wave)
  if (!on || p.segs != 1 || p.dyn_max || max_len <= p.pipe_max || n <= 16 * nw) return HF3FS_CRC_OK;
  uint32_t* sc = nullptr;
  if (int rc = c->balance_scratch(s, &sc)) return rc;
  if (!sc) return HF3FS_CRC_OK;
  const uint32_t nblocks = (uint32_t)std::min<uint64_t>(Context::kBalBlocksMax, std::max<uint64_t>(1, n / 1024));
  uint64_t* partial = (uint64_t*)sc;
  uint32_t* bal = sc + 2 * Context::kBalBlocksMax;
  HIP_OR_FAIL(launch_balance(src, n, (uint32_t)nw, partial, nblocks, bal, s));
  p.bal = bal;
  return HF3FS_CRC_OK;
}

// Byte runs (launch_balance with boff): scratch for a ragged list of long
// ranges that every wave should split at exact byte shares of the batch.
struct ByteRuns {
  uint64_t* partial;
  uint32_t* bal;
  uint64_t* boff;
  uint32_t blocks;
  bool placed;  // bal / boff already placed on the stream (update prep's runs workgroup)
  uint32_t rep = 1;  // runs per wave (Plan::run_rep): bal / boff hold rep x W + 1 entries
};

// zeroed_queue: the caller zeroed `out` and hands over a zeroed ticket counter
// (update_batch: one zeroing launch per call instead of two per hash pass).
// runs: hash as byte runs (out must be zeroed: the parts are xor-ed).
int run_ranges_list(Context* c, uint8_t type, const ListSource& src, uint64_t max_len, uint32_t* out,
                    hipStream_t s, uint64_t seg_hint = 0, const uint32_t* dyn_max = nullptr,
                    const uint32_t* skip = nullptr, uint32_t* zeroed_queue = nullptr,
                    const ByteRuns* runs = nullptr) {
  if (src.n == 0) return HF3FS_CRC_OK;
  Plan p = make_plan(c, src.n, max_len, seg_hint);
  p.dyn_max = dyn_max;
  p.skip = skip;
  if (dyn_max) p.grid = (uint32_t)c->cus;  // task count unknown on the host: full persistent grid
  if (runs) {
    p.grid = (uint32_t)c->cus;
    p.queue = nullptr;
    if (!runs->placed)
      HIP_OR_FAIL(launch_balance(src, src.n, p.grid * kWaves * runs->rep, runs->partial, runs->blocks, runs->bal, s,
                                 runs->boff));
    p.bal = runs->bal;
    p.boff = runs->boff;
    p.run_rep = runs->rep;
    HIP_OR_FAIL(launch_ranges_list(type, src, p, out, c->tables, s));
    return HF3FS_CRC_OK;
  }
  if (zeroed_queue) {
    const bool tickets = (src.n * p.segs > (uint64_t)p.grid * kWaves || dyn_max) && tickets_allowed();
    p.queue = tickets ? zeroed_queue : nullptr;
  } else if (int rc = launch_prepare(c, p, src.n, out, s)) {
    return rc;
  }
  if (int rc = plan_balance(c, p, src, src.n, max_len, s)) return rc;
  HIP_OR_FAIL(launch_ranges_list(type, src, p, out, c->tables, s));
  return HF3FS_CRC_OK;
}

// The verify scratch of the calling thread on stream s.  Growth waits for the
// stream's queued work before freeing the old buffer (not graph-capturable
// then; a warm-up call of the largest size avoids it).  Only this thread ever
// launched work reading the old buffer, all of it on s.
// The calling (stream, thread) pair's buffer in `table`, at least `words` long.
// Only that pair ever uses the entry, so growth detaches it under the lock and
// waits for the stream, frees and allocates with the lock released (other
// threads' calls never wait for this stream), then publishes the new buffer.
// Option poison (test only): the words handed out are first filled with that
// pattern on the stream, so a call that read a word before writing it would
// see junk (tests/test_gpu_parity.py::test_update_batch_poisoned_scratch).
int pair_buffer(Context* c, std::map<StreamKey, Context::Scratch> Context::*table, hipStream_t s, size_t words,
                size_t grow_to, uint32_t** out) {
  const StreamKey key = stream_key(s);
  Context::Scratch e;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    Context::Scratch& slot = (c->*table)[key];
    if (slot.words >= words) {
      e = slot;
    } else {
      e = slot;
      slot = Context::Scratch{};
    }
  }
  if (e.words < words) {
    // only this thread launched work on the old buffer, all of it on s.  On a failure
    // before the new buffer exists the old entry goes back into the slot (nothing leaks).
    hipError_t err = e.ptr ? hipStreamSynchronize(s) : hipSuccess;
    if (err == hipSuccess && e.ptr) {
      err = hipFree(e.ptr);
      if (err == hipSuccess) e = Context::Scratch{};
    }
    uint32_t* fresh = nullptr;
    if (err == hipSuccess) err = hipMalloc(&fresh, grow_to * sizeof(uint32_t));
    std::lock_guard<std::mutex> lk(c->mu);
    if (err != hipSuccess) {
      (c->*table)[key] = e;  // the old buffer (or none, if it was freed)
      return fail(HF3FS_CRC_DEVICE_ERROR, "scratch growth to %zu words: %s", grow_to, hipGetErrorString(err));
    }
    e = Context::Scratch{fresh, grow_to};
    (c->*table)[key] = e;
  }
  if (const uint32_t pattern = options().poison.load()) HIP_OR_FAIL(launch_fill_words(e.ptr, words, pattern, s));
  *out = e.ptr;
  return HF3FS_CRC_OK;
}

// The verify values of a call with d_computed == NULL: the calling (stream, thread)
// pair's buffer, or during a capture a buffer owned by the captured graph (so a
// replay never writes a pair buffer that release_stream or a later growth freed).
int stream_scratch(Context* c, hipStream_t s, size_t words, uint32_t** out) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIP_OR_FAIL(hipStreamIsCapturing(s, &cs));
  if (cs != hipStreamCaptureStatusNone) {
    HIP_OR_FAIL(capture_malloc(c->device, s, words * 4, (void**)out));
    if (const uint32_t pattern = options().poison.load()) HIP_OR_FAIL(launch_fill_words(*out, words, pattern, s));
    return HF3FS_CRC_OK;
  }
  reap_captured();
  return pair_buffer(c, &Context::scratch, s, words, words, out);
}

// Scratch of one batch call (update, record jobs, frames, file digest): library-
// owned hipMalloc memory, never the stream-ordered pool.  Outside a stream capture
// it is the calling (stream, thread) pair's persistent buffer (pair_buffer).
// During a capture it is a buffer of the captured call alone, owned by the captured
// graph and freed after the graph is gone (capture_malloc).  Rounds 1 and 3
// saw the first DELTA update of a process -- the first call whose per-call
// hipMallocAsync scratch the pool had to grow -- verify a correct payload as
// mismatched in 2-3 of 16 fresh processes, and a retry pass.
int call_scratch(Context* c, hipStream_t s, size_t bytes, void** out) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIP_OR_FAIL(hipStreamIsCapturing(s, &cs));
  const size_t words = (bytes + 3) / 4;
  if (cs != hipStreamCaptureStatusNone) {
    HIP_OR_FAIL(capture_malloc(c->device, s, words * 4, out));
    if (const uint32_t pattern = options().poison.load()) HIP_OR_FAIL(launch_fill_words(*out, words, pattern, s));
    return HF3FS_CRC_OK;
  }
  reap_captured();
  uint32_t* p = nullptr;
  std::size_t have = 0;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    auto it = c->call.find(stream_key(s));
    if (it != c->call.end()) have = it->second.words;
  }
  const size_t grow_to = std::max<size_t>((words + 65535) / 65536 * 65536, 2 * have);
  if (int rc = pair_buffer(c, &Context::call, s, words, grow_to, &p)) return rc;
  *out = p;
  return HF3FS_CRC_OK;
}

// prep -> k_crc_ranges -> finalize over per-record jobs, with stream-ordered
// scratch {maxl[4], addr[n], len[n], v[n]}: the shape shared by the record
// batches (read results, scrub, frames).
// Scrub batches (whole stored chunks: their lengths are close to the bound) of
// n * max_len >= kRecordRunsBytes with max_len >= kRecordRunsMinLen hash as byte runs (every
// wave the same byte share, the balance placed on the device from the prep's lengths):
// 4096 x 4 MiB scrub records ran 3.5 % slower as 1 MiB ticketed segments (the planner's
// choice for a device-side length bound).  Read results keep the planner: their partial
// reads are far below the bound (the chunk size), and two balance launches would cost more
// than they save on a reaped batch of small reads.
constexpr uint64_t kRecordRunsBytes = 1ull << 30;
constexpr uint32_t kRecordRunsMinLen = 64 << 10;
constexpr uint64_t kRunWindowBytes = 4ull << 20;  // most bytes of one byte run (create_strided)

template <class Prep, class Fin>
int run_record_jobs(Context* c, uint8_t type, uint64_t n, uint32_t max_len, uint32_t start, hipStream_t s,
                    Prep prep, Fin fin, const char* what, bool runs_ok = false) {
  const bool use_runs = runs_ok && max_len >= kRecordRunsMinLen && n * (uint64_t)max_len >= kRecordRunsBytes;
  const uint32_t nw = (uint32_t)c->cus * kWaves;
  const uint32_t rblocks = (uint32_t)std::min<uint64_t>(kRunBlocksMax, std::max<uint64_t>(1, n / 256));
  const size_t head = (16 + n * (8 + 8 + 4) + 63) / 64 * 64;
  const size_t bytes = head + (use_runs ? (rblocks + 2 * (nw + 1)) * 8 + (nw + 1) * 4 : 0) + 64;
  void* scratch = nullptr;
  if (int rc = call_scratch(c, s, bytes, &scratch)) return rc;
  uint8_t* base = (uint8_t*)scratch;
  uint32_t* maxl = (uint32_t*)base;
  uint64_t* addr = (uint64_t*)(base + 16);
  uint64_t* len = addr + n;
  uint32_t* v = (uint32_t*)(len + n);
  int rc = HF3FS_CRC_OK;
  hipError_t e = launch_zero_words(maxl, 4, s);
  if (e == hipSuccess) e = prep(addr, len, maxl);
  if (e == hipSuccess && use_runs) e = launch_zero_words(v, n, s);  // the runs xor their parts in
  if (e != hipSuccess) rc = fail(HF3FS_CRC_DEVICE_ERROR, "%s prep: %s", what, hipGetErrorString(e));
  if (!rc) {
    ListSource src{addr, len, nullptr, n, start};
    if (use_runs) {
      uint64_t* partial = (uint64_t*)(base + head);
      const ByteRuns runs{partial, (uint32_t*)(partial + rblocks + 2 * (nw + 1)), partial + rblocks, rblocks, false};
      rc = run_ranges_list(c, type, src, max_len, v, s, 0, maxl, nullptr, nullptr, &runs);
    } else {
      rc = run_ranges_list(c, type, src, max_len, v, s, 0, maxl);
    }
  }
  if (!rc) {
    e = fin(v);
    if (e != hipSuccess) rc = fail(HF3FS_CRC_DEVICE_ERROR, "%s finalize: %s", what, hipGetErrorString(e));
  }
  return rc;
}

}  // namespace

int hf3fs_crc::current_tables(const DeviceTables** out) {
  Context* c = nullptr;
  if (int rc = get_context(&c)) return rc;
  *out = c->tables;
  return HF3FS_CRC_OK;
}

// ===========================================================================
extern "C" {

const char* hf3fs_crc_version(void) { return "hf3fs_crc 0.1 gfx950"; }

int hf3fs_crc_init(int device) {
  int prev = 0;
  HIP_OR_FAIL(hipGetDevice(&prev));
  HIP_OR_FAIL(hipSetDevice(device));
  Context* c = nullptr;
  int rc = get_context(&c);
  (void)hipSetDevice(prev);
  return rc;
}

void hf3fs_crc_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  for (auto& c : g_ctx) {
    if (!c) continue;
    (void)hipSetDevice(c->device);
    (void)hipFree(c->tables);
    for (uint32_t* slab : c->slabs) (void)hipFree(slab);
    for (auto& kv : c->scratch)
      if (kv.second.ptr) (void)hipFree(kv.second.ptr);
    for (auto& kv : c->call)
      if (kv.second.ptr) (void)hipFree(kv.second.ptr);
    (void)hipFree(c->diag);
    if (c->hint_host) (void)hipHostFree(c->hint_host);
    for (auto& kv : c->sides) Context::destroy_side(kv.second);
    c->sides.clear();
    for (auto& kv : c->bal_scratch)
      if (kv.second) (void)hipFree(kv.second);
    for (int k = 0; k < 2; ++k) {
      if (c->pinned[k]) (void)hipHostFree(c->pinned[k]);
      if (c->pdesc[k]) (void)hipHostFree(c->pdesc[k]);
      if (c->dstage[k]) (void)hipFree(c->dstage[k]);
      if (c->ddesc[k]) (void)hipFree(c->ddesc[k]);
      if (c->streams[k]) (void)hipStreamDestroy(c->streams[k]);
    }
  }
  g_ctx.clear();
  // every captured call's buffers: graphs still alive after shutdown must not be replayed
  std::vector<CapturedBuf> all;
  {
    CapRegistry& R = cap_reg();
    std::lock_guard<std::mutex> lk2(R.mu);
    all.swap(R.dead);
    for (auto& kv : R.live) all.insert(all.end(), kv.second.bufs.begin(), kv.second.bufs.end());
    R.live.clear();
    R.by_capture.clear();
    R.dead_n.store(0);
    R.dead_bytes.store(0);
  }
  free_captured(all);
}

int hf3fs_crc_release_stream(void* stream) {
  Context* c = nullptr;
  if (int rc = get_context(&c)) return rc;
  hipStream_t s = (hipStream_t)stream;
  HIP_OR_FAIL(hipStreamSynchronize(s));
  reap_captured(true);
  std::vector<void*> dead;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    for (auto* table : {&c->scratch, &c->call})
      for (auto it = table->begin(); it != table->end();) {
        if (it->first.first == s) {
          dead.push_back(it->second.ptr);
          it = table->erase(it);
        } else {
          ++it;
        }
      }
    for (auto it = c->bal_scratch.begin(); it != c->bal_scratch.end();) {
      if (it->first.first == s) {
        dead.push_back(it->second);
        it = c->bal_scratch.erase(it);
      } else {
        ++it;
      }
    }
    // ticket counters are 16 B slots of shared slabs: the stream's slot is dropped, not freed
    for (auto it = c->counters.begin(); it != c->counters.end();) it = it->first.first == s ? c->counters.erase(it) : ++it;
    for (auto it = c->sides.begin(); it != c->sides.end();) {
      if (it->first.first == s) {
        Context::destroy_side(it->second);
        it = c->sides.erase(it);
      } else {
        ++it;
      }
    }
    // the stream's one-shot hint words: cleared (the slot's next pair starts with the ticketed
    // call that counts its pieces) and back on the free list
    for (auto it = c->hint_slot.begin(); it != c->hint_slot.end();) {
      if (it->first.first == s) {
        __atomic_store_n(c->hint_host + it->second, 0ull, __ATOMIC_RELEASE);
        c->hint_free.push_back(it->second);
        it = c->hint_slot.erase(it);
      } else {
        ++it;
      }
    }
  }
  for (void* p : dead)
    if (p) HIP_OR_FAIL(hipFree(p));
  return HF3FS_CRC_OK;
}

int hf3fs_crc_release_graph_scratch(void) {
  reap_captured(true);  // buffers of graphs already destroyed
  std::vector<CapturedBuf> orphans;
  {
    CapRegistry& R = cap_reg();
    std::lock_guard<std::mutex> lk(R.mu);
    for (auto it = R.live.begin(); it != R.live.end();) {
      if (it->second.orphan) {
        orphans.insert(orphans.end(), it->second.bufs.begin(), it->second.bufs.end());
        it = R.live.erase(it);
      } else {
        ++it;
      }
    }
    // finished captures: no later allocation joins them
    for (auto it = R.by_capture.begin(); it != R.by_capture.end();)
      it = R.live.count(it->second) ? ++it : R.by_capture.erase(it);
  }
  free_captured(orphans);
  return HF3FS_CRC_OK;
}

int hf3fs_crc_graph_scratch_stats(uint64_t* live_buffers, uint64_t* live_bytes, uint64_t* dead_buffers) {
  CapRegistry& R = cap_reg();
  std::lock_guard<std::mutex> lk(R.mu);
  uint64_t bytes = 0, n = 0;
  for (auto& kv : R.live)
    for (const CapturedBuf& b : kv.second.bufs) {
      bytes += b.bytes;
      ++n;
    }
  if (live_buffers) *live_buffers = n;
  if (live_bytes) *live_bytes = bytes;
  if (dead_buffers) *dead_buffers = R.dead.size();
  return HF3FS_CRC_OK;
}

int hf3fs_crc_stream_wait(void* stream, uint32_t poll_us) {
  hipStream_t s = (hipStream_t)stream;
  if (poll_us == 0) {
    HIP_OR_FAIL(hipStreamSynchronize(s));
    return HF3FS_CRC_OK;
  }
  hipError_t e;
  while ((e = hipStreamQuery(s)) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(poll_us));
  HIP_OR_FAIL(e);
  return HF3FS_CRC_OK;
}

int hf3fs_crc_anomalies(int device, hf3fs_crc_anomaly* out, int reset) {
  if (!out) return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  int prev = 0;
  HIP_OR_FAIL(hipGetDevice(&prev));
  HIP_OR_FAIL(hipSetDevice(device));
  Context* c = nullptr;
  int rc = get_context(&c);
  if (!rc) {
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, c->diag, sizeof(*out), hipMemcpyDeviceToHost);
    if (e == hipSuccess && reset) {
      const hf3fs_crc_anomaly none{};
      e = hipMemcpy(c->diag, &none, sizeof(none), hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) rc = fail(HF3FS_CRC_DEVICE_ERROR, "anomalies: %s", hipGetErrorString(e));
  }
  (void)hipSetDevice(prev);
  return rc;
}

int hf3fs_crc_serialize_batch(uint8_t type, const uint32_t* d_values, uint64_t n, uint8_t* d_out, void* stream) {
  if (!valid_type(type)) return fail(HF3FS_CRC_INVALID_ARG, "unknown checksum type %u", type);
  if (n == 0) return HF3FS_CRC_OK;
  if (!d_values || !d_out) return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  HIP_OR_FAIL(launch_serialize(type, d_values, n, d_out, (hipStream_t)stream));
  return HF3FS_CRC_OK;
}

int hf3fs_crc_finalize_batch(uint32_t* d_values, uint64_t n, void* stream) {
  if (n == 0) return HF3FS_CRC_OK;
  if (!d_values) return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  HIP_OR_FAIL(launch_finalize_values(d_values, n, (hipStream_t)stream));
  return HF3FS_CRC_OK;
}

int hf3fs_crc_create_batch(uint8_t type, const void* const* d_bufs, const uint64_t* d_lens,
                           const uint32_t* d_starts, uint32_t* d_out, uint64_t n, uint64_t max_len, void* stream) {
  if (!valid_type(type)) return fail(HF3FS_CRC_INVALID_ARG, "unknown checksum type %u", type);
  if (n == 0) return HF3FS_CRC_OK;
  if (!d_bufs || !d_lens || !d_out) return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  hipStream_t s = (hipStream_t)stream;
  if (type == kTypeNone) {
    HIP_OR_FAIL(launch_zero_words(d_out, n, s));
    return HF3FS_CRC_OK;
  }
  Context* c = nullptr;
  if (int rc = get_context(&c)) return rc;
  ListSource src{reinterpret_cast<const uint64_t*>(d_bufs), d_lens, d_starts, n, ~0u};
  if (options().list_runs.load()) {  // byte runs (option list_runs; the update pre hash's schedule)
    const uint32_t rep = std::max<uint32_t>(1, options().prehash_rep.load());  // runs per wave, as the pre hash
    const uint32_t nw = (uint32_t)c->cus * kWaves * rep;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(kRunBlocksMax, std::max<uint64_t>(1, n / 256));
    void* scr = nullptr;
    if (int rc = call_scratch(c, s, (blocks + 2 * (nw + 1)) * 8 + (nw + 1) * 4, &scr)) return rc;
    uint64_t* partial = (uint64_t*)scr;
    const ByteRuns runs{partial, (uint32_t*)(partial + blocks + 2 * (nw + 1)), partial + blocks, blocks, false, rep};
    HIP_OR_FAIL(launch_zero_words(d_out, n, s));
    return run_ranges_list(c, type, src, max_len, d_out, s, 0, nullptr, nullptr, nullptr, &runs);
  }
  return run_ranges_list(c, type, src, max_len, d_out, s);
}

int hf3fs_crc_create_strided(uint8_t type, const void* d_base, uint64_t stride, uint64_t len, uint64_t n,
                             uint32_t start, uint32_t* d_out, void* stream) {
  if (!valid_type(type)) return fail(HF3FS_CRC_INVALID_ARG, "unknown checksum type %u", type);
  if (n == 0) return HF3FS_CRC_OK;
  if ((!d_base && len) || !d_out) return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  hipStream_t s = (hipStream_t)stream;
  if (type == kTypeNone) {
    HIP_OR_FAIL(launch_zero_words(d_out, n, s));
    return HF3FS_CRC_OK;
  }
  Context* c = nullptr;
  if (int rc = get_context(&c)) return rc;
  // Equal-length buffers: whole buffers per wave (no shift, no memset) when
  // they divide evenly over the resident waves, else segments; never tickets
  // (uniform tasks balance statically; tickets cost ~1.3% here, A/B in
  // profiles/r01_ab_bulk.json).
  const uint64_t waves = (uint64_t)c->cus * kWaves;
  const bool whole = n % waves == 0 || n >= 8 * waves;
  Plan p = make_plan(c, n, len, whole ? std::max<uint64_t>(len, 1) : 0);
  StridedSource src{(uint64_t)d_base, stride, len, n, start};
  // Otherwise, for a large batch of long buffers: byte runs, every wave one exact share
  // (placed in closed form), instead of segments on a static stride: 1024 x 64 MiB (d4)
  // 10.43 -> 10.25 ms in one process (profiles/r05_d4_runs_probe.log).  More than
  // kRunWindowBytes per wave (batches past 16 GiB, whole buffers included): run_rep runs of
  // <= 4 MiB per wave, so the chip's reads sweep the batch in 16 GiB windows -- one 16 MiB run
  // per wave over a 64 GiB batch read at 6.68 TB/s against 6.95 for four 4 MiB tasks per wave
  // on the same bytes, and 4096 x 16 MiB whole buffers (the same wave -> address map as the
  // 64 MiB runs) at 6.72 (profiles/r06_d4_geometry.log).
  const uint64_t per_wave = n * len / waves;
  const uint32_t rep = per_wave > kRunWindowBytes ? (uint32_t)((per_wave + kRunWindowBytes - 1) / kRunWindowBytes) : 1u;
  const bool big = n < (1ull << 31) && n * len >= kRecordRunsBytes && len >= kRecordRunsMinLen;
  // (whole buffers of <= 4 MiB on their static stride sweep the batch in such windows already)
  const bool window = rep > 1 && !(whole && len <= kRunWindowBytes);
  if (big && ((!whole && p.segs > 1) || window) && (uint64_t)rep * waves < (1ull << 31)) {
    const uint32_t nv = (uint32_t)(rep * waves);  // runs
    void* scr = nullptr;
    if (int rc = call_scratch(c, s, (size_t)(nv + 1) * 12 + 64, &scr)) return rc;
    uint64_t* boff = (uint64_t*)scr;
    uint32_t* bal = (uint32_t*)(boff + nv + 1);
    HIP_OR_FAIL(launch_zero_words(d_out, n, s));  // the parts are xor-ed in
    HIP_OR_FAIL(launch_runs_uniform(n, len, nv, bal, boff, s));
    p.grid = (uint32_t)c->cus;
    p.queue = nullptr;
    p.bal = bal;
    p.boff = boff;
    p.run_rep = rep;
    HIP_OR_FAIL(launch_ranges_strided(type, src, p, d_out, c->tables, s));
    return HF3FS_CRC_OK;
  }
  if (int rc = launch_prepare(c, p, n, d_out, s)) return rc;
  p.queue = nullptr;
  HIP_OR_FAIL(launch_ranges_strided(type, src, p, d_out, c->tables, s));
  return HF3FS_CRC_OK;
}

static int verify_tail(Context* c, const uint32_t* computed, const uint32_t* d_expected, uint8_t* d_mismatch,
                       uint32_t* d_count, uint64_t n, hipStream_t s) {
  HIP_OR_FAIL(launch_zero_words(d_count, 1, s));
  HIP_OR_FAIL(launch_compare(computed, d_expected, d_mismatch, d_count, n, s));
  (void)c;
  return HF3FS_CRC_OK;
}

int hf3fs_crc_verify_batch(uint8_t type, const void* const* d_bufs, const uint64_t* d_lens,
                           const uint32_t* d_expected, uint8_t* d_mismatch, uint32_t* d_mismatch_count,
                           uint32_t* d_computed, uint64_t n, uint64_t max_len, void* stream) {
  if (!valid_type(type)) return fail(HF3FS_CRC_INVALID_ARG, "unknown checksum type %u", type);
  if (!d_mismatch_count) return fail(HF3FS_CRC_INVALID_ARG, "null mismatch count");
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) {
    HIP_OR_FAIL(launch_zero_words(d_mismatch_count, 1, s));
    return HF3FS_CRC_OK;
  }
  if (!d_expected || !d_mismatch) return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  Context* c = nullptr;
  if (int rc = get_context(&c)) return rc;
  uint32_t* comp = d_computed;
  if (!comp) {
    if (int rc = stream_scratch(c, s, n, &comp)) return rc;
  }
  if (int rc = hf3fs_crc_create_batch(type, d_bufs, d_lens, nullptr, comp, n, max_len, stream)) return rc;
  return verify_tail(c, comp, d_expected, d_mismatch, d_mismatch_count, n, s);
}

int hf3fs_crc_verify_strided(uint8_t type, const void* d_base, uint64_t stride, uint64_t len, uint64_t n,
                             const uint32_t* d_expected, uint8_t* d_mismatch, uint32_t* d_mismatch_count,
                             uint32_t* d_computed, void* stream) {
  if (!valid_type(type)) return fail(HF3FS_CRC_INVALID_ARG, "unknown checksum type %u", type);
  if (!d_mismatch_count) return fail(HF3FS_CRC_INVALID_ARG, "null mismatch count");
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) {
    HIP_OR_FAIL(launch_zero_words(d_mismatch_count, 1, s));
    return HF3FS_CRC_OK;
  }
  if (!d_expected || !d_mismatch) return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  Context* c = nullptr;
  if (int rc = get_context(&c)) return rc;
  uint32_t* comp = d_computed;
  if (!comp) {
    if (int rc = stream_scratch(c, s, n, &comp)) return rc;
  }
  if (int rc = hf3fs_crc_create_strided(type, d_base, stride, len, n, ~0u, comp, stream)) return rc;
  return verify_tail(c, comp, d_expected, d_mismatch, d_mismatch_count, n, s);
}

int hf3fs_crc_verify_blocks(uint8_t type, const void* d_arena, const uint64_t* d_offsets, const uint32_t* d_lens,
                            const uint32_t* d_expected, uint8_t* d_mismatch, uint32_t* d_mismatch_count,
                            uint32_t* d_computed, uint64_t n, uint32_t max_len, void* stream) {
  if (!valid_type(type)) return fail(HF3FS_CRC_INVALID_ARG, "unknown checksum type %u", type);
  if (!d_mismatch_count) return fail(HF3FS_CRC_INVALID_ARG, "null mismatch count");
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) {
    HIP_OR_FAIL(launch_zero_words(d_mismatch_count, 1, s));
    return HF3FS_CRC_OK;
  }
  if (!d_arena || !d_offsets || !d_lens || !d_expected || !d_mismatch)
    return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  Context* c = nullptr;
  if (int rc = get_context(&c)) return rc;
  uint32_t* comp = d_computed;
  if (!comp) {
    if (int rc = stream_scratch(c, s, n, &comp)) return rc;
  }
  if (type == kTypeNone) {
    HIP_OR_FAIL(launch_zero_words(comp, n, s));
  } else {
    Plan p = make_plan(c, n, max_len);
    if (int rc = launch_prepare(c, p, n, comp, s)) return rc;
    ArenaSource src{(uint64_t)d_arena, d_offsets, d_lens, n};
    if (int rc = plan_balance(c, p, src, n, max_len, s)) return rc;
    HIP_OR_FAIL(launch_ranges_arena(type, src, p, comp, c->tables, s));
  }
  return verify_tail(c, comp, d_expected, d_mismatch, d_mismatch_count, n, s);
}

int hf3fs_crc_combine_batch(uint8_t type, uint32_t* d_acc, const uint32_t* d_crc2, const uint64_t* d_len2,
                            uint64_t n, void* stream) {
  if (!valid_type(type)) return fail(HF3FS_CRC_INVALID_ARG, "unknown checksum type %u", type);
  if (n == 0 || type == kTypeNone) return HF3FS_CRC_OK;
  if (!d_acc || !d_crc2 || !d_len2) return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  Context* c = nullptr;
  if (int rc = get_context(&c)) return rc;
  HIP_OR_FAIL(launch_combine(type, d_acc, d_crc2, d_len2, n, c->tables, (hipStream_t)stream));
  return HF3FS_CRC_OK;
}

int hf3fs_crc_fill_synth(void* d_dst, uint64_t stride, uint64_t chunk_len, uint64_t n_chunks, uint64_t seed,
                         uint64_t first_chunk_id, void* stream) {
  if (!d_dst && n_chunks && chunk_len) return fail(HF3FS_CRC_INVALID_ARG, "null destination");
  if (((uint64_t)d_dst | stride) & 7) return fail(HF3FS_CRC_INVALID_ARG, "fill_synth needs 8-byte alignment");
  HIP_OR_FAIL(
      launch_fill_synth((uint8_t*)d_dst, stride, chunk_len, n_chunks, seed, first_chunk_id, (hipStream_t)stream));
  return HF3FS_CRC_OK;
}

// Pipeline per mode: DELTA runs the three streaming passes (pre hash, apply:
// the payload is read twice); REFERENCE the fused per-IO kernel (its prefix/suffix pass follows
// either way).  Option update_pipeline = unfused | fused forces one (A/B and the parity tests,
// which run both on every mode).  Apply pieces (three-pass pipeline): up to apply_pieces (8) per
// range, at least apply_min_kib (64 KiB) each (the tests cut finer).
void update_pipeline(int mode, bool* unfused, uint32_t* pieces, uint32_t* piece_min) {
  const Options& o = options();
  const int forced = o.update_pipeline.load();
  *unfused = forced < 0 ? mode == HF3FS_UPDATE_MODE_DELTA : forced == 0;
  *pieces = *unfused ? o.apply_pieces.load() : 0;  // only the three-pass pipeline has an apply pass
  *piece_min = o.apply_min_kib.load() << 10;
}

size_t hf3fs_crc_update_scratch_bytes(uint64_t n, int mode) {
  Context* c = nullptr;
  if (get_context(&c)) return 0;
  bool unfused = false;
  uint32_t pieces = 0, piece_min = 0;
  update_pipeline(mode, &unfused, &pieces, &piece_min);
  return update_scratch_bytes(n, pieces, (uint32_t)c->cus * kWaves, 0);
}

// The apply of a three-pass update call: one-shot (a workgroup per piece of
// 2^shift destination bytes) on a grid sized from the pair's previous call, or the ticketed
// tasks when no call has counted pieces yet (option apply_grid) or the piece table would be
// too large.
struct ApplyPlan {
  bool one_shot = false;
  uint32_t shift = 13;
  uint32_t grid = 0;
  uint64_t ptab_cap = 0;
  uint64_t* hint = nullptr;  // device view of the pair's pinned hint word
};
int plan_apply(Context* c, hipStream_t s, uint64_t n, uint32_t max_len, ApplyPlan* ap) {
  const Options& o = options();
  const uint32_t kib = o.apply_piece_kib.load();
  ap->shift = kib <= 4 ? 12 : kib <= 8 ? 13 : 14;
  ap->grid = (uint32_t)c->cus * 8;
  uint64_t* host = nullptr;
  if (int rc = c->hint_word(s, &host, &ap->hint)) return rc;
  const int mode = o.apply_grid.load();
  const uint64_t cap = update_piece_cap(n, max_len, ap->shift);
  if (mode == 0 || cap >= (1ull << 31) || cap * 4 > (1ull << 30)) return HF3FS_CRC_OK;  // tickets
  const uint64_t h = __atomic_load_n(host, __ATOMIC_ACQUIRE);
  const uint64_t prev_pieces = h >> 32, prev_n = h & 0xffffffffull;
  if (mode == 2) {  // test: a small grid, every workgroup loops over several pieces
    ap->grid = (uint32_t)c->cus;
  } else if (prev_n) {  // the previous call's pieces per IO, 3 % + 64 workgroups of headroom
    const uint64_t want = prev_pieces * n / prev_n;
    ap->grid = (uint32_t)std::min<uint64_t>(cap, std::max<uint64_t>(1, want + want / 32 + 64));
  } else if (mode < 0) {
    return HF3FS_CRC_OK;  // auto, first call of the pair: tickets (they count the pieces)
  }
  ap->one_shot = true;
  ap->ptab_cap = cap;
  return HF3FS_CRC_OK;
}

int hf3fs_crc_update_batch(uint8_t type, hf3fs_crc_update_io* d_ios, uint64_t n, uint32_t max_len, int mode,
                           void* stream) {
  if (!valid_type(type)) return fail(HF3FS_CRC_INVALID_ARG, "unknown checksum type %u", type);
  if (mode != HF3FS_UPDATE_MODE_REFERENCE && mode != HF3FS_UPDATE_MODE_DELTA)
    return fail(HF3FS_CRC_INVALID_ARG, "unknown update mode %d", mode);
  if (n == 0) return HF3FS_CRC_OK;
  if (!d_ios) return fail(HF3FS_CRC_INVALID_ARG, "null ios");
  Context* c = nullptr;
  if (int rc = get_context(&c)) return rc;
  hipStream_t s = (hipStream_t)stream;
  const uint8_t ktype = type == kTypeNone ? kTypeCrc32c : type;
  bool unfused = false;
  uint32_t pieces = 0, piece_min = 0;
  update_pipeline(mode, &unfused, &pieces, &piece_min);
  // Pre-hash task size: 512 KiB segments of the payload / old-byte jobs (A/B on d3 DELTA:
  // 1.766-1.772 ms per batch vs 1.788-1.797 at 256 KiB, 1.85 at 1 MiB; gpurun_out r03 seg sweep).
  constexpr uint64_t kPreSeg = 512 << 10;
  // pre-hash byte runs: prehash_rep runs per wave (option; Plan::run_rep)
  const uint32_t rep = std::max<uint32_t>(1, options().prehash_rep.load());
  const uint32_t nw = (uint32_t)c->cus * kWaves * rep;
  ApplyPlan ap;
  Context::Side side;
  if (unfused)
    if (int rc = plan_apply(c, s, n, max_len, &ap)) return rc;
  void* base = nullptr;
  if (int rc = call_scratch(c, s, update_scratch_bytes(n, pieces, nw, ap.ptab_cap), &base)) return rc;
  UpdateScratch sc;
  update_scratch_carve(base, n, pieces, piece_min, nw, ap.ptab_cap, &sc);
  sc.piece_shift = ap.shift;
  sc.one_shot = ap.one_shot ? 1u : 0u;
  sc.diag = c->diag;
  sc.runs_used = unfused;
  sc.fault_io = options().fault_io.load();
  // Pre hash as byte runs: every wave the same share of payload + old bytes, ranges split
  // anywhere (A/B vs 512 KiB tickets: 1.721-1.732 vs 1.726-1.738 ms per d3 DELTA batch).
  const bool prep_runs = 2 * n <= kPrepRunJobs;  // prep's runs workgroup places them (else launch_balance)
  const ByteRuns runs{sc.run_partial, sc.run_bal, sc.run_boff, sc.run_blocks, prep_runs, rep};
  // ONE zeroing launch: the job maxima, the task count and every ticket counter of this
  // call live in sc.ctl; prep zeroes the per-IO hash outputs itself.
  hipError_t e = launch_zero_words(sc.ctl, kCtlWords, s);
  if (e != hipSuccess) return fail(HF3FS_CRC_DEVICE_ERROR, "zero: %s", hipGetErrorString(e));
  if (!unfused) {  // one kernel: prep + payload verify + write (+ delta old-byte hash)
    e = launch_update_fused(d_ios, n, max_len, type, mode, sc, c->tables,
                            (uint32_t)std::min<uint64_t>(n, (uint64_t)c->cus), (int)options().apply_nt.load(), s);
    if (e != hipSuccess) return fail(HF3FS_CRC_DEVICE_ERROR, "update fused: %s", hipGetErrorString(e));
  } else {  // three passes: prep, the pre jobs through k_crc_ranges, apply (+ finalize of most IOs)
    e = launch_update_prep(d_ios, n, max_len, type, mode, sc, prep_runs, s);
    if (e != hipSuccess) return fail(HF3FS_CRC_DEVICE_ERROR, "update prep: %s", hipGetErrorString(e));
    ListSource pre{sc.pre_addr, sc.pre_len, sc.pre_start, 2 * n, 0u};
    if (int rc = run_ranges_list(c, ktype, pre, max_len, sc.pre_out, s, kPreSeg, sc.ctl + kCtlPreMax, nullptr,
                                 sc.ctl + kCtlQueuePre, &runs))
      return rc;
    if (ap.one_shot) {  // every verdict and every IO without a post job, beside the apply
      if (int rc = c->side_of(s, &side)) return rc;
      HIP_OR_FAIL(hipEventRecord(side.fork, s));
      HIP_OR_FAIL(hipStreamWaitEvent(side.side, side.fork, 0));
      e = launch_update_finalize(d_ios, n, type, mode, sc, c->tables, max_len, 1, false, side.side);
      if (e != hipSuccess) return fail(HF3FS_CRC_DEVICE_ERROR, "update finalize: %s", hipGetErrorString(e));
      HIP_OR_FAIL(hipEventRecord(side.join, side.side));
    }
    e = launch_update_apply(d_ios, n, max_len, type, mode, sc, c->tables, true, ap.grid,
                            (int)options().apply_nt.load(), ap.ptab_cap, ap.hint, s);
    if (e != hipSuccess) return fail(HF3FS_CRC_DEVICE_ERROR, "update apply: %s", hipGetErrorString(e));
  }
  ListSource post{sc.post_addr, sc.post_len, sc.post_start, 2 * n, 0u};
  if (int rc = run_ranges_list(c, ktype, post, max_len, sc.post_out, s, 256 << 10, sc.ctl + kCtlPostMax, nullptr,
                               sc.ctl + kCtlQueuePost))
    return rc;
  // the last launch also re-checks every payload it reports as mismatched (option audit)
  // the three-pass pipeline's verdicts came from the apply (ticketed) or the side stream
  // (one-shot): only the post-job IOs and the audit are left
  if (ap.one_shot) HIP_OR_FAIL(hipStreamWaitEvent(s, side.join, 0));
  e = launch_update_finalize(d_ios, n, type, mode, sc, c->tables, max_len, unfused ? 2 : 0,
                             options().audit.load() != 0, s);
  if (e != hipSuccess) return fail(HF3FS_CRC_DEVICE_ERROR, "update finalize: %s", hipGetErrorString(e));
  if (options().debug.load()) {  // diagnostics: job maxima and the first pre/post hashes
    uint32_t mx[2] = {0, 0}, pre[4] = {0, 0, 0, 0}, post[4] = {0, 0, 0, 0};
    uint64_t plen[4] = {0, 0, 0, 0};
    const size_t k = std::min<uint64_t>(4, 2 * n);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(mx, sc.ctl, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(pre, sc.pre_out, 4 * k, hipMemcpyDeviceToHost);
    (void)hipMemcpy(post, sc.post_out, 4 * k, hipMemcpyDeviceToHost);
    (void)hipMemcpy(plen, sc.pre_len, 8 * k, hipMemcpyDeviceToHost);
    fprintf(stderr, "[hf3fs_crc debug] update n=%llu mode=%d max=%u/%u pre=%08x,%08x len=%llu,%llu post=%08x,%08x\n",
            (unsigned long long)n, mode, mx[0], mx[1], pre[0], pre[1], (unsigned long long)plen[0],
            (unsigned long long)plen[1], post[0], post[1]);
  }
  return HF3FS_CRC_OK;
}

int hf3fs_crc_read_result_batch(uint8_t type, hf3fs_crc_read_io* d_ios, uint64_t n, uint32_t max_len,
                                void* stream) {
  if (type != kTypeCrc32c && type != kTypeCrc32) return fail(HF3FS_CRC_INVALID_ARG, "type must be CRC32C or CRC32");
  if (n == 0) return HF3FS_CRC_OK;
  if (!d_ios) return fail(HF3FS_CRC_INVALID_ARG, "null ios");
  Context* c = nullptr;
  if (int rc = get_context(&c)) return rc;
  hipStream_t s = (hipStream_t)stream;
  return run_record_jobs(
      c, type, n, max_len, ~0u, s,
      [&](uint64_t* addr, uint64_t* len, uint32_t* maxl) {
        return launch_read_prep(d_ios, n, type, max_len, addr, len, maxl, s);
      },
      [&](const uint32_t* v) { return launch_read_finalize(d_ios, n, v, s); }, "read");
}

int hf3fs_crc_scrub_batch(uint8_t type, hf3fs_crc_scrub_io* d_ios, uint64_t n, uint32_t max_len,
                          uint32_t* d_mismatch_count, void* stream) {
  if (type != kTypeCrc32c && type != kTypeCrc32) return fail(HF3FS_CRC_INVALID_ARG, "type must be CRC32C or CRC32");
  if (!d_mismatch_count) return fail(HF3FS_CRC_INVALID_ARG, "null mismatch count");
  hipStream_t s = (hipStream_t)stream;
  HIP_OR_FAIL(launch_zero_words(d_mismatch_count, 1, s));
  if (n == 0) return HF3FS_CRC_OK;
  if (!d_ios) return fail(HF3FS_CRC_INVALID_ARG, "null ios");
  Context* c = nullptr;
  if (int rc = get_context(&c)) return rc;
  return run_record_jobs(
      c, type, n, max_len, ~0u, s,
      [&](uint64_t* addr, uint64_t* len, uint32_t* maxl) {
        return launch_scrub_prep(d_ios, n, type, max_len, addr, len, maxl, s);
      },
      [&](const uint32_t* v) { return launch_scrub_finalize(d_ios, n, v, d_mismatch_count, s); }, "scrub", true);
}

int hf3fs_crc_frame_verify_batch(const void* d_buf, hf3fs_crc_frame* d_frames, uint64_t n, uint32_t max_size,
                                 uint32_t* d_mismatch_count, void* stream) {
  if (!d_mismatch_count) return fail(HF3FS_CRC_INVALID_ARG, "null mismatch count");
  hipStream_t s = (hipStream_t)stream;
  if (n == 0 || !d_frames || !d_buf || n >= (1ull << 31)) {  // (the map launch zeroes the count otherwise)
    HIP_OR_FAIL(launch_zero_words(d_mismatch_count, 1, s));
    if (n == 0) return HF3FS_CRC_OK;
    if (!d_frames || !d_buf) return fail(HF3FS_CRC_INVALID_ARG, "null argument");
    return fail(HF3FS_CRC_INVALID_ARG, "too many frames (%llu)", (unsigned long long)n);
  }
  Context* c = nullptr;
  if (int rc = get_context(&c)) return rc;
  const uint8_t* buf = (const uint8_t*)d_buf;
  // The stream path (frame_kernels.h) is tried for batches of walked frames;
  // the device falls back to one record job per frame when they are not sorted
  // and disjoint.  Option frame_stream = 0 / 1 forces it off / on (A/B).
  const Options& o = options();
  const int fs = o.frame_stream.load();
  const bool try_stream = fs < 0 ? n >= kFrameStreamMinFrames : fs != 0;
  const uint64_t waves = (uint64_t)c->cus * kWaves;
  const uint64_t segw = o.frame_segw.load();
  const uint64_t cap = try_stream ? frame_stream_cap(waves, segw) : 0;
  // scratch {flags[4], sums[2] (u64: payload bytes, gap bytes), ticket counter, (pad to 64 B),
  // addr[n], len[n], v[n], params, seg_first[cap], seg_lin[cap], seg_pre[cap]}; the stream path's
  // boundary values ev[2n] reuse addr (the record path's, idle then).  ONE zeroing launch: the
  // flags; the map launch zeroes the mismatch count and, on the record path, v.
  const size_t head = (4 * kFrameFlagWords + n * (8 + 8 + 4) + 63) / 64 * 64;
  const size_t bytes = head + sizeof(FrameStreamParams) + 12 * cap + 64;
  void* scratch = nullptr;
  if (int rc = call_scratch(c, s, bytes, &scratch)) return rc;
  uint8_t* base = (uint8_t*)scratch;
  uint32_t* flags = (uint32_t*)base;
  uint64_t* addr = (uint64_t*)(base + 4 * kFrameFlagWords);
  uint64_t* len = addr + n;
  uint32_t* v = (uint32_t*)(len + n);
  FrameStreamParams* prm = (FrameStreamParams*)(base + head);
  uint32_t* seg_first = (uint32_t*)(prm + 1);
  uint32_t* seg_lin = seg_first + cap;
  uint32_t* seg_pre = seg_lin + cap;
  uint32_t* ev = (uint32_t*)addr;
  int rc = HF3FS_CRC_OK;
  hipError_t e = launch_zero_words(flags, kFrameFlagWords, s);
  if (e == hipSuccess && try_stream) e = launch_frame_check(d_frames, n, max_size, flags, s);
  if (e == hipSuccess)
    e = launch_frame_map(buf, d_frames, n, segw * waves ? segw * waves : 1, waves, flags, prm, seg_first, max_size, addr,
                         len, v, d_mismatch_count, try_stream, s);
  if (e != hipSuccess) rc = fail(HF3FS_CRC_DEVICE_ERROR, "frame map: %s", hipGetErrorString(e));
  if (!rc) {  // record path (returns at once when the stream path took the batch); v and the
              // ticket counter (flags[8]) are zeroed already
    ListSource src{addr, len, nullptr, n, 0u};  // calcSerde hashes with init 0 (MessageHeader.h:35)
    rc = run_ranges_list(c, kTypeCrc32c, src, max_size, v, s, 0, flags, flags + 1, flags + 8);
  }
  if (!rc && try_stream) {
    e = launch_frame_stream(buf, d_frames, n, flags, prm, seg_first, seg_lin, ev, (uint32_t)c->cus, c->tables, s);
    if (e == hipSuccess) e = launch_frame_seg_scan(flags, prm, seg_lin, seg_pre, c->tables, s);
    if (e != hipSuccess) rc = fail(HF3FS_CRC_DEVICE_ERROR, "frame stream: %s", hipGetErrorString(e));
  }
  if (!rc) {
    e = launch_frame_finalize(buf, d_frames, n, v, flags, prm, ev, seg_lin, seg_pre, d_mismatch_count, c->tables, s);
    if (e != hipSuccess) rc = fail(HF3FS_CRC_DEVICE_ERROR, "frame finalize: %s", hipGetErrorString(e));
  }
  return rc;
}

int hf3fs_crc_file_digest_batch_ex(const hf3fs_crc_block_digest* d_blocks, const uint64_t* d_file_off,
                                   hf3fs_crc_file_digest* d_out, uint64_t n_files, uint64_t max_blocks, uint32_t flags,
                                   void* stream) {
  if (n_files == 0) return HF3FS_CRC_OK;
  if (!d_file_off || !d_out || (!d_blocks && max_blocks)) return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  if (flags & ~uint32_t(HF3FS_DIGEST_FILL_ZERO)) return fail(HF3FS_CRC_INVALID_ARG, "unknown flags %#x", flags);
  const bool fill_zero = flags & HF3FS_DIGEST_FILL_ZERO;
  const uint32_t splits = digest_splits(max_blocks);
  if (n_files * splits >= (1ull << 24)) return fail(HF3FS_CRC_INVALID_ARG, "too many files (%llu)",
                                                    (unsigned long long)n_files);
  Context* c = nullptr;
  if (int rc = get_context(&c)) return rc;
  hipStream_t s = (hipStream_t)stream;
  const size_t bytes = digest_scratch_bytes(n_files, splits, fill_zero);
  void* scratch = nullptr;
  if (bytes)
    if (int rc = call_scratch(c, s, bytes, &scratch)) return rc;
  hipError_t e =
      launch_file_digest(d_blocks, d_file_off, n_files, max_blocks, splits, fill_zero, scratch, d_out, c->tables, s);
  if (e != hipSuccess) return fail(HF3FS_CRC_DEVICE_ERROR, "file digest: %s", hipGetErrorString(e));
  return HF3FS_CRC_OK;
}

int hf3fs_crc_file_digest_batch(const hf3fs_crc_block_digest* d_blocks, const uint64_t* d_file_off,
                                hf3fs_crc_file_digest* d_out, uint64_t n_files, uint64_t max_blocks, void* stream) {
  return hf3fs_crc_file_digest_batch_ex(d_blocks, d_file_off, d_out, n_files, max_blocks, HF3FS_DIGEST_FILL_ZERO,
                                        stream);
}

// ---------------------------------------------------------------------------
// Host buffers: pieces of <= kStage bytes are packed into a pinned stage,
// copied H2D and hashed (start 0 -> linear CRC of the piece) on one of two
// streams while the next stage is packed; the pieces of each buffer are then
// stitched on the host with the combine algebra:
//   raw(buf, start) = start * x^(8 len) ^ sum_j lin(piece_j) * x^(8 * bytes after piece j).
}  // extern "C"
namespace {
int create_host_staged(Context* c, uint8_t type, const void* const* h_bufs, const uint64_t* h_lens,
                       const uint32_t* h_starts, uint32_t* h_out, uint64_t n);
}
extern "C" {
int hf3fs_crc_create_host(uint8_t type, const void* const* h_bufs, const uint64_t* h_lens, const uint32_t* h_starts,
                          uint32_t* h_out, uint64_t n) {
  if (!valid_type(type)) return fail(HF3FS_CRC_INVALID_ARG, "unknown checksum type %u", type);
  if (n == 0) return HF3FS_CRC_OK;
  if (!h_bufs || !h_lens || !h_out) return fail(HF3FS_CRC_INVALID_ARG, "null argument");
  if (type == kTypeNone) {
    for (uint64_t i = 0; i < n; ++i) h_out[i] = 0;
    return HF3FS_CRC_OK;
  }
  Context* c = nullptr;
  if (int rc = get_context(&c)) return rc;
  std::lock_guard<std::mutex> lk(c->stage_mu);
  // An error return must not leave copies in flight into the pinned stages the
  // next call refills: drain both staging streams first.
  const int rc = create_host_staged(c, type, h_bufs, h_lens, h_starts, h_out, n);
  if (rc != HF3FS_CRC_OK)
    for (int k = 0; k < 2; ++k)
      if (c->streams[k]) (void)hipStreamSynchronize(c->streams[k]);
  return rc;
}

}  // extern "C"

namespace {
int create_host_staged(Context* c, uint8_t type, const void* const* h_bufs, const uint64_t* h_lens,
                       const uint32_t* h_starts, uint32_t* h_out, uint64_t n) {
  constexpr size_t kStage = Context::kStage;
  constexpr size_t kMaxPieces = 4096;
  if (!c->pinned[0]) {
    for (int k = 0; k < 2; ++k) {
      HIP_OR_FAIL(hipHostMalloc((void**)&c->pinned[k], kStage, hipHostMallocDefault));
      HIP_OR_FAIL(hipHostMalloc((void**)&c->pdesc[k], kMaxPieces * 5 * sizeof(uint64_t), hipHostMallocDefault));
      HIP_OR_FAIL(hipMalloc(&c->dstage[k], kStage));
      HIP_OR_FAIL(hipMalloc(&c->ddesc[k], kMaxPieces * 5 * sizeof(uint64_t)));
      HIP_OR_FAIL(hipStreamCreateWithFlags(&c->streams[k], hipStreamNonBlocking));
    }
  }
  const uint32_t poly = poly_of(type);
  for (uint64_t i = 0; i < n; ++i) h_out[i] = gf_mul(h_starts ? h_starts[i] : ~0u, xpow_bits(8 * h_lens[i], poly), poly);

  struct Piece {
    uint64_t buf, tail;  // buffer index, bytes after the piece in its buffer
  };
  std::vector<Piece> pieces[2];
  uint64_t npieces[2] = {0, 0};
  bool busy[2] = {false, false};
  int k = 0;
  uint64_t bi = 0, boff = 0;
  auto drain = [&](int slot) -> int {
    if (!busy[slot]) return HF3FS_CRC_OK;
    HIP_OR_FAIL(hipStreamSynchronize(c->streams[slot]));
    const uint32_t* res = reinterpret_cast<const uint32_t*>(c->pdesc[slot] + 4 * kMaxPieces);
    for (uint64_t j = 0; j < npieces[slot]; ++j) {
      const Piece& pc = pieces[slot][j];
      h_out[pc.buf] ^= gf_mul(res[j], xpow_bits(8 * pc.tail, poly), poly);
    }
    busy[slot] = false;
    return HF3FS_CRC_OK;
  };
  while (bi < n) {
    if (int rc = drain(k)) return rc;
    pieces[k].clear();
    uint64_t used = 0, np = 0;
    uint64_t* addrs = c->pdesc[k];
    uint64_t* lens = c->pdesc[k] + kMaxPieces;
    while (bi < n && np < kMaxPieces && used < kStage) {
      const uint64_t len = h_lens[bi];
      if (boff >= len) {
        ++bi;
        boff = 0;
        continue;
      }
      const uint64_t take = std::min<uint64_t>(len - boff, kStage - used);
      memcpy(c->pinned[k] + used, (const uint8_t*)h_bufs[bi] + boff, take);
      addrs[np] = (uint64_t)(c->dstage[k] + used);
      lens[np] = take;
      pieces[k].push_back({bi, len - boff - take});
      ++np;
      used = (used + take + 15) & ~uint64_t(15);
      boff += take;
    }
    if (np == 0) break;
    npieces[k] = np;
    hipStream_t s = c->streams[k];
    HIP_OR_FAIL(hipMemcpyAsync(c->dstage[k], c->pinned[k], std::min<uint64_t>(used, kStage), hipMemcpyHostToDevice, s));
    HIP_OR_FAIL(hipMemcpyAsync(c->ddesc[k], c->pdesc[k], 2 * kMaxPieces * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    uint32_t* dout = reinterpret_cast<uint32_t*>(c->ddesc[k] + 4 * kMaxPieces);
    ListSource src{c->ddesc[k], c->ddesc[k] + kMaxPieces, nullptr, np, 0u};
    if (int rc = run_ranges_list(c, type, src, kStage, dout, s)) return rc;
    HIP_OR_FAIL(hipMemcpyAsync(c->pdesc[k] + 4 * kMaxPieces, dout, np * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    busy[k] = true;
    k ^= 1;
  }
  if (int rc = drain(0)) return rc;
  if (int rc = drain(1)) return rc;
  return HF3FS_CRC_OK;
}
}  // namespace
