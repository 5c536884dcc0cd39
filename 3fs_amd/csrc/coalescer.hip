// coalescer.hip -- batches concurrent per-IO ChecksumInfo::create calls into
// one device launch.
//
// The reference hashes one IO at a time on the thread that completes it: 32
// AioReadWorker threads call AioReadJob::setResult per read
// (src/storage/aio/BatchReadJob.cc:24-35, AioReadWorker.h:27), 32 UpdateWorker
// threads verify each write (src/storage/store/ChunkReplica.cc:193-207,
// UpdateWorker.h:15), and client coroutines create/verify per IO
// (src/client/storage/StorageClientImpl.cc:1720-1737,1878-1882).  A GPU launch
// per IO would cost more than the CRC of a 4-64 KiB block, so callers submit
// single requests here and a launcher thread turns everything that arrived
// while the previous batch was on the device into one hf3fs_crc_create_batch
// launch (Nagle-style: an idle device launches at once, a busy one lets the
// next batch grow).
//
// Request bytes are either device-accessible already (HBM, or host memory
// registered with hf3fs_crc_host_register, e.g. 3FS's RDMA BufferPool slabs,
// src/storage/service/BufferPool.h:24-27) or plain host memory that the caller
// thread copies into the open slot's pinned stage, which the kernel reads in
// place over PCIe.  Descriptors live in pinned memory read by the kernel too,
// so a batch costs one launch + one 4 B/IO device-to-host copy.
//
// Threads: submitters (any number) -> launcher (1) -> completer (1, runs the
// callbacks in launch order).  One mutex guards the slot ring.
//
// Service mode (options.service_wgs > 0): CRC32C requests skip the launch
// altogether.  A submitter takes a ticket, writes its request into ring slot
// ticket % ring (pinned coherent host memory) and publishes that slot alone
// (seq = ticket + 1, stored last) -- no submitter ever waits for another one.
// `service_wgs` resident workgroups of k_crc_service serve the tickets
// round-robin (ticket t by workgroup t % service_wgs, no claim protocol),
// hash each request with all 16 waves of the workgroup and write
// value + done back to host memory, where the submitter (or, for callbacks,
// the service completer thread) spins on it.  The kernel exits after
// service_idle_us without requests; whoever waits on a request relaunches it
// when it has exited.  Every host-side spin is bounded: a request not served
// within kServiceTimeout fails the service for good (its state is dumped to
// stderr) instead of hanging the callers.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <immintrin.h>

#include "../../include/hf3fs_crc.h"
#include "crc_kernels.h"
#include "internal.h"

namespace {

using Clock = std::chrono::steady_clock;
constexpr auto kServiceTimeout = std::chrono::seconds(10);
constexpr auto kServiceCheckEvery = std::chrono::microseconds(20);  // relaunch check from submitters

struct Waiter {
  hf3fs_crc_done_fn fn;
  void* arg;
};

// Requests of one checksum type inside a slot.
struct Sub {
  uint64_t* addr = nullptr;  // pinned + mapped: written by submitters, read by the kernel
  uint64_t* len = nullptr;
  uint32_t* start = nullptr;
  uint64_t* daddr = nullptr;  // device views of the same pinned words
  uint64_t* dlen = nullptr;
  uint32_t* dstart = nullptr;
  uint32_t* dout = nullptr;  // device
  uint32_t* hout = nullptr;  // pinned
  std::vector<Waiter> waiters;
  uint32_t count = 0;
  uint64_t max_len = 0;
};

enum class SlotState { kFree, kOpen, kFlying };

struct Slot {
  Sub sub[2];  // [0] CRC32C, [1] CRC32
  uint8_t* stage = nullptr;   // pinned staging for HF3FS_CRC_REQ_HOST_COPY requests
  uint8_t* dstage = nullptr;  // its device view
  uint64_t stage_used = 0;
  int writers = 0;  // submitters still copying into the stage
  bool sealed = false;
  SlotState state = SlotState::kFree;
  Clock::time_point first;
  hipEvent_t done = nullptr;
  int rc = HF3FS_CRC_OK;
  uint32_t total() const { return sub[0].count + sub[1].count; }
};

struct SyncWait {
  std::mutex m;
  std::condition_variable cv;
  std::atomic<int> done{0};
  int status = 0;
  uint32_t value = 0;
};

void sync_done(void* arg, int status, uint32_t value) {
  auto* w = static_cast<SyncWait*>(arg);
  std::lock_guard<std::mutex> lk(w->m);
  w->status = status;
  w->value = value;
  w->done.store(1, std::memory_order_release);
  w->cv.notify_one();
}

// Request ring served by the persistent kernel (service mode).
struct Service {
  uint32_t ring = 0, mask = 0, wgs = 0;
  uint64_t slot_stage = 0, idle_ticks = 0;
  hf3fs_crc::ServiceReq* req = nullptr;  // pinned, coherent, mapped
  hf3fs_crc::ServiceResp* resp = nullptr;
  hf3fs_crc::ServiceCtrl* ctrl = nullptr;
  hf3fs_crc::ServiceReq* dreq = nullptr;  // device views
  hf3fs_crc::ServiceResp* dresp = nullptr;
  hf3fs_crc::ServiceCtrl* dctrl = nullptr;
  uint8_t* stage = nullptr;  // ring x slot_stage, pinned coherent
  uint8_t* dstage = nullptr;
  uint32_t* dnext = nullptr;  // device, per workgroup: its next ticket (persists across launches)
  std::vector<std::atomic<uint32_t>> ack;  // ticket + 1 once the consumer read the slot's result
  std::vector<Waiter> cbs;
  std::atomic<uint64_t> reserve{0};
  const hf3fs_crc::DeviceTables* tables = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t ev = nullptr;
  std::mutex launch_mu;
  std::atomic<int64_t> last_check{0};  // steady-clock ns of the last relaunch check
  std::atomic<int> failed{0};  // launch error or lost request: service requests fail instead of waiting forever
  std::atomic<uint64_t> launches{0};
  // async requests, completed by the service completer thread
  std::mutex q_mu;
  std::condition_variable q_cv;
  std::deque<uint64_t> q;
  bool q_stop = false;
  std::thread completer;
};

}  // namespace

struct hf3fs_crc_coalescer {
  hf3fs_crc_coalescer_options opt{};
  hipStream_t stream = nullptr;
  std::vector<Slot> slots;
  std::mutex mu;
  std::condition_variable cv_launch;  // launcher waits here
  std::condition_variable cv_fill;    // submitters wait for room
  std::condition_variable cv_fly;     // completer waits for launched slots
  int open = -1;                      // slot being filled (-1: none free)
  std::deque<int> fly;                // launched slots, in launch order
  bool stop = false;
  bool launcher_done = false;
  std::thread launcher, completer;
  // stats
  uint64_t n_requests = 0, n_batches = 0, n_bytes = 0, max_batch_seen = 0;
  std::atomic<uint64_t> n_service{0};
  Service* svc = nullptr;

  int init();
  void teardown();
  int submit(uint8_t type, const void* addr, uint64_t len, uint32_t start, uint32_t flags, hf3fs_crc_done_fn fn,
             void* arg);
  void launcher_loop();
  void completer_loop();
  int launch(Slot& s);
  bool ready_locked(Clock::time_point now) const;
  void open_next_locked();
  // service mode
  int service_init();
  void service_teardown();
  bool service_eligible(uint8_t type, uint64_t len, uint32_t flags) const;
  int service_submit(const void* addr, uint64_t len, uint32_t start, uint32_t flags, hf3fs_crc_done_fn fn, void* arg,
                     uint64_t* ticket);
  int service_wait(uint64_t ticket, uint32_t* value);
  void service_ensure_running(bool force_check);
  void service_completer_loop();
  void service_dump(const char* where, uint64_t ticket);
};

namespace {

int cfail(int code, const char* msg, hipError_t e = hipSuccess) {
  std::string m = msg;
  if (e != hipSuccess) {
    m += ": ";
    m += hipGetErrorString(e);
  }
  return hf3fs_crc::set_error(code, m.c_str());
}

#define CO_HIP(expr)                                                      \
  do {                                                                    \
    hipError_t _e = (expr);                                               \
    if (_e != hipSuccess) return cfail(HF3FS_CRC_DEVICE_ERROR, #expr, _e); \
  } while (0)

template <class T>
int pinned_alloc(T** host, T** dev, size_t count) {
  CO_HIP(hipHostMalloc((void**)host, count * sizeof(T), hipHostMallocMapped));
  CO_HIP(hipHostGetDevicePointer((void**)dev, *host, 0));
  return HF3FS_CRC_OK;
}

}  // namespace

int hf3fs_crc_coalescer::init() {
  CO_HIP(hipSetDevice(opt.device));
  CO_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  slots.resize(opt.slots);
  for (auto& s : slots) {
    for (auto& b : s.sub) {
      if (int rc = pinned_alloc(&b.addr, &b.daddr, opt.max_batch)) return rc;
      if (int rc = pinned_alloc(&b.len, &b.dlen, opt.max_batch)) return rc;
      if (int rc = pinned_alloc(&b.start, &b.dstart, opt.max_batch)) return rc;
      CO_HIP(hipHostMalloc((void**)&b.hout, opt.max_batch * sizeof(uint32_t), hipHostMallocDefault));
      CO_HIP(hipMalloc((void**)&b.dout, opt.max_batch * sizeof(uint32_t)));
      b.waiters.reserve(opt.max_batch);
    }
    if (opt.stage_bytes)
      if (int rc = pinned_alloc(&s.stage, &s.dstage, opt.stage_bytes)) return rc;
    CO_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
  }
  open = 0;
  slots[0].state = SlotState::kOpen;
  launcher = std::thread([this] { launcher_loop(); });
  completer = std::thread([this] { completer_loop(); });
  if (opt.service_wgs) return service_init();
  return HF3FS_CRC_OK;
}

void hf3fs_crc_coalescer::teardown() {
  service_teardown();
  {
    std::lock_guard<std::mutex> lk(mu);
    stop = true;
  }
  cv_launch.notify_all();
  cv_fly.notify_all();
  cv_fill.notify_all();
  if (launcher.joinable()) launcher.join();
  if (completer.joinable()) completer.join();
  (void)hipSetDevice(opt.device);
  for (auto& s : slots) {
    for (auto& b : s.sub) {
      if (b.addr) (void)hipHostFree(b.addr);
      if (b.len) (void)hipHostFree(b.len);
      if (b.start) (void)hipHostFree(b.start);
      if (b.hout) (void)hipHostFree(b.hout);
      if (b.dout) (void)hipFree(b.dout);
    }
    if (s.stage) (void)hipHostFree(s.stage);
    if (s.done) (void)hipEventDestroy(s.done);
  }
  if (stream) (void)hipStreamDestroy(stream);
}

void hf3fs_crc_coalescer::open_next_locked() {
  open = -1;
  for (size_t i = 0; i < slots.size(); ++i)
    if (slots[i].state == SlotState::kFree) {
      open = (int)i;
      slots[i].state = SlotState::kOpen;
      return;
    }
}

int hf3fs_crc_coalescer::submit(uint8_t type, const void* addr, uint64_t len, uint32_t start, uint32_t flags,
                                hf3fs_crc_done_fn fn, void* arg) {
  if (type != HF3FS_CHECKSUM_NONE && type != HF3FS_CHECKSUM_CRC32C && type != HF3FS_CHECKSUM_CRC32)
    return cfail(HF3FS_CRC_INVALID_ARG, "unknown checksum type");
  if (!fn) return cfail(HF3FS_CRC_INVALID_ARG, "null callback");
  if (flags & ~uint32_t(HF3FS_CRC_REQ_HOST_COPY)) return cfail(HF3FS_CRC_INVALID_ARG, "unknown request flags");
  // create's special cases need no bytes (Common.h:150, :157-171 with an empty iterator)
  if (type == HF3FS_CHECKSUM_NONE) {
    fn(arg, HF3FS_CRC_OK, 0);
    return HF3FS_CRC_OK;
  }
  if (len == 0) {
    fn(arg, HF3FS_CRC_OK, start);
    return HF3FS_CRC_OK;
  }
  if (!addr) return cfail(HF3FS_CRC_INVALID_ARG, "null buffer");
  if (service_eligible(type, len, flags)) {
    uint64_t t = 0;
    return service_submit(addr, len, start, flags, fn, arg, &t);
  }
  const bool copy = flags & HF3FS_CRC_REQ_HOST_COPY;
  const uint64_t need = copy ? (len + 15) & ~uint64_t(15) : 0;
  if (copy && need > opt.stage_bytes) {
    // Larger than a stage: hash it through the synchronous staged host path
    // (still on the device), on the coalescer's device.
    int prev = 0;
    CO_HIP(hipGetDevice(&prev));
    CO_HIP(hipSetDevice(opt.device));
    uint32_t out = 0;
    int rc = hf3fs_crc_create_host(type, &addr, &len, &start, &out, 1);
    (void)hipSetDevice(prev);
    if (rc) return rc;
    fn(arg, HF3FS_CRC_OK, out);
    return HF3FS_CRC_OK;
  }
  const int t = type == HF3FS_CHECKSUM_CRC32 ? 1 : 0;
  std::unique_lock<std::mutex> lk(mu);
  Slot* s = nullptr;
  for (;;) {
    if (stop) return cfail(HF3FS_CRC_INVALID_ARG, "coalescer is shutting down");
    if (open >= 0) {
      Slot& o = slots[open];
      if (!o.sealed && o.sub[t].count < opt.max_batch && o.stage_used + need <= opt.stage_bytes) {
        s = &o;
        break;
      }
      if (!o.sealed) {  // full: launch it as soon as its copies land
        o.sealed = true;
        cv_launch.notify_one();
      }
    }
    cv_fill.wait(lk);
  }
  Sub& b = s->sub[t];
  const uint32_t i = b.count++;
  uint8_t* dst = nullptr;
  if (copy) {
    dst = s->stage + s->stage_used;
    b.addr[i] = (uint64_t)(s->dstage + s->stage_used);
    s->stage_used += need;
    ++s->writers;
  } else {
    b.addr[i] = (uint64_t)addr;
  }
  b.len[i] = len;
  b.start[i] = start;
  b.waiters.push_back({fn, arg});
  if (len > b.max_len) b.max_len = len;
  if (s->total() == 1) s->first = Clock::now();
  ++n_requests;
  n_bytes += len;
  if (b.count == opt.max_batch) s->sealed = true;
  if (copy) {
    lk.unlock();
    std::memcpy(dst, addr, len);
    lk.lock();
    --s->writers;
  }
  lk.unlock();
  cv_launch.notify_one();
  return HF3FS_CRC_OK;
}

// Launch the open slot when it has work whose bytes have all landed, and
// either it is full, the device has fewer than `inflight` batches, or the
// oldest request waited max_wait_us.
bool hf3fs_crc_coalescer::ready_locked(Clock::time_point now) const {
  if (open < 0) return false;
  const Slot& s = slots[open];
  if (s.total() == 0 || s.writers) return false;
  if (s.sealed || stop) return true;
  if (fly.size() >= opt.inflight) return false;
  return now - s.first >= std::chrono::microseconds(opt.max_wait_us);
}

void hf3fs_crc_coalescer::launcher_loop() {
  (void)hipSetDevice(opt.device);
  std::unique_lock<std::mutex> lk(mu);
  for (;;) {
    Clock::time_point now = Clock::now();
    if (!ready_locked(now)) {
      if (stop && (open < 0 || slots[open].total() == 0)) break;
      if (open >= 0 && slots[open].total() && !slots[open].writers && fly.size() < opt.inflight)
        cv_launch.wait_until(lk, slots[open].first + std::chrono::microseconds(opt.max_wait_us));
      else
        cv_launch.wait(lk);
      continue;
    }
    const int si = open;
    Slot& s = slots[si];
    s.state = SlotState::kFlying;
    open_next_locked();
    ++n_batches;
    if (s.total() > max_batch_seen) max_batch_seen = s.total();
    lk.unlock();
    cv_fill.notify_all();  // a fresh slot may be open now
    s.rc = launch(s);
    lk.lock();
    fly.push_back(si);
    cv_fly.notify_one();
  }
  launcher_done = true;
  lk.unlock();
  cv_fly.notify_all();
}

int hf3fs_crc_coalescer::launch(Slot& s) {
  for (int t = 0; t < 2; ++t) {
    Sub& b = s.sub[t];
    if (!b.count) continue;
    const uint8_t type = t ? HF3FS_CHECKSUM_CRC32 : HF3FS_CHECKSUM_CRC32C;
    int rc = hf3fs_crc_create_batch(type, (const void* const*)b.daddr, b.dlen, b.dstart, b.dout, b.count, b.max_len,
                                    stream);
    if (rc) return rc;
    CO_HIP(hipMemcpyAsync(b.hout, b.dout, b.count * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
  }
  CO_HIP(hipEventRecord(s.done, stream));
  return HF3FS_CRC_OK;
}

void hf3fs_crc_coalescer::completer_loop() {
  (void)hipSetDevice(opt.device);
  std::unique_lock<std::mutex> lk(mu);
  for (;;) {
    cv_fly.wait(lk, [&] { return !fly.empty() || launcher_done; });
    if (fly.empty()) break;  // launcher finished and everything completed
    const int si = fly.front();
    Slot& s = slots[si];
    lk.unlock();
    int rc = s.rc;
    if (rc == HF3FS_CRC_OK) {
      if (hipEventSynchronize(s.done) != hipSuccess) rc = HF3FS_CRC_DEVICE_ERROR;
    } else {
      (void)hipStreamSynchronize(stream);  // a partly launched batch must finish before its slot is reused
    }
    for (auto& b : s.sub) {
      for (uint32_t i = 0; i < b.count; ++i) b.waiters[i].fn(b.waiters[i].arg, rc, rc ? 0u : b.hout[i]);
      b.waiters.clear();
      b.count = 0;
      b.max_len = 0;
    }
    lk.lock();
    s.stage_used = 0;
    s.sealed = false;
    s.rc = HF3FS_CRC_OK;
    s.state = SlotState::kFree;
    fly.pop_front();
    if (open < 0) open_next_locked();
    cv_fill.notify_all();
    cv_launch.notify_one();
  }
}

// ---------------------------------------------------------------------------
// service mode
namespace {
inline void cpu_relax() { _mm_pause(); }
inline int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}
template <class T>
int coherent_alloc(T** host, T** dev, size_t count) {
  CO_HIP(hipHostMalloc((void**)host, count * sizeof(T), hipHostMallocMapped | hipHostMallocCoherent));
  CO_HIP(hipHostGetDevicePointer((void**)dev, *host, 0));
  memset((void*)*host, 0, count * sizeof(T));
  return HF3FS_CRC_OK;
}

// Bounded spin of a service-mode waiter: now and then it relaunches an exited
// service kernel and yields (a waiter must never starve the thread whose
// request it waits behind), and it gives up -- failing the service for good
// -- when its request has not been served for kServiceTimeout.
struct Spin {
  uint32_t k = 0;
  Clock::time_point since{};
  int step(hf3fs_crc_coalescer* co, uint64_t ticket, const char* where) {
    cpu_relax();
    if ((++k & 255) != 0) return HF3FS_CRC_OK;
    co->service_ensure_running(true);
    Service* v = co->svc;
    if (int rc = v->failed.load(std::memory_order_acquire)) return cfail(rc, "coalescer service has failed");
    const Clock::time_point now = Clock::now();
    if (since == Clock::time_point{}) {
      since = now;
    } else if (now - since > kServiceTimeout) {
      co->service_dump(where, ticket);
      v->failed.store(HF3FS_CRC_DEVICE_ERROR, std::memory_order_release);
      return cfail(HF3FS_CRC_DEVICE_ERROR, "coalescer service: request not served in time");
    }
    std::this_thread::yield();
    return HF3FS_CRC_OK;
  }
};
}  // namespace

int hf3fs_crc_coalescer::service_init() {
  auto* v = new Service();
  svc = v;
  v->ring = opt.service_ring;
  v->mask = v->ring - 1;
  v->wgs = opt.service_wgs;
  v->slot_stage = (opt.service_stage + 15) & ~uint64_t(15);
  v->ack = std::vector<std::atomic<uint32_t>>(v->ring);
  for (auto& a : v->ack) a.store(0, std::memory_order_relaxed);
  v->cbs.resize(v->ring);
  if (int rc = coherent_alloc(&v->req, &v->dreq, v->ring)) return rc;
  if (int rc = coherent_alloc(&v->resp, &v->dresp, v->ring)) return rc;
  if (int rc = coherent_alloc(&v->ctrl, &v->dctrl, 1)) return rc;
  if (v->slot_stage)
    if (int rc = coherent_alloc(&v->stage, &v->dstage, v->ring * v->slot_stage)) return rc;
  {  // workgroup w serves tickets w, w + wgs, ...
    std::vector<uint32_t> first(v->wgs);
    for (uint32_t w = 0; w < v->wgs; ++w) first[w] = w;
    CO_HIP(hipMalloc((void**)&v->dnext, v->wgs * sizeof(uint32_t)));
    CO_HIP(hipMemcpy(v->dnext, first.data(), v->wgs * sizeof(uint32_t), hipMemcpyHostToDevice));
  }
  int khz = 0;
  CO_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, opt.device));
  v->idle_ticks = (uint64_t)opt.service_idle_us * (uint64_t)(khz > 0 ? khz : 100000) / 1000;
  if (int rc = hf3fs_crc::current_tables(&v->tables)) return rc;
  CO_HIP(hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking));
  CO_HIP(hipEventCreateWithFlags(&v->ev, hipEventDisableTiming));
  CO_HIP(hipDeviceSynchronize());
  v->completer = std::thread([this] { service_completer_loop(); });
  service_ensure_running(true);
  if (v->failed.load()) return HF3FS_CRC_DEVICE_ERROR;  // message recorded by service_ensure_running
  return HF3FS_CRC_OK;
}

// Relaunch the service kernel when the previous launch has exited (idle
// timeout).  Without force_check, at most one check per kServiceCheckEvery.
void hf3fs_crc_coalescer::service_ensure_running(bool force_check) {
  Service* v = svc;
  if (v->failed.load(std::memory_order_relaxed)) return;
  const int64_t now = now_ns();
  if (!force_check &&
      now - v->last_check.load(std::memory_order_relaxed) <
          std::chrono::duration_cast<std::chrono::nanoseconds>(kServiceCheckEvery).count())
    return;
  std::unique_lock<std::mutex> lk(v->launch_mu, std::try_to_lock);
  if (!lk.owns_lock()) return;  // another thread is on it
  v->last_check.store(now, std::memory_order_relaxed);
  if (hipEventQuery(v->ev) != hipSuccess) return;  // still running
  (void)hipSetDevice(opt.device);
  __atomic_store_n(&v->ctrl->stop, 0u, __ATOMIC_RELEASE);
  hf3fs_crc::ServiceArgs a{v->dreq, v->dresp, v->dctrl, v->dnext, v->ring, v->idle_ticks};
  hipError_t e = hf3fs_crc::launch_service(a, v->wgs, v->tables, v->stream);
  if (e == hipSuccess) e = hipEventRecord(v->ev, v->stream);
  if (e != hipSuccess) {
    // nobody would ever serve the ring: fail every service request from now on
    cfail(HF3FS_CRC_DEVICE_ERROR, "coalescer service kernel launch", e);
    std::fprintf(stderr, "hf3fs_crc coalescer service: launch failed: %s\n", hipGetErrorString(e));
    v->failed.store(HF3FS_CRC_DEVICE_ERROR, std::memory_order_release);
    return;
  }
  v->launches.fetch_add(1, std::memory_order_relaxed);
}

// What a request that was not served in time saw (stderr).
void hf3fs_crc_coalescer::service_dump(const char* where, uint64_t t) {
  Service* v = svc;
  const uint32_t slot = (uint32_t)t & v->mask;
  const hf3fs_crc::ServiceCtrl* c = v->ctrl;
  std::fprintf(stderr,
               "hf3fs_crc coalescer service: %s: ticket %llu slot %u seq %u resp.done %u | reserved %llu "
               "launches %llu event %d | device at its last exit: reason %u ticket %u seq %u\n",
               where, (unsigned long long)t, slot, __atomic_load_n(&v->req[slot].seq, __ATOMIC_ACQUIRE),
               __atomic_load_n(&v->resp[slot].done, __ATOMIC_ACQUIRE), (unsigned long long)v->reserve.load(),
               (unsigned long long)v->launches.load(), (int)hipEventQuery(v->ev),
               __atomic_load_n(&c->dbg_exit, __ATOMIC_ACQUIRE), __atomic_load_n(&c->dbg_ticket, __ATOMIC_ACQUIRE),
               __atomic_load_n(&c->dbg_seq, __ATOMIC_ACQUIRE));
}

bool hf3fs_crc_coalescer::service_eligible(uint8_t type, uint64_t len, uint32_t flags) const {
  if (!svc || type != HF3FS_CHECKSUM_CRC32C || len == 0) return false;
  return !(flags & HF3FS_CRC_REQ_HOST_COPY) || len <= svc->slot_stage;
}

int hf3fs_crc_coalescer::service_submit(const void* addr, uint64_t len, uint32_t start, uint32_t flags,
                                        hf3fs_crc_done_fn fn, void* arg, uint64_t* ticket) {
  Service* v = svc;
  if (int rc = v->failed.load(std::memory_order_acquire)) return cfail(rc, "coalescer service has failed");
  const uint64_t t = v->reserve.fetch_add(1, std::memory_order_relaxed);
  const uint32_t slot = (uint32_t)t & v->mask;
  // the slot's previous ticket must have been consumed
  if (t >= v->ring) {
    const uint32_t prev = (uint32_t)(t - v->ring + 1);
    Spin spin;
    while (v->ack[slot].load(std::memory_order_acquire) != prev)
      if (int rc = spin.step(this, t, "slot reuse")) return rc;
  }
  uint64_t a = (uint64_t)addr;
  if (flags & HF3FS_CRC_REQ_HOST_COPY) {
    std::memcpy(v->stage + (uint64_t)slot * v->slot_stage, addr, len);
    a = (uint64_t)(v->dstage + (uint64_t)slot * v->slot_stage);
  }
  hf3fs_crc::ServiceReq& r = v->req[slot];
  r.addr = a;
  r.len = len;
  r.start = start;
  v->cbs[slot] = Waiter{fn, arg};
  __atomic_store_n(&r.seq, (uint32_t)(t + 1), __ATOMIC_RELEASE);  // publish this slot
  if (fn) {
    {
      std::lock_guard<std::mutex> lk(v->q_mu);
      v->q.push_back(t);
    }
    v->q_cv.notify_one();
  }
  service_ensure_running(false);
  n_service.fetch_add(1, std::memory_order_relaxed);
  *ticket = t;
  return HF3FS_CRC_OK;
}

// Spin until the service published the ticket's result, then release the slot.
int hf3fs_crc_coalescer::service_wait(uint64_t t, uint32_t* value) {
  Service* v = svc;
  const uint32_t slot = (uint32_t)t & v->mask;
  const uint32_t want = (uint32_t)(t + 1);
  Spin spin;
  while (__atomic_load_n(&v->resp[slot].done, __ATOMIC_ACQUIRE) != want)
    if (int rc = spin.step(this, t, "result")) return rc;
  *value = __atomic_load_n(&v->resp[slot].value, __ATOMIC_RELAXED);
  v->ack[slot].store(want, std::memory_order_release);
  return HF3FS_CRC_OK;
}

void hf3fs_crc_coalescer::service_completer_loop() {
  Service* v = svc;
  for (;;) {
    uint64_t t;
    {
      std::unique_lock<std::mutex> lk(v->q_mu);
      v->q_cv.wait(lk, [&] { return !v->q.empty() || v->q_stop; });
      if (v->q.empty()) return;
      t = v->q.front();
      v->q.pop_front();
    }
    // the callback must be read before the slot is released
    const Waiter w = v->cbs[(uint32_t)t & v->mask];
    uint32_t value = 0;
    const int rc = service_wait(t, &value);
    w.fn(w.arg, rc, rc ? 0u : value);
  }
}

void hf3fs_crc_coalescer::service_teardown() {
  Service* v = svc;
  if (!v) return;
  if (v->completer.joinable()) {
    {
      std::lock_guard<std::mutex> lk(v->q_mu);
      v->q_stop = true;
    }
    v->q_cv.notify_all();
    v->completer.join();  // drains the queued async requests first
  }
  if (v->ctrl) __atomic_store_n(&v->ctrl->stop, 1u, __ATOMIC_RELEASE);
  (void)hipSetDevice(opt.device);
  if (v->stream) {
    // every service workgroup leaves on `stop` (or its idle timeout): bounded wait
    const Clock::time_point until = Clock::now() + kServiceTimeout;
    while (hipStreamQuery(v->stream) == hipErrorNotReady) {
      if (Clock::now() > until) {
        std::fprintf(stderr, "hf3fs_crc coalescer service: kernel did not exit; its ring stays mapped\n");
        return;  // the kernel may still touch the ring: leak it rather than free it under the kernel
      }
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    (void)hipStreamDestroy(v->stream);
  }
  if (v->ev) (void)hipEventDestroy(v->ev);
  if (v->req) (void)hipHostFree(v->req);
  if (v->resp) (void)hipHostFree(v->resp);
  if (v->ctrl) (void)hipHostFree(v->ctrl);
  if (v->stage) (void)hipHostFree(v->stage);
  if (v->dnext) (void)hipFree(v->dnext);
  delete v;
  svc = nullptr;
}

// ===========================================================================
extern "C" {

void hf3fs_crc_coalescer_default_options(hf3fs_crc_coalescer_options* o) {
  if (!o) return;
  o->device = 0;
  (void)hipGetDevice(&o->device);
  o->max_batch = 4096;
  o->max_wait_us = 0;
  o->stage_bytes = 32ull << 20;
  o->slots = 4;
  o->inflight = 2;
  o->service_wgs = 0;
  o->service_ring = 1024;
  o->service_idle_us = 2000;
  o->service_stage = 64 << 10;
}

int hf3fs_crc_coalescer_create(const hf3fs_crc_coalescer_options* opt, hf3fs_crc_coalescer** out) {
  if (!out) return cfail(HF3FS_CRC_INVALID_ARG, "null out");
  *out = nullptr;
  hf3fs_crc_coalescer_options o;
  hf3fs_crc_coalescer_default_options(&o);
  if (opt) o = *opt;
  if (o.max_batch == 0 || o.max_batch > (1u << 20) || o.slots < 2 || o.slots > 64 || o.inflight == 0 ||
      o.inflight >= o.slots)
    return cfail(HF3FS_CRC_INVALID_ARG, "bad coalescer options");
  if (o.service_wgs && (o.service_wgs > 4096 || o.service_ring < 2 || o.service_ring > (1u << 20) ||
                        (o.service_ring & (o.service_ring - 1)) || o.service_idle_us == 0))
    return cfail(HF3FS_CRC_INVALID_ARG, "bad coalescer service options");
  int prev = 0;
  CO_HIP(hipGetDevice(&prev));
  auto* c = new hf3fs_crc_coalescer();
  c->opt = o;
  int rc = c->init();
  (void)hipSetDevice(prev);
  if (rc) {
    std::string msg = hf3fs_crc_last_error();
    c->teardown();
    delete c;
    return cfail(rc, msg.c_str());
  }
  *out = c;
  return HF3FS_CRC_OK;
}

void hf3fs_crc_coalescer_destroy(hf3fs_crc_coalescer* c) {
  if (!c) return;
  c->teardown();
  delete c;
}

int hf3fs_crc_coalescer_submit(hf3fs_crc_coalescer* c, uint8_t type, const void* buf, uint64_t len, uint32_t start,
                               uint32_t flags, hf3fs_crc_done_fn fn, void* arg) {
  if (!c) return cfail(HF3FS_CRC_INVALID_ARG, "null coalescer");
  return c->submit(type, buf, len, start, flags, fn, arg);
}

int hf3fs_crc_coalescer_create_one(hf3fs_crc_coalescer* c, uint8_t type, const void* buf, uint64_t len,
                                   uint32_t start, uint32_t flags, uint32_t* out) {
  if (!c || !out) return cfail(HF3FS_CRC_INVALID_ARG, "null argument");
  if (buf && (flags & ~uint32_t(HF3FS_CRC_REQ_HOST_COPY)) == 0 && c->service_eligible(type, len, flags)) {
    uint64_t t = 0;
    if (int rc = c->service_submit(buf, len, start, flags, nullptr, nullptr, &t)) return rc;
    return c->service_wait(t, out);
  }
  SyncWait w;
  if (int rc = c->submit(type, buf, len, start, flags, sync_done, &w)) return rc;
  // Spin briefly (a batch usually lands within tens of microseconds), then sleep.
  const auto until = Clock::now() + std::chrono::microseconds(200);
  while (!w.done.load(std::memory_order_acquire) && Clock::now() < until) std::this_thread::yield();
  {
    std::unique_lock<std::mutex> lk(w.m);
    w.cv.wait(lk, [&] { return w.done.load(std::memory_order_acquire) != 0; });
  }
  if (w.status) return cfail(w.status, "coalesced batch failed");
  *out = w.value;
  return HF3FS_CRC_OK;
}

int hf3fs_crc_coalescer_stats(hf3fs_crc_coalescer* c, uint64_t* out4) {
  if (!c || !out4) return cfail(HF3FS_CRC_INVALID_ARG, "null argument");
  std::lock_guard<std::mutex> lk(c->mu);
  out4[0] = c->n_requests + c->n_service.load();
  out4[1] = c->n_batches;
  out4[2] = c->n_bytes;
  out4[3] = c->max_batch_seen;
  return HF3FS_CRC_OK;
}

int hf3fs_crc_host_register(void* h_ptr, uint64_t len, void** d_ptr) {
  if (!h_ptr || !len || !d_ptr) return cfail(HF3FS_CRC_INVALID_ARG, "null argument");
  CO_HIP(hipHostRegister(h_ptr, len, hipHostRegisterMapped));
  CO_HIP(hipHostGetDevicePointer(d_ptr, h_ptr, 0));
  return HF3FS_CRC_OK;
}

int hf3fs_crc_host_unregister(void* h_ptr) {
  if (!h_ptr) return cfail(HF3FS_CRC_INVALID_ARG, "null argument");
  CO_HIP(hipHostUnregister(h_ptr));
  return HF3FS_CRC_OK;
}

}  // extern "C"
