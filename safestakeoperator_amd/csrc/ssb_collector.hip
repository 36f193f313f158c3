// ssb_collector.hip -- the per-slot collector: the native batched caller in front
// of ssb_threshold_aggregate_batch_cached_dev (include/ssbls.h, "Per-slot collector").
//
// Reference call site: every committee's duty ends with ONE
// ThresholdSignature::new(t).threshold_aggregate(sigs, pks, ids, msg) (HotstuffOperatorCommittee::sign,
// src/validation/impls/hotstuff.rs:141-169, the call at :165-166), thousands of them per slot, each a
// handful of shares.  Here those calls become ssb_collector_submit: the job's bytes go straight into
// the open window's pinned, device-mapped buffer, and the window runs as one engine batch.
//
// Concurrency.  Submitters reserve (job, share range) in the open window with a compare-and-swap on a
// packed word (bit 63 closed | 15-bit incarnation tag | jobs << 27 | shares): jobs and shares are
// handed out in order, so the jobs form a prefix and their share ranges are contiguous (share_off is
// written by the submitters themselves).  The tag is the window's incarnation (window objects are
// reused): a submitter that loaded `open` and was preempted while that window was closed, delivered
// and reopened fails its CAS instead of reserving in the wrong incarnation, and it waits for the
// incarnation to change, not the pointer (with a plain fetch_add the add could land inside
// reset() -- a lost job -- or on the closed word of a window that then reopened -- a caller blocked
// forever).  A window without room asks the worker to close it and retries in the next one.  The
// worker closes a window with fetch_or(closed): the reservations made before it are exactly `jobs` of
// the returned word; it waits until all of them have been copied, deduplicates the signing roots
// (hash_to_G2 runs once per distinct root), and launches the window on the next one-stream pipeline
// slot.  Up to `in_flight`
// windows run on the device while the next fills; a window's buffer is reused only after its event
// completes, and results are delivered in launch order -- by a second thread, so that delivering a
// window's results (copies + callbacks, tens of microseconds per window) never delays closing and
// launching the next one (round 4: with one thread doing both, the collector's rate varied 0.72-1.0
// of the engine's with the time the deliveries took).
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
#include <unordered_map>
#include <vector>

#include "../../include/ssbls.h"

namespace ssb {
int ctx_device(const ssb_ctx* ctx);
std::recursive_mutex& ctx_mutex(ssb_ctx* ctx);
int ctx_attach_collector(ssb_ctx* ctx, int d, int in_flight);
}

namespace {

// the reservation word: bit 63 closed | tag (bits 48..62) | jobs (bits 27..47) | shares (bits 0..26)
constexpr uint64_t CLOSED = 1ull << 63;
constexpr int JOB_SHIFT = 27, TAG_SHIFT = 48;
constexpr uint64_t SHARE_MASK = (1ull << JOB_SHIFT) - 1, JOB_MASK = (1ull << (TAG_SHIFT - JOB_SHIFT)) - 1;
constexpr uint64_t TAG_FIELD = 0x7fffull << TAG_SHIFT;
constexpr uint32_t MAX_WINDOW_JOBS = 1u << 20, MAX_WINDOW_SHARES = 1u << 26;
inline uint64_t tag_of(uint64_t gen) { return (gen & 0x7fffull) << TAG_SHIFT; }
inline uint32_t jobs_of(uint64_t r) { return (uint32_t)((r >> JOB_SHIFT) & JOB_MASK); }
constexpr uint32_t MAX_JOB_SHARES = 64;
constexpr size_t WIRE_REC = 202;   // bincode(bls::Signature): u64 length 194, "0x", 192 hex digits
inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }
inline int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
inline void cpu_relax() { __builtin_ia32_pause(); }

struct window {
  uint8_t* h = nullptr;   // pinned host buffer (inputs, then the engine's outputs)
  uint8_t* d = nullptr;   // its device address
  size_t i_sig = 0, i_pk = 0, i_ids = 0, i_off = 0, i_t = 0, i_jr = 0, i_roots = 0, o_sig = 0, o_st = 0, o_err = 0, o_ver = 0,
         o_wst = 0;   // (wire collectors: i_sig holds 202-byte records; o_wst their statuses)
  std::atomic<uint64_t> resv{CLOSED};
  std::atomic<uint64_t> gen{0};   // the incarnation (== seq while open), tagged into resv
  std::atomic<uint32_t> settled{0};
  std::atomic<uint32_t> committed{0};
  std::atomic<int64_t> t_first{0};
  std::vector<ssb_job_result*> res;
  std::vector<ssb_job_done_fn> cb;
  std::vector<void*> user;
  std::vector<uint8_t> root_in;   // per job, the 32-byte root as submitted
  hipEvent_t ev = nullptr;
  bool ev_ok = false;     // ev was recorded after the window's launches (sync on it before reuse)
  uint64_t seq = 0;
  uint32_t nj = 0, ns = 0;
  int rc = SSB_OK;
  uint32_t* off() { return (uint32_t*)(h + i_off); }
};

}  // namespace

struct ssb_collector {
  ssb_ctx* ctx = nullptr;
  int device = 0;
  uint32_t J = 0, N = 0, in_flight = 1;
  bool wire = false;               // SSB_COLLECTOR_WIRE: shares held as wire records
  int64_t window_ns = 0;
  std::vector<window*> all;
  std::atomic<window*> open{nullptr};
  std::deque<window*> inflight, freel;
  std::mutex mu;                   // worker state, the queues, the condition variables
  std::condition_variable cv_worker, cv_submit, cv_done, cv_deliver, cv_free;
  bool sealing_done = false;       // the worker has closed its last window (destroy)
  uint64_t seal_upto = 0;          // a submitter found window seq <= this full: close it
  uint32_t max_windows = 1;        // windows on the device: two per slot (one running, one queued)
  std::atomic<bool> stopping{false};
  uint64_t seq_next = 1, flush_upto = 0, delivered_seq = 0;
  uint32_t slot_rr = 0;
  std::atomic<uint64_t> n_windows{0}, n_jobs{0}, n_shares{0};
  // profile: ns the worker spent closing + launching windows and waiting for a device window to free
  // up, ns the deliverer spent delivering results; submitter waits for a new window
  std::atomic<uint64_t> ns_seal{0}, ns_deliver{0}, ns_backpressure{0}, n_full_waits{0};
  std::thread worker, deliverer;
  std::vector<uint32_t> rtab;      // worker-only: root dedup table (index + 1)

  // a new incarnation of a free window: every counter first, the reservation word LAST (release),
  // so a submitter whose CAS succeeds on the new tag sees the zeroed counters
  void reset(window* w) {
    w->settled.store(0, std::memory_order_relaxed);
    w->committed.store(0, std::memory_order_relaxed);
    w->t_first.store(0, std::memory_order_relaxed);
    w->off()[0] = 0;
    w->nj = w->ns = 0;
    w->rc = SSB_OK;
    w->ev_ok = false;
    w->seq = seq_next++;
    w->gen.store(w->seq, std::memory_order_release);
    w->resv.store(tag_of(w->seq), std::memory_order_release);
  }
  void seal(window* w);
  void deliver(window* w);
  void run();            // the worker: closes and launches windows
  void deliver_loop();   // the deliverer: waits for the oldest window on the device, delivers it
};

namespace {

// until the open window is another one or another incarnation of w (a window object is reused)
void wait_new_window(ssb_collector* c, window* w, uint64_t gen) {
  c->n_full_waits.fetch_add(1, std::memory_order_relaxed);
  std::unique_lock<std::mutex> lk(c->mu);
  // (also when w's reservation word already carries gen's tag and is open: reset() stores gen before
  // the word, so a submitter may have read the new gen beside the old closed word -- then nothing
  // would change until some other submitter filled w)
  c->cv_submit.wait(lk, [&] {
    const uint64_t r = w->resv.load(std::memory_order_acquire);
    return c->open.load(std::memory_order_acquire) != w || w->gen.load(std::memory_order_acquire) != gen || c->stopping ||
           (!(r & CLOSED) && (r & TAG_FIELD) == tag_of(gen));
  });
}

}  // namespace

// close-time work on the worker thread: distinct roots, the job -> root map, then the launch
void ssb_collector::seal(window* w) {
  const uint32_t nj = w->committed.load(std::memory_order_acquire);
  w->nj = nj;
  w->ns = nj ? w->off()[nj] : 0;
  uint32_t* jr = (uint32_t*)(w->h + w->i_jr);
  uint8_t* roots = w->h + w->i_roots;
  const uint32_t mask = (uint32_t)rtab.size() - 1;
  std::fill(rtab.begin(), rtab.end(), 0u);
  uint32_t nr = 0;
  for (uint32_t j = 0; j < nj; ++j) {
    const uint8_t* r = w->root_in.data() + 32 * (size_t)j;
    uint64_t k;
    memcpy(&k, r, 8);
    uint32_t hsh = (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> 32) & mask;
    for (;;) {
      const uint32_t e = rtab[hsh];
      if (!e) {
        memcpy(roots + 32 * (size_t)nr, r, 32);
        rtab[hsh] = ++nr;
        jr[j] = nr - 1;
        break;
      }
      if (!memcmp(roots + 32 * (size_t)(e - 1), r, 32)) { jr[j] = e - 1; break; }
      hsh = (hsh + 1) & mask;
    }
  }
  static const uint8_t dst[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";   // src/crypto/impls/blst.rs:11
  std::lock_guard<std::recursive_mutex> g(ssb::ctx_mutex(ctx));   // the slot's stream and the launches, atomically
  const int k = (int)(slot_rr++ % in_flight);
  void* st = ssb_slot_stream(ctx, k);
  if (!st) {   // (cannot happen while attached: the slots are ours) -- nothing launched, nothing to wait for
    w->rc = SSB_EINVAL;
    w->ev_ok = false;
    n_windows.fetch_add(1, std::memory_order_relaxed);
    return;
  }
  uint8_t* d = w->d;
  if (wire)
    w->rc = ssb_threshold_aggregate_batch_wire_cached_dev(
        ctx, nj, w->ns, (const uint32_t*)(d + w->i_off), (const uint32_t*)(d + w->i_t), d + w->i_sig, WIRE_REC,
        (const uint32_t*)(d + w->i_pk), (const uint64_t*)(d + w->i_ids), (const uint32_t*)(d + w->i_jr), nr, d + w->i_roots,
        dst, sizeof(dst) - 1, 0, d + w->o_sig, (int32_t*)(d + w->o_st), (uint64_t*)(d + w->o_err), d + w->o_ver,
        (int32_t*)(d + w->o_wst), st);
  else
    w->rc = ssb_threshold_aggregate_batch_cached_dev(
        ctx, nj, w->ns, (const uint32_t*)(d + w->i_off), (const uint32_t*)(d + w->i_t), d + w->i_sig,
        (const uint32_t*)(d + w->i_pk), (const uint64_t*)(d + w->i_ids), (const uint32_t*)(d + w->i_jr), nr, d + w->i_roots,
        dst, sizeof(dst) - 1, 0, d + w->o_sig, (int32_t*)(d + w->o_st), (uint64_t*)(d + w->o_err), d + w->o_ver, st);
  // the event follows whatever the call enqueued, a failed call's partial launches included: the
  // deliverer waits on it before the window's buffer is refilled; if it cannot be
  // recorded, the stream is drained here instead
  w->ev_ok = st && hipEventRecord(w->ev, (hipStream_t)st) == hipSuccess;
  if (!w->ev_ok) {
    if (st) (void)hipStreamSynchronize((hipStream_t)st);
    (void)hipGetLastError();
    if (w->rc == SSB_OK) w->rc = SSB_EHIP;
  }
  n_windows.fetch_add(1, std::memory_order_relaxed);
}

void ssb_collector::deliver(window* w) {
  const int32_t* st = (const int32_t*)(w->h + w->o_st);
  const uint64_t* er = (const uint64_t*)(w->h + w->o_err);
  const uint8_t* sg = w->h + w->o_sig;
  const uint8_t* vr = w->h + w->o_ver;
  const uint32_t* off = w->off();
  for (uint32_t j = 0; j < w->nj; ++j) {
    ssb_job_result* r = w->res[j];
    const uint32_t b = off[j], n = off[j + 1] - off[j];
    r->n_shares = n;
    r->rc = w->rc;
    if (w->rc == SSB_OK) {
      memcpy(r->sig96, sg + 96 * (size_t)j, 96);
      r->status = st[j];
      r->err[0] = er[2 * (size_t)j];
      r->err[1] = er[2 * (size_t)j + 1];
      uint64_t bits = 0, absent = 0;
      for (uint32_t i = 0; i < n && i < 64; ++i) bits |= (uint64_t)(vr[b + i] != 0) << i;
      if (wire) {
        const int32_t* ws = (const int32_t*)(w->h + w->o_wst);
        for (uint32_t i = 0; i < n && i < 64; ++i) absent |= (uint64_t)(ws[b + i] != 0) << i;
      }
      r->verdicts = bits;
      r->absent = absent;
    } else {
      memset(r->sig96, 0, 96);
      r->status = SSB_DVF_ENGINE_ERROR;
      r->err[0] = (uint64_t)(int64_t)w->rc;
      r->err[1] = 0;
      r->verdicts = 0;
      r->absent = 0;
    }
    __atomic_store_n(&r->done, 1u, __ATOMIC_RELEASE);
    if (w->cb[j]) w->cb[j](w->user[j], r);
  }
  n_jobs.fetch_add(w->nj, std::memory_order_relaxed);
  n_shares.fetch_add(w->ns, std::memory_order_relaxed);
}

void ssb_collector::run() {
  hipSetDevice(device);
  std::unique_lock<std::mutex> lk(mu);
  for (;;) {
    window* w = open.load(std::memory_order_relaxed);
    const uint64_t r = w->resv.load(std::memory_order_acquire);
    const uint32_t nres = jobs_of(r);
    const int64_t t0 = w->t_first.load(std::memory_order_relaxed);
    const int64_t now = now_ns();
    const bool due = nres > 0 && (seal_upto >= w->seq || stopping || flush_upto >= w->seq || nres >= J ||
                                  (t0 && now - t0 >= window_ns));
    if (due) {
      if (inflight.size() >= max_windows || freel.empty()) {   // every device window busy: wait for a delivery
        const int64_t b0 = now_ns();
        cv_free.wait(lk, [&] { return inflight.size() < max_windows && !freel.empty(); });
        ns_backpressure.fetch_add((uint64_t)(now_ns() - b0), std::memory_order_relaxed);
        continue;
      }
      window* nw = freel.front();
      freel.pop_front();
      reset(nw);
      open.store(nw, std::memory_order_release);
      cv_submit.notify_all();
      lk.unlock();
      const int64_t s0 = now_ns();
      const uint32_t pre = jobs_of(w->resv.fetch_or(CLOSED, std::memory_order_acq_rel));
      while (w->settled.load(std::memory_order_acquire) < pre) cpu_relax();   // submitters mid-copy
      seal(w);
      ns_seal.fetch_add((uint64_t)(now_ns() - s0), std::memory_order_relaxed);
      lk.lock();
      inflight.push_back(w);
      cv_deliver.notify_one();
      continue;
    }
    if (stopping && nres == 0) break;
    // sleep until the window is due or a submitter fills it / starts it
    int64_t wait = (int64_t)1000000000;
    if (nres > 0 && t0) wait = std::max<int64_t>(0, t0 + window_ns - now);
    else if (nres > 0) wait = 20000;
    if (wait > 0) cv_worker.wait_for(lk, std::chrono::nanoseconds(wait));
  }
  sealing_done = true;
  cv_deliver.notify_all();
}

void ssb_collector::deliver_loop() {
  hipSetDevice(device);
  std::unique_lock<std::mutex> lk(mu);
  for (;;) {
    cv_deliver.wait(lk, [&] { return !inflight.empty() || sealing_done; });
    if (inflight.empty()) break;   // (sealing_done: nothing more will be launched)
    window* f = inflight.front();  // stays queued while it runs: FIFO delivery, and the worker counts it
    lk.unlock();
    if (f->ev_ok && hipEventSynchronize(f->ev) != hipSuccess && f->rc == SSB_OK) f->rc = SSB_EHIP;
    const int64_t d0 = now_ns();
    deliver(f);
    ns_deliver.fetch_add((uint64_t)(now_ns() - d0), std::memory_order_relaxed);
    lk.lock();
    inflight.pop_front();
    delivered_seq = f->seq;
    freel.push_back(f);
    cv_free.notify_all();
    cv_done.notify_all();
  }
  cv_done.notify_all();
}

namespace {
void free_windows(ssb_collector* c) {
  for (window* w : c->all) {
    if (w->ev) hipEventDestroy(w->ev);
    if (w->h) hipHostFree(w->h);
    delete w;
  }
  c->all.clear();
}
// wake the worker about a change of a window's reservation word (which it reads outside `mu`):
// taking `mu` first means the worker is either before its check or already waiting (no lost wakeup)
// (full_gen: the incarnation found without room -- closing is asked for THAT incarnation only, so a
// late request never closes its successor; 0: just a wake-up)
void poke_worker(ssb_collector* c, uint64_t full_gen) {
  {
    std::lock_guard<std::mutex> lk(c->mu);
    if (full_gen > c->seal_upto) c->seal_upto = full_gen;
  }
  c->cv_worker.notify_one();
}
// lowercase hex of a 96-byte compressed signature into a wire record (a compressed share submitted
// to a wire collector): exactly bincode::serialize(&sig), which the device decodes back
void to_wire(uint8_t* rec, const uint8_t* sig96) {
  static const char* hx = "0123456789abcdef";
  const uint64_t len = 194;
  memcpy(rec, &len, 8);
  rec[8] = '0'; rec[9] = 'x';
  for (int b = 0; b < 96; ++b) { rec[10 + 2 * b] = (uint8_t)hx[sig96[b] >> 4]; rec[11 + 2 * b] = (uint8_t)hx[sig96[b] & 15]; }
}
}  // namespace

extern "C" {

int ssb_collector_create2(ssb_ctx* ctx, uint32_t max_jobs, uint32_t max_shares, uint32_t window_us, int in_flight,
                          uint32_t flags, ssb_collector** out) {
  if (!out) return SSB_EINVAL;
  *out = nullptr;
  if (!ctx || max_jobs == 0 || max_jobs > MAX_WINDOW_JOBS || max_shares < MAX_JOB_SHARES || max_shares > MAX_WINDOW_SHARES ||
      in_flight < 1 || (flags & ~(uint32_t)SSB_COLLECTOR_WIRE) || ssb_check_pipeline_config(in_flight, 1) != SSB_OK)
    return SSB_EINVAL;
  // one hardware queue per slot stream, one left for the process (ssb_hw_queue_budget): a larger
  // in_flight would put independent windows on shared queues, where they serialise
  const int budget = ssb_hw_queue_budget();
  if (in_flight > budget - 1) {
    const int cap = budget - 1 > 1 ? budget - 1 : 1;
    fprintf(stderr, "ssb_collector_create: in_flight %d lowered to %d -- the process has GPU_MAX_HW_QUEUES=%d hardware "
                    "queues (set GPU_MAX_HW_QUEUES >= in_flight + 1, at most 32, before the first HIP call)\n",
            in_flight, cap, budget);
    in_flight = cap;
  }
  int rc;
  {
    std::lock_guard<std::recursive_mutex> g(ssb::ctx_mutex(ctx));
    // attached: ssb_set_pipeline_depth / ssb_set_slot_streams refuse to change the slots until
    // ssb_collector_destroy detaches (the worker picks slots round robin over in_flight of them)
    if ((rc = ssb::ctx_attach_collector(ctx, 1, in_flight))) return rc;
  }
  auto detach = [&] {
    std::lock_guard<std::recursive_mutex> g(ssb::ctx_mutex(ctx));
    ssb::ctx_attach_collector(ctx, -1, 0);
  };
  ssb_collector* c = new (std::nothrow) ssb_collector();
  if (!c) { detach(); return SSB_ENOMEM; }
  c->ctx = ctx;
  c->device = ssb::ctx_device(ctx);
  c->J = max_jobs;
  c->N = max_shares;
  c->in_flight = (uint32_t)in_flight;
  c->wire = (flags & SSB_COLLECTOR_WIRE) != 0;
  c->max_windows = 2u * (uint32_t)in_flight;
  c->window_ns = (int64_t)window_us * 1000;
  uint32_t rt = 1;
  while (rt < 2 * max_jobs) rt <<= 1;
  c->rtab.assign(rt, 0u);
  if (hipSetDevice(c->device) != hipSuccess) { delete c; detach(); return SSB_EHIP; }
  const size_t J = max_jobs, N = max_shares;
  for (int i = 0; i < 2 * in_flight + 2; ++i) {
    window* w = new (std::nothrow) window();
    if (!w) { free_windows(c); delete c; detach(); return SSB_ENOMEM; }
    c->all.push_back(w);
    size_t o = 0;
    auto at = [&](size_t bytes) { const size_t r = o; o += al(bytes); return r; };
    w->i_sig = at(N * (c->wire ? WIRE_REC : 96)); w->i_pk = at(N * 4); w->i_ids = at(N * 8); w->i_off = at((J + 1) * 4);
    w->i_t = at(J * 4); w->i_jr = at(J * 4); w->i_roots = at(J * 32); w->o_sig = at(J * 96); w->o_st = at(J * 4);
    w->o_err = at(J * 16); w->o_ver = at(N);
    if (c->wire) w->o_wst = at(N * 4);
    if (hipHostMalloc((void**)&w->h, o, hipHostMallocMapped | hipHostMallocNonCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&w->d, w->h, 0) != hipSuccess ||
        hipEventCreateWithFlags(&w->ev, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      if (w->h) { hipHostFree(w->h); w->h = nullptr; }
      free_windows(c);
      delete c;
      detach();
      return SSB_ENOMEM;
    }
    w->res.assign(J, nullptr);
    w->cb.assign(J, nullptr);
    w->user.assign(J, nullptr);
    w->root_in.assign(J * 32, 0);
    c->freel.push_back(w);
  }
  window* w0 = c->freel.front();
  c->freel.pop_front();
  c->reset(w0);
  c->open.store(w0);
  c->worker = std::thread([c] { c->run(); });
  c->deliverer = std::thread([c] { c->deliver_loop(); });
  *out = c;
  return SSB_OK;
}

int ssb_collector_create(ssb_ctx* ctx, uint32_t max_jobs, uint32_t max_shares, uint32_t window_us, int in_flight,
                         ssb_collector** out) {
  return ssb_collector_create2(ctx, max_jobs, max_shares, window_us, in_flight, 0u, out);
}

void ssb_collector_destroy(ssb_collector* c) {
  if (!c) return;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    c->stopping.store(true);
  }
  c->cv_worker.notify_all();
  c->cv_submit.notify_all();
  if (c->worker.joinable()) c->worker.join();        // closes the last window, then sealing_done
  if (c->deliverer.joinable()) c->deliverer.join();  // delivers every window on the device
  free_windows(c);
  {
    std::lock_guard<std::recursive_mutex> g(ssb::ctx_mutex(c->ctx));
    ssb::ctx_attach_collector(c->ctx, -1, 0);
  }
  delete c;
}

int ssb_collector_register_keys(ssb_collector* c, size_t n, const uint8_t* pk48, uint32_t* out_index) {
  if (!c) return SSB_EINVAL;
  return ssb_pk_cache_add(c->ctx, n, pk48, out_index);   // (the context's lock serialises it with the launches)
}

}  // extern "C"
namespace {
// one job into the open window: a CAS reservation on the incarnation's tagged word, then the copy;
// `put` writes share i's signature bytes at `dst` (96 bytes, or a wire record in a wire collector)
template <class Put>
int submit_job(ssb_collector* c, uint32_t t, uint32_t n, Put put, const uint32_t* pk_index, const uint64_t* ids,
               const uint8_t* root32, ssb_job_result* result, ssb_job_done_fn cb, void* user) {
  __atomic_store_n(&result->done, 0u, __ATOMIC_RELAXED);
  for (;;) {
    if (c->stopping.load(std::memory_order_acquire)) return SSB_EINVAL;   // (a submit must not race destroy)
    window* w = c->open.load(std::memory_order_acquire);
    const uint64_t g = w->gen.load(std::memory_order_acquire);
    uint64_t r = w->resv.load(std::memory_order_acquire);
    bool placed = false, full = false;
    uint32_t j = 0, s = 0;
    while (!(r & CLOSED) && (r & TAG_FIELD) == tag_of(g)) {
      j = jobs_of(r);
      s = (uint32_t)(r & SHARE_MASK);
      if (j >= c->J || (uint64_t)s + n > c->N) { full = true; break; }
      if (w->resv.compare_exchange_weak(r, r + (1ull << JOB_SHIFT) + n, std::memory_order_acq_rel,
                                        std::memory_order_acquire)) { placed = true; break; }
    }
    if (!placed) {   // closed, another incarnation, or no room: have it closed, retry in the next window
      if (full) poke_worker(c, g);
      if (c->stopping) return SSB_EINVAL;
      wait_new_window(c, w, g);
      continue;
    }
    if (j == 0) w->t_first.store(now_ns(), std::memory_order_relaxed);
    uint8_t* h = w->h;
    const size_t rec = c->wire ? WIRE_REC : 96;
    for (uint32_t i = 0; i < n; ++i) put(h + w->i_sig + rec * ((size_t)s + i), i);
    memcpy(h + w->i_pk + 4 * (size_t)s, pk_index, 4 * (size_t)n);
    memcpy(h + w->i_ids + 8 * (size_t)s, ids, 8 * (size_t)n);
    w->off()[j + 1] = s + n;
    ((uint32_t*)(h + w->i_t))[j] = t;
    memcpy(w->root_in.data() + 32 * (size_t)j, root32, 32);
    w->res[j] = result;
    w->cb[j] = cb;
    w->user[j] = user;
    w->committed.fetch_add(1, std::memory_order_release);
    w->settled.fetch_add(1, std::memory_order_release);
    if (j == 0 || j + 1 == c->J) poke_worker(c, 0);   // a window starts (its timer) / is full
    return SSB_OK;
  }
}
}  // namespace
extern "C" {

int ssb_collector_submit(ssb_collector* c, uint32_t t, uint32_t n, const uint8_t* sig96, const uint32_t* pk_index,
                         const uint64_t* ids, const uint8_t* root32, ssb_job_result* result, ssb_job_done_fn cb,
                         void* user) {
  if (!c || !result || !root32 || t == 0 || t > SSB_MAX_T || n > MAX_JOB_SHARES || (n && (!sig96 || !pk_index || !ids)))
    return SSB_EINVAL;
  if (c->wire)
    return submit_job(c, t, n, [&](uint8_t* d, uint32_t i) { to_wire(d, sig96 + 96 * (size_t)i); }, pk_index, ids, root32,
                      result, cb, user);
  return submit_job(c, t, n, [&](uint8_t* d, uint32_t i) { memcpy(d, sig96 + 96 * (size_t)i, 96); }, pk_index, ids, root32,
                    result, cb, user);
}

int ssb_collector_submit_wire(ssb_collector* c, uint32_t t, uint32_t n, const uint8_t* const* wire, const size_t* wire_len,
                              const uint32_t* pk_index, const uint64_t* ids, const uint8_t* root32, ssb_job_result* result,
                              ssb_job_done_fn cb, void* user) {
  if (!c || !c->wire || !result || !root32 || t == 0 || t > SSB_MAX_T || n > MAX_JOB_SHARES ||
      (n && (!wire || !wire_len || !pk_index || !ids)))
    return SSB_EINVAL;
  // bincode::deserialize (bincode 1.3: trailing bytes allowed) reads the first 202 bytes of a record:
  // a longer record is decoded from those, a shorter one cannot be a Signature (its length
  // field is overwritten so that it never parses on the device: the share is absent)
  return submit_job(c, t, n, [&](uint8_t* d, uint32_t i) {
    const size_t l = wire[i] ? (wire_len[i] < WIRE_REC ? wire_len[i] : WIRE_REC) : 0;
    if (l) memcpy(d, wire[i], l);
    if (l < WIRE_REC) { memset(d + l, 0, WIRE_REC - l); const uint64_t bad = ~0ull; memcpy(d, &bad, 8); }
  }, pk_index, ids, root32, result, cb, user);
}

int ssb_collector_wait(ssb_collector* c, const ssb_job_result* r) {
  if (!c || !r) return SSB_EINVAL;
  if (__atomic_load_n(&r->done, __ATOMIC_ACQUIRE)) return SSB_OK;
  std::unique_lock<std::mutex> lk(c->mu);
  c->cv_done.wait(lk, [&] { return __atomic_load_n(&r->done, __ATOMIC_ACQUIRE) != 0; });
  return SSB_OK;
}

int ssb_collector_flush(ssb_collector* c) {
  if (!c) return SSB_EINVAL;
  std::unique_lock<std::mutex> lk(c->mu);
  window* w = c->open.load(std::memory_order_acquire);
  const bool empty = jobs_of(w->resv.load(std::memory_order_acquire)) == 0;
  const uint64_t target = empty ? w->seq - 1 : w->seq;
  if (target > c->flush_upto) c->flush_upto = target;
  c->cv_worker.notify_one();
  c->cv_done.wait(lk, [&] { return c->delivered_seq >= target; });
  return SSB_OK;
}

int ssb_collector_profile(ssb_collector* c, double* seal_ms, double* deliver_ms, double* backpressure_ms,
                          uint64_t* full_waits) {
  if (!c) return SSB_EINVAL;
  if (seal_ms) *seal_ms = c->ns_seal.load() * 1e-6;
  if (deliver_ms) *deliver_ms = c->ns_deliver.load() * 1e-6;
  if (backpressure_ms) *backpressure_ms = c->ns_backpressure.load() * 1e-6;
  if (full_waits) *full_waits = c->n_full_waits.load();
  return SSB_OK;
}

int ssb_collector_stats(ssb_collector* c, uint64_t* windows, uint64_t* jobs, uint64_t* shares) {
  if (!c) return SSB_EINVAL;
  if (windows) *windows = c->n_windows.load();
  if (jobs) *jobs = c->n_jobs.load();
  if (shares) *shares = c->n_shares.load();
  return SSB_OK;
}

}  // extern "C"

// ---- The local-signing window -------------------------------------------------
// Every duty of every validator an operator serves ends its local part with ONE
// DvfSigner::local_sign_and_store(signing_root) -> SecretKey::sign (src/node/dvfcore.rs:241-251; the
// call at src/validation/signing_method.rs:318 for attestations, blocks, aggregates, and the selection
// proofs / RANDAO reveals of :269-292): one G2 scalar multiplication and one hash_to_G2 on a tokio
// task each.  Here those calls become ssb_signer_submit: the worker closes a window at max_jobs
// submissions or window_us after its first, hashes every distinct root once and signs the whole
// window with one ssb_sign_batch, then completes each submission (result + callback).  The secret
// keys are wiped from the window's host buffer once signed.
namespace {
struct sign_job {
  uint8_t sk[32];   // little-endian scalar
  uint8_t root[32];
  ssb_sign_result* r;
  ssb_sign_done_fn cb;
  void* user;
};
void wipe(void* p, size_t n) {
  volatile uint8_t* v = (volatile uint8_t*)p;
  for (size_t i = 0; i < n; ++i) v[i] = 0;
}
}  // namespace

struct ssb_signer {
  ssb_ctx* ctx = nullptr;
  int device = 0;
  uint32_t J = 1;
  int64_t window_ns = 0;
  std::mutex mu;
  std::condition_variable cv_worker, cv_done;
  std::vector<sign_job> open;      // the filling window
  int64_t t_first = 0;
  bool stopping = false;
  uint64_t submitted = 0, delivered = 0, flush_upto = 0;
  std::atomic<uint64_t> n_windows{0};
  std::thread worker;

  void run() {
    hipSetDevice(device);
    std::vector<sign_job> win;
    std::vector<uint8_t> sk, roots, out;
    std::vector<uint32_t> ridx;
    std::unordered_map<std::string, uint32_t> rmap;
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      const int64_t now = now_ns();
      const bool due = !open.empty() && (stopping || open.size() >= J || flush_upto > delivered || now - t_first >= window_ns);
      if (!due) {
        if (stopping && open.empty()) break;
        if (open.empty()) cv_worker.wait(lk);
        else cv_worker.wait_for(lk, std::chrono::nanoseconds(std::max<int64_t>(1000, t_first + window_ns - now)));
        continue;
      }
      win.swap(open);
      open.clear();
      if (win.size() > J) {   // submitters filled past max_jobs while the last window ran: the rest waits
        open.assign(win.begin() + J, win.end());   // (its first job has waited since t_first: due at once)
        wipe(&win[J], (win.size() - J) * sizeof(sign_job));
        win.resize(J);
      }
      lk.unlock();
      const size_t n = win.size();
      sk.resize(32 * n); ridx.resize(n); roots.clear(); out.assign(96 * n, 0); rmap.clear();
      for (size_t i = 0; i < n; ++i) {
        memcpy(sk.data() + 32 * i, win[i].sk, 32);
        auto it = rmap.emplace(std::string((const char*)win[i].root, 32), (uint32_t)rmap.size()).first;
        if (it->second == roots.size() / 32) roots.insert(roots.end(), win[i].root, win[i].root + 32);
        ridx[i] = it->second;
      }
      static const uint8_t dst[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";   // src/crypto/impls/blst.rs:11
      const int rc = ssb_sign_batch(ctx, n, sk.data(), ridx.data(), roots.size() / 32, roots.data(), dst, sizeof(dst) - 1,
                                    out.data());
      wipe(sk.data(), sk.size());
      for (size_t i = 0; i < n; ++i) {
        wipe(win[i].sk, 32);
        ssb_sign_result* r = win[i].r;
        if (rc == SSB_OK) memcpy(r->sig96, out.data() + 96 * i, 96);
        else memset(r->sig96, 0, 96);
        r->rc = rc;
        __atomic_store_n(&r->done, 1u, __ATOMIC_RELEASE);
        if (win[i].cb) win[i].cb(win[i].user, r);
      }
      win.clear();
      n_windows.fetch_add(1, std::memory_order_relaxed);
      lk.lock();
      delivered += n;
      cv_done.notify_all();
    }
    cv_done.notify_all();
  }
};

extern "C" {

int ssb_signer_create(ssb_ctx* ctx, uint32_t max_jobs, uint32_t window_us, ssb_signer** out) {
  if (!out) return SSB_EINVAL;
  *out = nullptr;
  if (!ctx || max_jobs == 0 || max_jobs > MAX_WINDOW_JOBS) return SSB_EINVAL;
  ssb_signer* s = new (std::nothrow) ssb_signer();
  if (!s) return SSB_ENOMEM;
  s->ctx = ctx;
  s->device = ssb::ctx_device(ctx);
  s->J = max_jobs;
  s->window_ns = (int64_t)window_us * 1000;
  s->open.reserve(max_jobs);
  s->worker = std::thread([s] { s->run(); });
  *out = s;
  return SSB_OK;
}

void ssb_signer_destroy(ssb_signer* s) {
  if (!s) return;
  {
    std::lock_guard<std::mutex> lk(s->mu);
    s->stopping = true;
  }
  s->cv_worker.notify_all();
  if (s->worker.joinable()) s->worker.join();   // signs and delivers what was submitted
  delete s;
}

int ssb_signer_submit(ssb_signer* s, const uint8_t* sk32le, const uint8_t* root32, ssb_sign_result* result,
                      ssb_sign_done_fn cb, void* user) {
  if (!s || !sk32le || !root32 || !result) return SSB_EINVAL;
  __atomic_store_n(&result->done, 0u, __ATOMIC_RELAXED);
  sign_job j;
  memcpy(j.sk, sk32le, 32);
  memcpy(j.root, root32, 32);
  j.r = result; j.cb = cb; j.user = user;
  bool wake;
  {
    std::lock_guard<std::mutex> lk(s->mu);
    if (s->stopping) { wipe(j.sk, 32); return SSB_EINVAL; }
    if (s->open.empty()) s->t_first = now_ns();
    s->open.push_back(j);
    ++s->submitted;
    wake = s->open.size() == 1 || s->open.size() >= s->J;
  }
  wipe(j.sk, 32);
  if (wake) s->cv_worker.notify_one();
  return SSB_OK;
}

int ssb_signer_wait(ssb_signer* s, const ssb_sign_result* r) {
  if (!s || !r) return SSB_EINVAL;
  if (__atomic_load_n(&r->done, __ATOMIC_ACQUIRE)) return SSB_OK;
  std::unique_lock<std::mutex> lk(s->mu);
  s->cv_done.wait(lk, [&] { return __atomic_load_n(&r->done, __ATOMIC_ACQUIRE) != 0; });
  return SSB_OK;
}

int ssb_signer_flush(ssb_signer* s) {
  if (!s) return SSB_EINVAL;
  std::unique_lock<std::mutex> lk(s->mu);
  const uint64_t target = s->submitted;
  if (target > s->flush_upto) s->flush_upto = target;
  s->cv_worker.notify_one();
  s->cv_done.wait(lk, [&] { return s->delivered >= target; });
  return SSB_OK;
}

int ssb_signer_stats(ssb_signer* s, uint64_t* windows, uint64_t* signatures) {
  if (!s) return SSB_EINVAL;
  std::lock_guard<std::mutex> lk(s->mu);
  if (windows) *windows = s->n_windows.load();
  if (signatures) *signatures = s->delivered;
  return SSB_OK;
}

}  // extern "C"
