// ssbls.hip -- gfx950 kernels and the C ABI (include/ssbls.h) of the threshold-BLS engine.
//
// Pipeline of ssb_threshold_aggregate_batch_dev (three HIP streams, no host round trip):
//   side[0]: k_hash_to_g2  ||  main: decode -> RLC -> sums -> (wait hash) Miller -> final exp
//   side[1] (after decode): speculative select -> Lagrange -> combine, assuming every decodable
//   in-group share is valid; main then runs the exact select/combine only if the batch failed.
//   k_share_map       share -> job, share -> root                          (bookkeeping)
//   k_hash_to_g2      H(root) once per distinct signing root               (a-3)
//   k_decode          G2 decompress + subgroup check, G1 decompress        (a-2 steps 1/4)
//   k_rlc_mul         r_i*sig_i (G2), r_i*pk_i (G1), 64-bit RLC scalars    (a-7)
//   k_sum_g1_by_root  per-root sum of r_i*pk_i                              (a-7)
//   k_sum_g2_*        sum of r_i*sig_i                                      (a-7)
//   k_miller          one Miller loop per (root, sum) pair + (-g1, sum sig) (a-2 step 3)
//   k_final           product + ONE final exponentiation -> batch verdict
//   k_fallback_verify exact per-share verify, only if the batch failed
//   k_select          reference scan order / error semantics per job      (a-1)
//   k_lagrange        Lagrange coefficients, Montgomery batch inversion    (a-5)
//   k_combine_terms   lambda_i * sig_i  (verified shares: GLS, 4 digits on 4 lanes; a-4 unsafe: 255-bit)
//   k_combine_sum     sum, affine, compress                                 (a-4)
#include <hip/hip_runtime.h>
#include <chrono>
#include <thread>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <map>
#include <set>
#include <unordered_map>
#include <mutex>
#include <algorithm>
#include <cmath>
#include <cerrno>
#include <sys/random.h>

#include "ssb_units.h"
#include "ssb_kernels.h"
#include "../../include/ssbls.h"

using namespace ssb;
using namespace ssb::k;

namespace {

}  // namespace

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
// One pipeline slot: its own streams, events and workspace, so batches submitted to different
// slots (ssb_set_pipeline_depth) are independent and overlap on the device.
struct ssb_slot {
  hipStream_t stream = nullptr;     // main chain: decode -> RLC -> sums -> Miller -> final exp
  hipStream_t side[2] = {nullptr, nullptr};  // [0] hash_to_G2, [1] G1 products / sums
  hipEvent_t ev_in = nullptr, ev_hash = nullptr, ev_dec = nullptr, ev_comb = nullptr, ev_out = nullptr;
  hipEvent_t ev_sdec = nullptr, ev_r2 = nullptr, ev_r1 = nullptr, ev_user = nullptr, ev_fin = nullptr;
  bool out_pending = false;         // ev_out marks the end of the last _dev batch on this slot
  bool shared = false;              // side[] alias `stream` (one stream per slot)
  bool out_on_stream = false;       // the last batch's ev_out was recorded on `stream` itself
  // workspace arena (grown on demand, never shrunk)
  void* ws = nullptr;
  size_t ws_bytes = 0;
  // the fused one-stream path leaves the sort counts [0, clean_K) at clean_cnt and the tickets at
  // clean_tickets zeroed for the slot's next batch (its scan and its last blocks reset them); any
  // other use of the workspace clears this, and the next batch zeroes them in a prep launch
  uint32_t* clean_cnt = nullptr;
  uint32_t* clean_tickets = nullptr;
  uint32_t clean_K = 0;
  // host-buffer batches (ssb_threshold_aggregate_batch_submit): a pinned, device-mapped staging
  // buffer the kernels read their inputs from and write their outputs to in place, over PCIe
  // (zero-copy: no copy kernel, no copy queue); the outputs of the pending batch are copied to the
  // caller's pointers when it is waited for (or when the slot is reused)
  uint8_t* hst = nullptr;
  size_t hst_bytes = 0;
  hipEvent_t ev_host = nullptr;
  uint64_t host_ticket = 0;         // the batch whose outputs are still in the staging buffer (0: none)
  struct {
    uint8_t* sig; int32_t* st; uint64_t* err; uint8_t* ver;
    size_t nj, n, o_sig, o_st, o_err, o_ver;
  } ho = {};
};
constexpr int SSB_MAX_SLOTS = 24;

struct ssb_ctx {
  // Every entry point holds this for its whole call (SSB_LOCK): one context may be shared by the
  // threads of a process -- the collector's worker, a ThresholdSignature caller, registration --
  // and their calls are serialised (recursive: entry points call entry points)
  std::recursive_mutex mu;
  // the synchronous entry points (SSB_SYNC_LOCK): one at a time -- they share the io arena -- and
  // their final wait runs outside `mu`
  std::mutex sync_mu;
  int collectors = 0;               // attached ssb_collectors: the slot configuration is theirs
  int device = 0;
  // hardware queues the HIP runtime gives this process (GPU_MAX_HW_QUEUES, read by HIP when it
  // initialises; HIP's default is 4): ssb_set_pipeline_depth refuses more slot streams than fit
  int hw_queues = 4;
  ssb_slot sl[SSB_MAX_SLOTS];
  int nslots = 1, next = 0, slot_streams = 3;
  ssb_slot* cur = &sl[0];           // the slot the current call runs on
  std::string err;
  // host staging arena
  void* io = nullptr;
  size_t io_bytes = 0;
  struct evpair { hipEvent_t a = nullptr, b = nullptr; bool used = false; };
  std::map<std::string, evpair> timers;               // last launch of each kernel
  bool accumulate = false;                             // ssb_kernel_timing(ctx, 1)
  bool time_last = false;                              // ssb_kernel_timing(ctx, 2): last launch only
  std::map<std::string, std::vector<evpair>> history;  // every launch while accumulating
  std::vector<evpair> pool;
  g1_aff* negg1_pow = nullptr;                         // device: [2^s](-g1), s = 0..63 (G2 MSM pairs)
  // Context-wide streams of the three-stream (latency) configuration, shared by all its slots:
  // spec runs the speculative combines, tail the verdicts, the exact fallback and the exact combine
  // (the kernels with the largest private segments stay off the slots' queues).  One-stream slots
  // run every stage on the slot's own stream and leave both idle.
  hipStream_t spec = nullptr, tail = nullptr;
  // decoded public keys (ssb_pk_cache_set / ssb_pk_cache_add): affine points + DEC_* flags, indexed
  // by the caller; rows [0, pkc_n) are live, the arrays hold pkc_cap rows
  g1_aff* pkc_aff = nullptr; uint32_t* pkc_flags = nullptr; size_t pkc_n = 0, pkc_cap = 0;
  g1_aff* pkc_pow = nullptr;   // [pkc_cap][PKPOW_W] precomputed bases [2^(4 w)] pk (nullptr: allocation failed)
  // ssb_pk_cache_add: compressed key -> its row (first occurrence), built lazily after a _set
  std::unordered_map<std::string, uint32_t> pkc_map;
  bool pkc_map_valid = true;
  std::vector<uint8_t> pkc_set_keys;   // the keys of the last _set while pkc_map is not built
  uint8_t* pkc_stage = nullptr; size_t pkc_stage_bytes = 0;   // device staging of the keys being added
  // RLC key of each batch: fresh from getrandom() per call (default), or expanded from the caller's
  // seed (ssb_set_rlc_deterministic: reproducible runs / tests only)
  bool rlc_deterministic = false;
  uint64_t ticket_gen = 0;          // host-buffer batch tickets: (generation << 8) | slot
  std::set<uint64_t> failed_tickets;   // host batches whose completion failed (ssb_batch_wait -> SSB_EHIP)
};

namespace {

#define SSB_HIP(call)                                                                 \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    if (e_ != hipSuccess) {                                                           \
      ctx->err = std::string(#call) + ": " + hipGetErrorString(e_);                  \
      return SSB_EHIP;                                                                \
    }                                                                                 \
  } while (0)

#define SSB_LOCK(ctx) std::lock_guard<std::recursive_mutex> ssb_lock_((ctx)->mu)
// Synchronous entry points (the call waits for its own work, then returns host results): one at a
// time per context (sync_mu), on an idle slot when there is one (pick_idle_slot), and their final
// wait runs OUTSIDE the context lock, so a collector's worker keeps launching windows on the other
// slots meanwhile (a direct unsafe_aggregate held the lock through its stream
// synchronize, and seal() could launch on no slot until it returned).
#define SSB_SYNC_LOCK(ctx)                                                            \
  std::unique_lock<std::mutex> ssb_sync_((ctx)->sync_mu);                             \
  std::unique_lock<std::recursive_mutex> ssb_lock_((ctx)->mu)
#define SSB_SYNC_WAIT(st)                                                             \
  do {                                                                                \
    ssb_lock_.unlock();                                                               \
    const hipError_t e_ = hipStreamSynchronize(st);                                   \
    if (e_ != hipSuccess) {                                                           \
      ssb_lock_.lock();                                                               \
      ctx->err = std::string("hipStreamSynchronize: ") + hipGetErrorString(e_);       \
      return SSB_EHIP;                                                                \
    }                                                                                 \
  } while (0)

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }
const fp12 FP12_ONE_HOST = fp12_one();

struct carve {
  char* base; size_t off = 0;
  template <class T> T* take(size_t n) { T* p = (T*)(base + off); off += align_up(n * sizeof(T)); return p; }
};

// Every entry point takes the slot's workspace through here: the slot's main stream is ordered
// after the end of the slot's previous batch (whose last kernels run on the context streams).
int ensure_ws(ssb_ctx* ctx, size_t bytes, bool verify_layout = false) {
  ssb_slot* S = ctx->cur;
  if (S->out_pending && !S->out_on_stream) {   // (a same-stream wait would only add a queue packet)
    if (hipStreamWaitEvent(S->stream, S->ev_out, 0) != hipSuccess) { ctx->err = "hipStreamWaitEvent failed"; return SSB_EHIP; }
  }
  if (!verify_layout) S->clean_cnt = nullptr;   // another layout overwrites the counts (see run_verify)
  if (bytes <= ctx->cur->ws_bytes) return SSB_OK;
  S->clean_cnt = nullptr;
  if (S->out_pending) hipEventSynchronize(S->ev_out);
  if (ctx->cur->ws) { hipStreamSynchronize(ctx->cur->stream); hipFree(ctx->cur->ws); ctx->cur->ws = nullptr; ctx->cur->ws_bytes = 0; }
  size_t want = bytes + bytes / 4;
  if (hipMalloc(&ctx->cur->ws, want) != hipSuccess) { ctx->err = "hipMalloc workspace failed"; ctx->cur->ws = nullptr; return SSB_ENOMEM; }
  ctx->cur->ws_bytes = want;
  return SSB_OK;
}

// The slot a _dev call runs on: the slot whose main stream the caller passed (ssb_slot_stream), else
// the next one round robin.  (Round robin alone drifted out of step with a caller that cycles its
// own slot streams from a different starting point -- e.g. after a batch count that is not a
// multiple of the depth -- and every batch then chained two slots: 11 ms instead of 2.5 ms a batch.)
void pick_slot(ssb_ctx* ctx, void* stream) {
  for (int i = 0; stream && i < ctx->nslots; ++i)
    if ((void*)ctx->sl[i].stream == stream) {
      ctx->cur = &ctx->sl[i];
      ctx->next = (i + 1) % ctx->nslots;
      return;
    }
  ctx->cur = &ctx->sl[ctx->next];
  ctx->next = (ctx->next + 1) % ctx->nslots;
}

// The slot a synchronous call runs on: an idle one (its streams empty, no host batch pending), so the
// call does not queue behind pipelined batches; else the current one.
void pick_idle_slot(ssb_ctx* ctx) {
  for (int k = 0; k < ctx->nslots; ++k) {
    ssb_slot& S = ctx->sl[(ctx->next + k) % ctx->nslots];
    if (S.host_ticket || hipStreamQuery(S.stream) != hipSuccess) continue;
    if (!S.shared && (hipStreamQuery(S.side[0]) != hipSuccess || hipStreamQuery(S.side[1]) != hipSuccess)) continue;
    if (S.out_pending && hipEventQuery(S.ev_out) != hipSuccess) continue;
    ctx->cur = &S;
    break;
  }
  (void)hipGetLastError();   // (hipErrorNotReady of the queries is not an error of this call)
}

hipStream_t slot_tail(ssb_ctx* ctx) { return ctx->tail; }

// The context-wide spec / tail streams exist only while the slots are three-stream: one-stream slots
// run every stage on the slot's stream, and an idle stream still holds one of the process's hardware
// queues (more than ~23 mapped queues and the firmware time-slices them: measured 12.5 M partial
// sigs/s at 23, 5.1 M at 24, 3.6 M at 25, round 5).
int take_stream(ssb_ctx* ctx, hipStream_t* s);
void give_stream(ssb_ctx* ctx, hipStream_t& s);
int ctx_streams(ssb_ctx* ctx, bool on) {
  for (hipStream_t* x : {&ctx->spec, &ctx->tail}) {
    if (on && !*x && take_stream(ctx, x)) return SSB_EHIP;
    if (!on && *x) { hipStreamSynchronize(*x); give_stream(ctx, *x); }
  }
  return SSB_OK;
}

int ensure_io(ssb_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->io_bytes) return SSB_OK;
  if (ctx->io) { hipFree(ctx->io); ctx->io = nullptr; ctx->io_bytes = 0; }
  size_t want = bytes + bytes / 4;
  if (hipMalloc(&ctx->io, want) != hipSuccess) { ctx->err = "hipMalloc io failed"; ctx->io = nullptr; return SSB_ENOMEM; }
  ctx->io_bytes = want;
  return SSB_OK;
}

inline unsigned nblk(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

// streams = 3: main chain + hash_to_G2 + G1 side, overlapping inside the batch (lowest latency);
// streams = 1: the whole batch in order on one stream (side[] alias it) -- one hardware queue per
// slot, so many more slots fit the runtime's per-queue scratch reservations (highest throughput).
// A stream of the context, created now; its queue acquires its scratch at once, alone (streams are
// created one after the other: twenty slot queues growing their scratch at once on their first
// batches is round 2's HSA_STATUS_ERROR_OUT_OF_RESOURCES).  Released streams are destroyed, which
// returns their hardware queues and scratch to the runtime.  (Round 5 tried keeping released streams
// in a pool for the context's lifetime, so a slot never lands on a queue created later for someone
// else: the idle pooled queues kept their scratch, and a 20-slot fallback batch after the collector
// tests' contexts then failed with OUT_OF_RESOURCES.  bench.py instead creates its slots once, before
// the process group.)
int take_stream(ssb_ctx* ctx, hipStream_t* s) {
  (void)ctx;
  if (hipStreamCreateWithFlags(s, hipStreamNonBlocking) != hipSuccess) { *s = nullptr; return SSB_EHIP; }
  return launch::prime_queue(*s) ? SSB_EHIP : SSB_OK;
}
// (Round 5 measured slot streams in three priority bands -- hipStreamCreateWithPriority, so a burst's
// batches would finish staggered: 20 steps 9.2-10.0 M against 12.6-12.7 M without, 200 steps 10.5 M
// against 14.2-14.5 M, gpurun_out/r05prio.  Not kept.)
void give_stream(ssb_ctx* ctx, hipStream_t& s) {
  (void)ctx;
  if (s) { hipStreamSynchronize(s); hipStreamDestroy(s); }
  s = nullptr;
}
int init_slot(ssb_ctx* ctx, ssb_slot& S, int streams) {
  if (take_stream(ctx, &S.stream)) return SSB_EHIP;
  S.shared = streams == 1;
  for (int i = 0; i < 2; ++i) {
    if (S.shared) S.side[i] = S.stream;
    else if (take_stream(ctx, &S.side[i])) return SSB_EHIP;
  }
  for (hipEvent_t* e : {&S.ev_in, &S.ev_hash, &S.ev_dec, &S.ev_comb, &S.ev_out, &S.ev_sdec, &S.ev_r2, &S.ev_r1, &S.ev_user, &S.ev_fin,
                        &S.ev_host})
    if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) return SSB_EHIP;
  return SSB_OK;
}
// the pending host-buffer batch of the slot: wait for it, copy its outputs to the caller's pointers.
// If the wait fails the batch is lost: every job's status becomes SSB_DVF_ENGINE_ERROR (a lost batch
// never reads as SSB_DVF_OK in zero-filled outputs) and the ticket is remembered, so ssb_batch_wait
// on it returns SSB_EHIP whichever call delivered it.
hipError_t deliver_host(ssb_ctx* ctx, ssb_slot& S) {
  if (!S.host_ticket) return hipSuccess;
  const hipError_t e = hipEventSynchronize(S.ev_host);
  const auto& h = S.ho;
  const uint64_t ticket = S.host_ticket;
  S.host_ticket = 0;
  if (e != hipSuccess) {
    for (size_t j = 0; j < h.nj; ++j) { h.st[j] = SSB_DVF_ENGINE_ERROR; h.err[2 * j] = (uint64_t)(int64_t)e; h.err[2 * j + 1] = 0; }
    memset(h.sig, 0, h.nj * 96);
    if (h.ver && h.n) memset(h.ver, 0, h.n);
    ctx->failed_tickets.insert(ticket);
    ctx->err = std::string("batch completion failed: ") + hipGetErrorString(e);
    return e;
  }
  memcpy(h.sig, S.hst + h.o_sig, h.nj * 96);
  memcpy(h.st, S.hst + h.o_st, h.nj * 4);
  memcpy(h.err, S.hst + h.o_err, h.nj * 16);
  if (h.ver && h.n) memcpy(h.ver, S.hst + h.o_ver, h.n);
  return hipSuccess;
}
void sync_slot(ssb_ctx* ctx, ssb_slot& S) {
  deliver_host(ctx, S);
  if (S.stream) hipStreamSynchronize(S.stream);
  if (!S.shared) for (hipStream_t sd : S.side) if (sd) hipStreamSynchronize(sd);
  if (S.out_pending) hipEventSynchronize(S.ev_out);
}
void free_slot(ssb_ctx* ctx, ssb_slot& S) {
  deliver_host(ctx, S);
  if (S.ws) hipFree(S.ws);
  if (S.hst) hipHostFree(S.hst);
  if (!S.shared) for (hipStream_t& sd : S.side) give_stream(ctx, sd);
  for (hipEvent_t e : {S.ev_in, S.ev_hash, S.ev_dec, S.ev_comb, S.ev_out, S.ev_sdec, S.ev_r2, S.ev_r1, S.ev_user, S.ev_fin,
                       S.ev_host})
    if (e) hipEventDestroy(e);
  give_stream(ctx, S.stream);
}

// hipEvent pair around one kernel launch on the engine's stream (the stream the kernel runs on)
struct timed {
  ssb_ctx* ctx; ssb_ctx::evpair p; std::string name; hipStream_t st; bool on;
  // events only while timing is on (ssb_kernel_timing): two event packets per stage and batch are
  // not free on a queue that already carries a batch's ~40 kernels
  timed(ssb_ctx* c, const char* nm, hipStream_t s = nullptr)
      : ctx(c), name(nm), st(s ? s : c->cur->stream), on(c->accumulate || c->time_last) {
    if (!on) return;
    if (!ctx->pool.empty()) { p = ctx->pool.back(); ctx->pool.pop_back(); }
    else { hipEventCreate(&p.a); hipEventCreate(&p.b); }
    hipEventRecord(p.a, st);
  }
  ~timed() {
    if (!on) return;
    hipEventRecord(p.b, st);
    p.used = true;
    if (ctx->accumulate) { ctx->history[name].push_back(p); return; }
    auto it = ctx->timers.find(name);
    if (it != ctx->timers.end() && it->second.a) ctx->pool.push_back(it->second);
    ctx->timers[name] = p;
  }
};

int fill_dst(ssb_ctx* ctx, dst_arg& d, const uint8_t* dst, size_t dst_len) {
  if (dst_len > SSB_MAX_DST || (dst_len && !dst)) { ctx->err = "dst too long or null"; return SSB_EINVAL; }
  memset(&d, 0, sizeof(d));
  if (dst_len) memcpy(d.b, dst, dst_len);
  d.len = (int)dst_len;
  return SSB_OK;
}

// The batch's RLC key (ssb_units.h): 256 bits from the OS CSPRNG for every call, drawn after the
// caller has handed the inputs over, so no sender can know its shares' scalars; the caller's
// rlc_seed is XORed in (it can only add entropy).  Deterministic mode: the seed alone.
int draw_rlc_key(ssb_ctx* ctx, uint64_t seed, rlc_key& key) {
  if (ctx->rlc_deterministic) { key = rlc_key_from_seed(seed); return SSB_OK; }
  uint8_t* p = (uint8_t*)key.w;
  size_t got = 0;
  while (got < sizeof(key.w)) {
    const ssize_t r = getrandom(p + got, sizeof(key.w) - got, 0);
    if (r < 0) {
      if (errno == EINTR) continue;
      ctx->err = "getrandom failed: no entropy for the RLC scalars";
      return SSB_EINVAL;
    }
    got += (size_t)r;
  }
  key.w[0] ^= (uint32_t)seed;
  key.w[1] ^= (uint32_t)(seed >> 32);
  return SSB_OK;
}

// The verification stage shared by verify_batch and threshold_aggregate_batch.
//
// RLC sums as bucket MSMs (ssb_k_msm.hip).  The window width of each MSM minimises
//   madds (n W (1 - 2^-c))  +  1.5 x window-reduce additions (groups W (2^(c+1) + L (log2 L + 1)))
// and the bucket teams get ~8 entries per lane.
struct msm_plan { msm_cfg g2, g1; uint32_t K; int lj2, lj1; size_t n_ent; bool g1_msm; };
constexpr uint32_t MSM_WMAX = 32;          // windows of the G2 MSM (c >= 2)
constexpr uint32_t MSM_KMAX = 1024u * 1024u;  // bucket keys (two-level scan)

inline int msm_pick_c(size_t n, size_t groups, int cmin, int cmax) {
  double best = 1e300; int bc = cmin;
  for (int c = cmin; c <= cmax; ++c) {
    const double W = (64 + c - 1) / c, B = double(1u << c), L = B < 64 ? B : 64;
    // windows of <= 16 buckets reduce sequentially in one lane (k_msm_window_seq)
    const double reduce = c <= 4 ? 2.0 * (B - 1.0) : 2.0 * B + L * (std::log2(L) + 1.0);
    const double cost = double(n) * W * (1.0 - 1.0 / B) + 1.5 * double(groups) * W * reduce;
    if (cost < best) { best = cost; bc = c; }
  }
  return bc;
}
inline int msm_pick_lj(size_t n, size_t groups, int c) {
  const double per_bucket = double(n) / (double(groups) * double(1u << c));
  int lj = 0;
  while (lj < 6 && per_bucket / double(1 << (lj + 1)) >= 8.0) ++lj;
  return lj;
}
// G1 side: a per-root bucket MSM only when the roots' groups are large; otherwise per-share
// products (k_rlc_pk) + per-root segmented sums.  SSB_G1_PATH=msm|share forces one (tests).
bool g1_use_msm(size_t n, size_t n_roots) {
  const char* e = getenv("SSB_G1_PATH");
  if (e && !strcmp(e, "msm")) return true;
  if (e && !strcmp(e, "share")) return false;
  return n >= 128 * (n_roots ? n_roots : 1);
}
// Exact verdicts of a failed batch: group tests (default) or SSB_FALLBACK=share, one pairing check
// per candidate share (kept for the tests and as the measured comparison).
bool fallback_per_share() {
  const char* e = getenv("SSB_FALLBACK");
  return e && !strcmp(e, "share");
}
// One-stream slots run their whole batch on the slot's stream: the verdicts, the exact fallback
// (no-ops when the batch passed) and ONE combine from the verdicts follow the final exponentiation
// in order -- every hardware queue carries one slot (round 2: a shared tail stream finished the
// batches one at a time, ~0.7 ms apart, once the pairing chains of all slots ended together).  The
// three-stream latency configuration runs them on the context's spec / tail streams.
bool post_on_slot(const ssb_slot* s) { return s->shared; }
// One batch in flight on the context (ssb_set_pipeline_depth(1)): the MSM launches take their latency
// forms (lane-program G2 window sums, the cofactor clearing beside the bucket sums; ssb_k_msm.hip).
// SSB_MSM_LAT=0 keeps the pipelined forms (tests compare both).
bool latency_forms(const ssb_ctx* ctx) {
  // SSB_MSM_LAT: "0" never, "a" at every pipeline depth (experiment), unset: one slot only
  static const int mode = [] { const char* e = getenv("SSB_MSM_LAT"); return !e ? 1 : e[0] == '0' ? 0 : e[0] == 'a' ? 2 : 1; }();
  return mode == 2 || (mode == 1 && ctx->nslots == 1);
}
// g1_pre: the public keys come from the cache, which holds their precomputed bases (ctx->pkc_pow):
// the G1 side is one merged 4-bit MSM per root (msm_cfg::merged)
msm_plan plan_msm(size_t n, size_t n_roots, bool g1_pre = false) {
  msm_plan p;
  const size_t g1n = n_roots ? n_roots : 1;
  p.g1_msm = g1_use_msm(n, n_roots);
  int c2 = msm_pick_c(n, 1, 3, 8), c1 = msm_pick_c(n, g1n, 2, 8);  // c <= 8: <= 4 buckets per window lane
  auto keys = [&](int c, size_t g) { return (size_t)((64 + c - 1) / c) * g << c; };
  while (c1 > 2 && keys(c2, 1) + keys(c1, g1n) > MSM_KMAX) --c1;
  p.g2 = msm_cfg{(uint32_t)c2, (uint32_t)((64 + c2 - 1) / c2), 0u, 1u, 0u};
  p.g1 = msm_cfg{(uint32_t)c1, p.g1_msm ? (uint32_t)((64 + c1 - 1) / c1) : 0u, (uint32_t)keys(c2, 1), (uint32_t)g1n, 0u};
  p.K = (uint32_t)(keys(c2, 1) + (p.g1_msm ? keys(c1, g1n) : 0));
  p.lj2 = msm_pick_lj(n, 1, c2);
  p.lj1 = msm_pick_lj(n, g1n, c1);
  if (g1_pre && p.g1_msm) {
    p.g1 = msm_cfg{4u, PKPOW_W, (uint32_t)keys(c2, 1), (uint32_t)g1n, 1u};
    p.K = (uint32_t)(keys(c2, 1) + (g1n << 4));
    p.lj1 = msm_pick_lj(n * PKPOW_W, g1n, 4);   // every window's entries land in the root's 16 buckets
  }
  p.n_ent = n * (p.g2.W + p.g1.W);
  return p;
}
// workspace sizes: the larger of the two G1 layouts (a slot's workspace serves both)
msm_plan plan_size(size_t n, size_t n_roots) {
  msm_plan a = plan_msm(n, n_roots, false);
  const msm_plan b = plan_msm(n, n_roots, true);
  a.K = std::max(a.K, b.K);
  a.n_ent = std::max(a.n_ent, b.n_ent);
  return a;
}

struct verify_ws {
  msm_plan plan;
  g2_aff* H;          // pair Q points: H(root r) for r < n_roots, then the G2 MSM windows
  g1_aff* pair_p;     // pair P points: root sums, then [2^(c w)](-g1)
  g2_aff* sig_aff; g1_aff* pk_aff; uint32_t* flags; uint32_t* sflags; uint32_t* pflags; uint32_t* gflags; uint32_t* gexc;
  fp12* f; uint32_t* ok;
  uint32_t* tickets;   // fused launches: completion tickets of the blocks (zeroed by k_prep_fused, and
                       // again by the blocks that consume them): [0, 4) sort / windows / clears,
                       // [4, 4 + ntk_miller) k_miller_final's
  uint32_t ntk;
  char* hws;          // staged hash_to_G2 workspace
  uint32_t* cnt; uint32_t* start; uint32_t* cur; uint32_t* sbsum; uint32_t* ent;   // MSM counting sort
  uint32_t* order;                                                                 // buckets by count
  g2_jac* b2; g1_jac* b1; g1_jac* w1;                                              // MSM buckets / windows
  g1_jac* rpk; uint32_t* rcnt; uint32_t* rstart; uint32_t* rcur; uint32_t* perm;   // per-share G1 path
  g2_jac* rsig; uint32_t* gst; uint8_t* gv0; uint8_t* gv1;                         // failed-batch group tests
  uint64_t* k64; g2_jac* fbX; uint32_t* rtk; uint32_t* nfail;                                     // (level 0 per root)
  uint32_t* slist; uint32_t* xok; fp12* fex; uint32_t* kcnt; uint32_t* kstart; uint32_t* klist;   // committee stage
  size_t npairs;
};
// Miller values of the pairs plus the levels of the 8-ary product tree
inline size_t fp12_slots(size_t np) {
  size_t tot = np;
  while (np > 8) { np = (np + 7) / 8; tot += np; }
  return tot + 2;   // (+ k_miller_final's product before the final exponentiation)
}
// the ticket block of the fused path: [0, 4) sort / windows / clears, [4, 5 + ceil(np / 8))
// k_miller_final's, then the fallback's committee stage: nS (suspects listed), xtk[2]
inline uint32_t ntk_words(size_t np) { return 4 + 1 + (uint32_t)((np + 7) / 8) + 3; }

// the tree's per-share products rsig / rpk; the committee stage's group-test mode (k_fb_excl) keeps
// its four quarter sums per (root, id bucket) key in the same buffers
inline size_t fb_prod_slots(size_t n, size_t n_roots) { return std::max(n, 4 * launch::fb_keys(n_roots)); }
// the fallback's quarter sums: k_fb_root's four per root, k_fb_excl's four per part of X
inline size_t fb_x_slots(size_t n_roots) { return std::max(4 * n_roots, (size_t)(4 * launch::EX_X_PARTS)); }
size_t verify_ws_bytes(size_t n, size_t n_roots) {
  const msm_plan p = plan_size(n, n_roots);
  const size_t np = n_roots + MSM_WMAX;
  return align_up(np * sizeof(g2_aff)) + align_up(np * sizeof(g1_aff)) + align_up(n * sizeof(g2_aff)) +
         align_up(n * sizeof(g1_aff)) + align_up(n * 4) * 5 + align_up(fp12_slots(np) * sizeof(fp12)) + align_up(4) +
         align_up((4 + 1 + (np + 7) / 8) * 4) +
         align_up(launch::hash_ws_bytes(n_roots)) + 4 * align_up((size_t)p.K * 4) + align_up(1024 * 4) +
         align_up(p.n_ent * 4) + align_up(((size_t)p.g2.W << p.g2.c) * sizeof(g2_jac)) +
         align_up(((size_t)p.g1.ngroups * p.g1.W << p.g1.c) * sizeof(g1_jac)) +
         align_up((size_t)p.g1.ngroups * p.g1.W * sizeof(g1_jac)) + align_up(fb_prod_slots(n, n_roots) * sizeof(g1_jac)) +
         3 * align_up(n_roots * 4) + align_up(n * 4) + align_up(fb_prod_slots(n, n_roots) * sizeof(g2_jac)) +
         align_up((size_t)launch::fallback_levels(n) * (n_roots + 1) * 4) + 2 * align_up(n + n_roots) +
         align_up(n * 8) + align_up(fb_x_slots(n_roots) * sizeof(g2_jac)) + align_up(n_roots * 4) + align_up(4) +
         align_up(n * 4) + align_up(4) + align_up((size_t)launch::ex_pairs((int)n_roots) * sizeof(fp12)) + align_up(ntk_words(np) * 4) +
         3 * align_up(launch::fb_keys(n_roots) * 4) + align_up((launch::fb_keys(n_roots) + 1) * 4);
}

verify_ws carve_verify(carve& c, size_t n, size_t n_roots, bool g1_pre = false) {
  verify_ws w;
  const msm_plan sz = plan_size(n, n_roots);   // (the same layout for both G1 forms)
  w.plan = plan_msm(n, n_roots, g1_pre);
  const size_t np = n_roots + MSM_WMAX;
  w.H = c.take<g2_aff>(np); w.pair_p = c.take<g1_aff>(np);
  w.sig_aff = c.take<g2_aff>(n); w.pk_aff = c.take<g1_aff>(n);
  w.flags = c.take<uint32_t>(n); w.sflags = c.take<uint32_t>(n); w.pflags = c.take<uint32_t>(n);
  w.gflags = c.take<uint32_t>(n); w.gexc = c.take<uint32_t>(n);
  w.f = c.take<fp12>(fp12_slots(np)); w.ok = c.take<uint32_t>(1);
  w.ntk = ntk_words(np);
  w.tickets = c.take<uint32_t>(w.ntk);
  w.hws = c.take<char>(launch::hash_ws_bytes(n_roots));
  w.cnt = c.take<uint32_t>(sz.K); w.start = c.take<uint32_t>(sz.K); w.cur = c.take<uint32_t>(sz.K);
  w.sbsum = c.take<uint32_t>(1024); w.ent = c.take<uint32_t>(sz.n_ent); w.order = c.take<uint32_t>(sz.K);
  w.b2 = c.take<g2_jac>((size_t)sz.g2.W << sz.g2.c);
  w.b1 = c.take<g1_jac>((size_t)sz.g1.ngroups * sz.g1.W << sz.g1.c);   // >= the merged layout's ngroups << 4
  w.w1 = c.take<g1_jac>((size_t)sz.g1.ngroups * sz.g1.W);
  w.rpk = c.take<g1_jac>(fb_prod_slots(n, n_roots));
  w.rcnt = c.take<uint32_t>(n_roots); w.rstart = c.take<uint32_t>(n_roots); w.rcur = c.take<uint32_t>(launch::fb_keys(n_roots));
  w.perm = c.take<uint32_t>(n);
  w.rsig = c.take<g2_jac>(fb_prod_slots(n, n_roots));
  w.gst = c.take<uint32_t>((size_t)launch::fallback_levels(n) * (n_roots + 1));
  w.gv0 = c.take<uint8_t>(n + n_roots); w.gv1 = c.take<uint8_t>(n + n_roots);
  w.k64 = c.take<uint64_t>(n); w.fbX = c.take<g2_jac>(fb_x_slots(n_roots)); w.rtk = c.take<uint32_t>(n_roots); w.nfail = c.take<uint32_t>(1);
  w.slist = c.take<uint32_t>(n); w.xok = c.take<uint32_t>(1); w.fex = c.take<fp12>((size_t)launch::ex_pairs((int)n_roots));
  w.kcnt = c.take<uint32_t>(launch::fb_keys(n_roots)); w.kstart = c.take<uint32_t>(launch::fb_keys(n_roots));
  w.klist = c.take<uint32_t>(launch::fb_keys(n_roots) + 1);
  w.npairs = n_roots + w.plan.g2.W;
  return w;
}

// The fused one-stream path (every stage on the slot's stream, the counting sort and the hash
// stages riding along the per-share launches): one-stream slot, a per-root G1 bucket MSM with
// windows of <= 16 buckets, and the sort's keys within FUSED_SORT_KMAX.
bool fused_sort_path(const ssb_slot* S, size_t n, size_t n_roots, bool g1_pre = false) {
  if (!S->shared || !n || !n_roots) return false;
  const msm_plan P = plan_msm(n, n_roots, g1_pre);
  const char* sgp = getenv("SSB_SUBGROUP");
  return P.g1_msm && launch::msm_fused_ok(P.g1) && !(sgp && sgp[0] == 'l') && P.K <= launch::FUSED_SORT_KMAX;
}

// the merged G1 MSM over the key cache's precomputed bases: cached keys, bases present, and the
// fused one-stream path (the only one whose launches know the merged layout)
bool g1_pre_path(const ssb_ctx* ctx, const uint32_t* pk_index, size_t n, size_t n_roots) {
  if (!pk_index || !ctx->pkc_pow || getenv("SSB_NO_PKPOW")) return false;
  const msm_plan P = plan_msm(n, n_roots, true);
  return P.g1.merged && fused_sort_path(ctx->cur, n, n_roots, true);
}

// jm (aggregate path on the fused path): the share -> (job, root) map is computed by the decode
// launch (d_share_root == jm->share_root) instead of a k_share_map launch in front of the batch
template <class F>
int run_verify(ssb_ctx* ctx, const verify_ws& w, size_t n, size_t n_roots, const uint8_t* d_sig, const uint8_t* d_pk,
               const uint32_t* d_pk_index, const uint32_t* d_share_root, const uint8_t* d_roots, const dst_arg& dst, uint64_t rlc_seed,
               uint8_t* d_verdict, F on_decoded, hipStream_t tail, const spec_jobs* sj = nullptr,
               bool* spec_done = nullptr, const job_map* jm = nullptr) {
  rlc_key key;
  if (int rc = draw_rlc_key(ctx, rlc_seed, key)) return rc;
  hipStream_t st = ctx->cur->stream, sh = ctx->cur->side[0], s1 = ctx->cur->side[1];
  const msm_plan& P = w.plan;
  // One-stream slots: the G2 and G1 MSMs share launches (msm_both), and the hash_to_G2 stages ride
  // along the batch's own kernels -- the SWU map beside the subgroup checks, the cofactor clearing
  // beside the bucket sums, the affine output beside the window sums -- instead of standing in
  // front of the decode on the slot's stream (their few latency-bound waves fill no device).
  const bool fused = ctx->cur->shared && s1 == st && P.g1_msm && launch::msm_fused_ok(P.g1);
  const char* sgp = getenv("SSB_SUBGROUP");
  const bool fuse_hash = fused && sh == st && n && n_roots && !(sgp && sgp[0] == 'l');
  const launch::h2c_ws hw = launch::carve_h2c(w.hws, n_roots);
  // ... and the MSM entries' counting sort rides along the decode and the subgroup checks
  const bool fuse_sort = fuse_hash && P.K <= launch::FUSED_SORT_KMAX;
  if (jm && !fuse_sort) { ctx->err = "internal: share map expected on the fused path"; return SSB_EINVAL; }
  const launch::fused_sort fs{key, d_share_root, P.g2, P.g1, P.K, w.cnt, w.start, w.cur, w.ent, w.order,
                              w.pflags, (uint32_t)n_roots, w.flags, w.tickets, w.ntk, jm ? *jm : job_map{}};
  // hash_to_G2 per root runs beside decode / RLC / sums; the Miller loops wait for it
  // (events only between distinct streams: on one stream the order is given, and every record or
  // wait is one more packet in the slot's queue)
  if (sh != st) {
    SSB_HIP(hipEventRecord(ctx->cur->ev_in, st));
    SSB_HIP(hipStreamWaitEvent(sh, ctx->cur->ev_in, 0));
  }
  // counts and tickets left clean by the slot's previous batch (same workspace layout): no prep
  // launch -- the hash's first stage rides along the decode instead.  A small launch in front of
  // the decode waited for a free wave slot behind the other slots' decode waves (~1.5 ms on the
  // last batches of the driver's run, profiles/r02_gate_timeline.txt)
  const bool clean = fuse_sort && n && ctx->cur->clean_cnt == w.cnt && ctx->cur->clean_tickets == w.tickets &&
                     ctx->cur->clean_K >= P.K;
  // this batch's counts / tickets are clean at its end only on the fused path (its scan and last
  // blocks reset them); any other path writes the workspace without leaving them clean
  if (fuse_sort) { ctx->cur->clean_cnt = w.cnt; ctx->cur->clean_tickets = w.tickets; ctx->cur->clean_K = P.K; }
  else ctx->cur->clean_cnt = nullptr;
  if (fuse_sort && !clean) {
    launch::prep_fused(st, fs, (int)n_roots, d_roots, dst, hw);
  } else if (fuse_sort) {
  } else if (fuse_hash) {
    launch::h2c_u(st, (int)n_roots, d_roots, dst, hw);
  } else {
    if (n_roots) { timed t(ctx, "k_hash_to_g2", sh); launch::hash_to_g2(sh, (int)n_roots, d_roots, dst, w.H, w.hws); }
    if (sh != st) SSB_HIP(hipEventRecord(ctx->cur->ev_hash, sh));
  }
  if (fuse_sort) {
    timed t(ctx, "k_decode");
    launch::decode_count(st, (int)n, d_sig, d_pk, d_pk_index, (uint32_t)ctx->pkc_n, (const g1_aff*)ctx->pkc_aff,
                         (const uint32_t*)ctx->pkc_flags, w.sig_aff, w.pk_aff, w.sflags, w.pflags, fs, (int)n_roots,
                         d_roots, clean ? &dst : nullptr, clean ? &hw : nullptr);
  } else if (n) {
    timed t(ctx, "k_decode");
    if (d_pk_index) {
      hipLaunchKernelGGL(k_decode_sig, dim3(nblk(n, 64)), dim3(64), 0, st, (int)n, d_sig, w.sig_aff, w.sflags);
      hipLaunchKernelGGL(k_pk_gather, dim3(nblk(n, 256)), dim3(256), 0, st, (int)n, d_pk_index, (uint32_t)ctx->pkc_n,
                         (const g1_aff*)ctx->pkc_aff, (const uint32_t*)ctx->pkc_flags, w.pk_aff, w.pflags);
    } else {
      hipLaunchKernelGGL(k_decode2, dim3(nblk(2 * n, 64)), dim3(64), 0, st, (int)n, d_sig, d_pk, w.sig_aff, w.pk_aff, w.sflags, w.pflags);
    }
  }
  // side[1]: per-share G1 products and the root segments, beside the subgroup checks
  if (s1 != st) {
    SSB_HIP(hipEventRecord(ctx->cur->ev_sdec, st));
    SSB_HIP(hipStreamWaitEvent(s1, ctx->cur->ev_sdec, 0));
  }
  if (!P.g1_msm) {
    timed t(ctx, "k_rlc_pk", s1);
    if (n) hipLaunchKernelGGL(k_rlc_pk, dim3(nblk(n, 64)), dim3(64), 0, s1, (int)n, key, w.sflags, w.pflags, w.pk_aff, w.rpk);
    SSB_HIP(hipMemsetAsync(w.rcnt, 0, n_roots * 4, s1));
    if (n) hipLaunchKernelGGL(k_root_hist, dim3(nblk(n, 256)), dim3(256), 0, s1, (int)n, (int)n_roots, d_share_root, w.rcnt);
    hipLaunchKernelGGL(k_root_scan, dim3(1), dim3(64), 0, s1, (int)n_roots, w.rcnt, w.rstart, w.rcur);
    if (n) hipLaunchKernelGGL(k_root_scatter, dim3(nblk(n, 256)), dim3(256), 0, s1, (int)n, (int)n_roots, d_share_root, w.rcur, w.perm);
  }
  if (fuse_sort) {   // (the scans ran in the decode launch's last count block)
    timed t(ctx, "k_subgroup");
    launch::subgroup_map(st, (int)n, w.sflags, w.sig_aff, w.gflags, &hw, (int)n_roots, &fs);   // + flags, scatter
  } else {
  { timed t(ctx, "k_msm_sort"); launch::msm_sort(st, (int)n, key, w.sflags, w.pflags, d_share_root, P.g2, P.g1, P.K, w.cnt, w.start, w.cur, w.sbsum, w.ent, w.order); }
  if (n) {
    if (fuse_hash) { timed t(ctx, "k_subgroup"); launch::subgroup_map(st, (int)n, w.sflags, w.sig_aff, w.gflags, &hw, (int)n_roots); }
    else { timed t(ctx, "k_subgroup"); launch::subgroup(st, (int)n, w.sflags, w.sig_aff, w.gflags, w.gexc); }
    hipLaunchKernelGGL(k_flags, dim3(nblk(n, 256)), dim3(256), 0, st, (int)n, w.sflags, w.pflags, w.gflags, d_share_root,
                       (uint32_t)n_roots, w.flags);
  }
  }
  if (s1 != st || !post_on_slot(ctx->cur)) SSB_HIP(hipEventRecord(ctx->cur->ev_dec, st));   // s1 / the spec stream
  // G1 sums (per root) on side[1] -- then the caller's speculative combine, off the critical path --
  // G2 MSM on the main stream.  One-stream slots: both MSMs in the same three launches (they
  // overlap on the device instead of running back to back on the slot's stream).
  if (fused) {
    if (n) on_decoded();
    timed t(ctx, "k_msm_g2");
    if (P.g1.merged && !(fuse_sort && d_pk_index && ctx->pkc_pow)) { ctx->err = "internal: merged G1 MSM off the fused cached path"; return SSB_EINVAL; }
    launch::msm_both(st, P.g2, P.lj2, P.g1, P.lj1, w.order, w.start, w.cur, w.ent, w.flags, w.sig_aff, w.pk_aff, w.b2, w.b1,
                     w.H + n_roots, w.pair_p + n_roots, ctx->negg1_pow, w.w1, w.pair_p, fuse_hash ? &hw : nullptr,
                     (int)n_roots, w.H, fuse_sort ? w.tickets : nullptr, (const g1_aff*)ctx->pkc_pow, d_pk_index,
                     latency_forms(ctx));
  } else {
  if (s1 != st) SSB_HIP(hipStreamWaitEvent(s1, ctx->cur->ev_dec, 0));
  if (P.g1_msm) {
    timed t(ctx, "k_msm_g1", s1);
    launch::msm_g1(s1, P.g1, P.lj1, w.order, w.start, w.cur, w.ent, w.flags, w.pk_aff, w.b1, w.w1, w.pair_p);
  } else {
    timed t(ctx, "k_sum_g1", s1);
    hipLaunchKernelGGL(k_sum_seg, dim3((unsigned)n_roots), dim3(SEG_THREADS), 0, s1, (int)n_roots, w.rstart, w.rcnt, w.perm,
                       w.flags, w.rpk, (const g2_jac*)nullptr, w.pair_p, (g2_aff*)nullptr);
  }
  if (s1 != st) SSB_HIP(hipEventRecord(ctx->cur->ev_r1, s1));
  if (n) on_decoded();
  { timed t(ctx, "k_msm_g2"); launch::msm_g2(st, P.g2, P.lj2, w.order, w.start, w.cur, w.ent, w.flags, w.sig_aff, w.b2, w.H + n_roots, w.pair_p + n_roots, ctx->negg1_pow); }
  }
  if (!fused && s1 != st) SSB_HIP(hipStreamWaitEvent(st, ctx->cur->ev_r1, 0));
  if (!fuse_hash && sh != st) SSB_HIP(hipStreamWaitEvent(st, ctx->cur->ev_hash, 0));
  // one-stream slots: the speculative combine rides along the Miller loops (a few latency-bound
  // blocks), so a passing batch's tail is only no-op launches
  spec_jobs sjv{};
  unsigned nbsp = 0;
  if (sj && sj->n_jobs > 0 && st == ctx->cur->stream) { sjv = *sj; nbsp = (unsigned)((sj->n_jobs + 63) / 64); }
  if (spec_done) *spec_done = nbsp > 0;
  // the fused path: Miller loops, product tree and final exponentiation in ONE launch (completion
  // tickets of the fused path's workspace); the fast verdicts then come grid-wide from k_fb_rlc
  const bool miller_final = fuse_sort && !fallback_per_share();
  if (miller_final) {
    timed t(ctx, "k_miller");
    hipLaunchKernelGGL(k_miller_final, dim3((unsigned)w.npairs + nbsp), dim3(64), 0, st, (int)w.npairs, w.pair_p, w.H, w.f, sjv,
                       w.tickets + 4, w.ok);
  } else {
    {
      timed t(ctx, "k_miller");
      hipLaunchKernelGGL(k_miller_pairs, dim3((unsigned)w.npairs + nbsp), dim3(64), 0, st, (int)w.npairs, w.pair_p, w.H, w.f, sjv);
    }
    timed t(ctx, "k_final");
    int np = (int)w.npairs;
    fp12* cur = w.f;
    while (np > 8) {
      const int nparts = (np + 7) / 8;
      hipLaunchKernelGGL(k_fp12_prod8, dim3((unsigned)nparts), dim3(64), 0, st, np, cur, cur + np);
      cur += np; np = nparts;
    }
    // (the per-share fallback leaves the fast verdicts to k_final_lane; the group-test fallback
    // writes them grid-wide in k_fb_rlc)
    hipLaunchKernelGGL(k_final_lane, dim3(1), dim3(64), 0, st, np, cur, w.ok, (int)n, (const uint32_t*)w.flags,
                       fallback_per_share() ? d_verdict : (uint8_t*)nullptr);
  }
  // the exact fallback when the batch failed: on the slot's own stream (one-stream slots), or the
  // context's tail stream (three-stream configuration)
  const bool fb_tail = !post_on_slot(ctx->cur);
  hipStream_t fbs = fb_tail ? tail : st;
  if (fb_tail && tail != st) {
    SSB_HIP(hipEventRecord(ctx->cur->ev_fin, st));
    SSB_HIP(hipStreamWaitEvent(tail, ctx->cur->ev_fin, 0));
  }
  if (n) {
    timed t(ctx, "k_fallback_verify", fbs);
    // (the fast verdicts -- a passing batch, non-candidates -- come from k_final_lane on the per-share
    // path, from k_fb_rlc on the group-test path)
    if (fallback_per_share())
      hipLaunchKernelGGL(k_fallback_lane, dim3((unsigned)std::min<size_t>(n, 1024)), dim3(64), 0, fbs, (int)n, w.ok, w.flags,
                         d_share_root, w.H, w.sig_aff, w.pk_aff, d_verdict);
    else
    {
      // the committee stage (fused path of an aggregate batch: its jobs, and k_miller_final's product)
      const bool cm = miller_final && sj && sj->n_jobs > 0 && !getenv("SSB_NO_COMMITTEE");
      const uint32_t* ptk = w.tickets + w.ntk - 3;
      launch::fb_ws fw{w.rcnt, w.rstart, w.rcur, w.perm, w.gst, w.rtk, w.nfail, w.k64, w.fbX, w.rsig, w.rpk, w.gv0, w.gv1,
                       cm ? w.slist : nullptr, cm ? (uint32_t*)ptk : nullptr, cm ? (uint32_t*)ptk + 1 : nullptr,
                       cm ? w.xok : nullptr, cm ? w.fex : nullptr,
                       cm ? w.f + w.npairs + (w.npairs + 7) / 8 : nullptr, cm ? w.kcnt : nullptr, cm ? w.kstart : nullptr,
                       ctx->negg1_pow, cm ? w.klist : nullptr};
      const launch::fb_jobs fj = cm ? launch::fb_jobs{sj->n_jobs, sj->off, sj->tt, sj->ids} : launch::fb_jobs{0, nullptr, nullptr, nullptr};
      launch::fallback_bisect(fbs, (int)n, (int)n_roots, key, w.ok, w.flags, d_share_root, w.H, w.sig_aff, w.pk_aff, w.f,
                              fw, d_verdict, true, fj);
    }
  }
  if (!fb_tail && tail != st) {
    SSB_HIP(hipEventRecord(ctx->cur->ev_fin, st));
    SSB_HIP(hipStreamWaitEvent(tail, ctx->cur->ev_fin, 0));
  }
  SSB_HIP(hipGetLastError());
  return SSB_OK;
}

}  // namespace

namespace ssb {
int ctx_device(const ssb_ctx* ctx) { return ctx->device; }   // (ssb_collector.hip)
std::recursive_mutex& ctx_mutex(ssb_ctx* ctx) { return ctx->mu; }
// (ssb_collector.hip, under the context lock) a collector attaches with one-stream slots at depth
// in_flight -- configuring the context if it is the first -- or detaches (d < 0)
int ctx_attach_collector(ssb_ctx* ctx, int d, int in_flight) {
  if (d < 0) { if (ctx->collectors > 0) --ctx->collectors; return SSB_OK; }
  if (ctx->collectors) {
    if (ctx->slot_streams != 1 || ctx->nslots != in_flight) {
      ctx->err = "another collector is attached with a different in_flight (" + std::to_string(ctx->nslots) + ")";
      return SSB_EINVAL;
    }
  } else {
    int rc;
    if ((rc = ssb_set_slot_streams(ctx, 1)) || (rc = ssb_set_pipeline_depth(ctx, in_flight))) return rc;
  }
  ++ctx->collectors;
  return SSB_OK;
}
}

extern "C" {

int ssb_create(ssb_ctx** out, int device_ordinal) {
  if (!out) return SSB_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SSB_EHIP;
  if (device_ordinal < 0 || device_ordinal >= ndev) return SSB_EINVAL;
  if (hipSetDevice(device_ordinal) != hipSuccess) return SSB_EHIP;
  ssb_ctx* ctx = new (std::nothrow) ssb_ctx();
  if (!ctx) return SSB_ENOMEM;
  ctx->device = device_ordinal;
  ctx->hw_queues = ssb_hw_queue_budget();
  if (init_slot(ctx, ctx->sl[0], ctx->slot_streams) != SSB_OK) { free_slot(ctx, ctx->sl[0]); delete ctx; return SSB_EHIP; }
  if (ctx_streams(ctx, ctx->slot_streams == 3) != SSB_OK) { free_slot(ctx, ctx->sl[0]); delete ctx; return SSB_EHIP; }
  {  // [2^s](-g1) for the window pairs of the G2 MSM
    g1_aff h[64];
    g1_jac p; jac_from_aff(p, g1_neg_generator());
    for (int i = 0; i < 64; ++i) { jac_to_aff(h[i], p); jac_dbl(p, p); }
    if (hipMalloc(&ctx->negg1_pow, sizeof(h)) != hipSuccess ||
        hipMemcpy(ctx->negg1_pow, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) {
      free_slot(ctx, ctx->sl[0]); ctx_streams(ctx, false); delete ctx; return SSB_EHIP;
    }
  }
  *out = ctx;
  return SSB_OK;
}

void ssb_destroy(ssb_ctx* ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->device);
  for (int i = 0; i < ctx->nslots; ++i) sync_slot(ctx, ctx->sl[i]);
  for (auto& kv : ctx->timers) { if (kv.second.a) hipEventDestroy(kv.second.a); if (kv.second.b) hipEventDestroy(kv.second.b); }
  for (auto& kv : ctx->history) for (auto& p : kv.second) { hipEventDestroy(p.a); hipEventDestroy(p.b); }
  for (auto& p : ctx->pool) { hipEventDestroy(p.a); hipEventDestroy(p.b); }
  if (ctx->io) hipFree(ctx->io);
  if (ctx->negg1_pow) hipFree(ctx->negg1_pow);
  if (ctx->pkc_aff) hipFree(ctx->pkc_aff);
  if (ctx->pkc_flags) hipFree(ctx->pkc_flags);
  if (ctx->pkc_pow) hipFree(ctx->pkc_pow);
  if (ctx->pkc_stage) hipFree(ctx->pkc_stage);
  ctx_streams(ctx, false);
  for (int i = 0; i < ctx->nslots; ++i) free_slot(ctx, ctx->sl[i]);
  delete ctx;
}

int ssb_check_pipeline_config(int depth, int streams) {
  if (depth < 1 || depth > SSB_MAX_SLOTS || (streams != 1 && streams != 3)) return SSB_EINVAL;
  // the HIP runtime reserves scratch per hardware queue for the largest kernel each queue ran:
  // 8 slots x 3 streams ran out (HSA_STATUS_ERROR_OUT_OF_RESOURCES -- the side streams run the
  // large-scratch kernels); one-stream slots run clean up to SSB_MAX_SLOT_STREAMS
  if (depth * streams > SSB_MAX_SLOT_STREAMS || (streams == 3 && depth > SSB_MAX_THREE_STREAM_SLOTS)) return SSB_EINVAL;
  return SSB_OK;
}

int ssb_hw_queue_budget(void) {
  const char* v = getenv("GPU_MAX_HW_QUEUES");
  const int q = v ? atoi(v) : 0;
  return q > 0 ? q : 4;   // HIP's default
}

namespace {
// slot streams beyond the process's hardware queues share queues: independent batches then
// serialise behind each other (round 2: 21 active queues on 20 measured 6.5 M against 9.3 M), so
// such a configuration is refused with the reason instead of running silently slower
int check_queue_budget(ssb_ctx* ctx, int depth, int streams) {
  if (depth * streams <= ctx->hw_queues - 1) return SSB_OK;   // one queue left for the caller's stream
  ctx->err = "pipeline depth " + std::to_string(depth) + " x " + std::to_string(streams) +
             " streams per slot needs " + std::to_string(depth * streams + 1) +
             " hardware queues, but this process has GPU_MAX_HW_QUEUES=" + std::to_string(ctx->hw_queues) +
             " (HIP's default is 4; set GPU_MAX_HW_QUEUES, at most 32, in the environment before the first HIP call)";
  return SSB_EINVAL;
}
}  // namespace

namespace {
// a collector owns the slot configuration it was created with: its worker picks slots round robin
// over in_flight of them (a depth below in_flight left it a null slot stream)
int check_no_collector(ssb_ctx* ctx) {
  if (!ctx->collectors) return SSB_OK;
  ctx->err = "a collector is attached to this context: its slot configuration cannot change (ssb_collector_destroy first)";
  return SSB_EINVAL;
}
}  // namespace

int ssb_set_pipeline_depth(ssb_ctx* ctx, int depth) {
  if (!ctx) return SSB_EINVAL;
  SSB_LOCK(ctx);
  if (int rc = check_no_collector(ctx)) return rc;
  if (ssb_check_pipeline_config(depth, ctx->slot_streams) != SSB_OK) {
    ctx->err = "pipeline depth x streams per slot outside the supported range (one-stream slots: depth 1..20; three-stream slots: depth 1..5)";
    return SSB_EINVAL;
  }
  if (int rc = check_queue_budget(ctx, depth, ctx->slot_streams)) return rc;
  SSB_HIP(hipSetDevice(ctx->device));
  for (int i = ctx->nslots; i < depth; ++i) {
    if (init_slot(ctx, ctx->sl[i], ctx->slot_streams) != SSB_OK) { ctx->err = "stream/event creation failed"; return SSB_EHIP; }
    ctx->nslots = i + 1;
  }
  for (int i = depth; i < ctx->nslots; ++i) { sync_slot(ctx, ctx->sl[i]); free_slot(ctx, ctx->sl[i]); ctx->sl[i] = ssb_slot(); }
  ctx->nslots = depth;
  ctx->next = 0;
  // the synchronous entry points run on ctx->cur: never leave it on a removed (reset) slot
  ctx->cur = &ctx->sl[0];
  return SSB_OK;
}

int ssb_set_slot_streams(ssb_ctx* ctx, int streams) {
  if (!ctx) return SSB_EINVAL;
  SSB_LOCK(ctx);
  if (int rc = check_no_collector(ctx)) return rc;
  if (ssb_check_pipeline_config(ctx->nslots, streams) != SSB_OK) {
    ctx->err = "streams per slot must be 1 or 3, and three-stream slots at most 5 (lower the depth first)";
    return SSB_EINVAL;
  }
  if (int rc = check_queue_budget(ctx, ctx->nslots, streams)) return rc;
  if (streams == ctx->slot_streams) return SSB_OK;
  SSB_HIP(hipSetDevice(ctx->device));
  for (int i = 0; i < ctx->nslots; ++i) { sync_slot(ctx, ctx->sl[i]); free_slot(ctx, ctx->sl[i]); ctx->sl[i] = ssb_slot(); }
  ctx->slot_streams = streams;
  for (int i = 0; i < ctx->nslots; ++i)
    if (init_slot(ctx, ctx->sl[i], streams) != SSB_OK) { ctx->err = "stream/event creation failed"; return SSB_EHIP; }
  if (ctx_streams(ctx, streams == 3) != SSB_OK) { ctx->err = "stream creation failed"; return SSB_EHIP; }
  ctx->next = 0;
  ctx->cur = &ctx->sl[0];
  return SSB_OK;
}

int ssb_set_rlc_deterministic(ssb_ctx* ctx, int on) {
  if (!ctx) return SSB_EINVAL;
  SSB_LOCK(ctx);
  ctx->rlc_deterministic = on != 0;
  return SSB_OK;
}

int ssb_debug_hold(void* stream, const uint32_t* flag, uint32_t max_us) {
  if (!flag) return SSB_EINVAL;
  hipLaunchKernelGGL(k_hold, dim3(1), dim3(64), 0, (hipStream_t)stream, flag, max_us / 2 + 1);
  return hipGetLastError() == hipSuccess ? SSB_OK : SSB_EHIP;
}

void* ssb_slot_stream(ssb_ctx* ctx, int slot) {
  if (!ctx) return nullptr;
  SSB_LOCK(ctx);
  if (slot < 0 || slot >= ctx->nslots) return nullptr;
  return (void*)ctx->sl[slot].stream;
}

// a copy taken under the context lock, per calling thread: a failure on another thread cannot free
// the string while the caller reads it
const char* ssb_last_error(const ssb_ctx* ctx) {
  if (!ctx) return "null context";
  thread_local std::string copy;
  ssb_ctx* c = const_cast<ssb_ctx*>(ctx);
  std::lock_guard<std::recursive_mutex> g(c->mu);
  copy = c->err;
  return copy.c_str();
}

int ssb_last_kernel_ms(const ssb_ctx* ctx_c, const char* name, float* ms) {
  ssb_ctx* ctx = const_cast<ssb_ctx*>(ctx_c);
  if (!ctx || !name || !ms) return SSB_EINVAL;
  SSB_LOCK(ctx);
  auto it = ctx->timers.find(name);
  if (it == ctx->timers.end() || !it->second.used) { ctx->err = "no timing for kernel"; return SSB_EINVAL; }
  SSB_HIP(hipEventSynchronize(it->second.b));
  SSB_HIP(hipEventElapsedTime(ms, it->second.a, it->second.b));
  return SSB_OK;
}

int ssb_kernel_timing(ssb_ctx* ctx, int on) {
  if (!ctx) return SSB_EINVAL;
  SSB_LOCK(ctx);
  for (int i = 0; i < ctx->nslots; ++i) sync_slot(ctx, ctx->sl[i]);
  for (auto& kv : ctx->history) for (auto& p : kv.second) ctx->pool.push_back(p);
  ctx->history.clear();
  ctx->accumulate = on == 1;
  ctx->time_last = on == 2;
  return SSB_OK;
}

int ssb_kernel_time(ssb_ctx* ctx, const char* name, float* total_ms, int* launches) {
  if (!ctx || !name || !total_ms || !launches) return SSB_EINVAL;
  SSB_LOCK(ctx);
  *total_ms = 0.f; *launches = 0;
  auto it = ctx->history.find(name);
  if (it == ctx->history.end()) return SSB_OK;
  for (auto& p : it->second) {
    float ms = 0.f;
    SSB_HIP(hipEventSynchronize(p.b));
    SSB_HIP(hipEventElapsedTime(&ms, p.a, p.b));
    *total_ms += ms; *launches += 1;
  }
  return SSB_OK;
}

namespace {
int hash_to_g2_impl(ssb_ctx* ctx, size_t n, const uint8_t* msgs32, const uint8_t* lens, const uint8_t* dst, size_t dst_len,
                    uint8_t* out192) {
  if (!ctx) return SSB_EINVAL;
  SSB_SYNC_LOCK(ctx);
  if (n == 0) return SSB_OK;
  if (!msgs32 || !out192) { ctx->err = "null pointer"; return SSB_EINVAL; }
  if (lens)
    for (size_t i = 0; i < n; ++i) if (lens[i] > 32) { ctx->err = "message longer than 32 bytes"; return SSB_EINVAL; }
  SSB_HIP(hipSetDevice(ctx->device));
  pick_idle_slot(ctx);
  dst_arg d; int rc = fill_dst(ctx, d, dst, dst_len); if (rc) return rc;
  size_t need = align_up(n * 32) + align_up(n) + align_up(n * sizeof(g2_aff)) + align_up(n * 192) + align_up(launch::hash_ws_bytes(n));
  if ((rc = ensure_ws(ctx, need))) return rc;
  carve c{(char*)ctx->cur->ws};
  uint8_t* d_msg = c.take<uint8_t>(n * 32); uint8_t* d_len = c.take<uint8_t>(n); g2_aff* d_h = c.take<g2_aff>(n);
  uint8_t* d_out = c.take<uint8_t>(n * 192);
  char* hws = c.take<char>(launch::hash_ws_bytes(n));
  SSB_HIP(hipMemcpyAsync(d_msg, msgs32, n * 32, hipMemcpyHostToDevice, ctx->cur->stream));
  if (lens) SSB_HIP(hipMemcpyAsync(d_len, lens, n, hipMemcpyHostToDevice, ctx->cur->stream));
  { timed t(ctx, "k_hash_to_g2"); launch::hash_to_g2(ctx->cur->stream, (int)n, d_msg, d, d_h, hws, lens ? d_len : nullptr); }
  hipLaunchKernelGGL(k_serialize_g2, dim3(nblk(n, 64)), dim3(64), 0, ctx->cur->stream, (int)n, d_h, d_out);
  SSB_HIP(hipGetLastError());
  SSB_HIP(hipMemcpyAsync(out192, d_out, n * 192, hipMemcpyDeviceToHost, ctx->cur->stream));
  { hipStream_t st = ctx->cur->stream; SSB_SYNC_WAIT(st); }
  return SSB_OK;
}
}  // namespace

int ssb_hash_to_g2(ssb_ctx* ctx, size_t n, const uint8_t* msgs32, const uint8_t* dst, size_t dst_len, uint8_t* out192) {
  return hash_to_g2_impl(ctx, n, msgs32, nullptr, dst, dst_len, out192);
}

int ssb_hash_to_g2_msgs(ssb_ctx* ctx, size_t n, const uint8_t* msgs32, const uint8_t* msg_len, const uint8_t* dst,
                        size_t dst_len, uint8_t* out192) {
  if (ctx && n && !msg_len) { ctx->err = "null msg_len"; return SSB_EINVAL; }
  return hash_to_g2_impl(ctx, n, msgs32, msg_len, dst, dst_len, out192);
}

int ssb_feldman_verify_batch(ssb_ctx* ctx, size_t n, size_t t, const uint8_t* commitments48, const uint64_t* ids,
                             const uint8_t* shares32, const uint8_t* h48, uint8_t* verdicts) {
  if (!ctx) return SSB_EINVAL;
  SSB_SYNC_LOCK(ctx);
  if (n == 0) return SSB_OK;
  if (!commitments48 || !ids || !shares32 || !h48 || !verdicts || t == 0 || t > 1024 || n > (size_t)INT32_MAX) {
    ctx->err = "null pointer, t not in [1, 1024] or n too large"; return SSB_EINVAL;
  }
  SSB_HIP(hipSetDevice(ctx->device));
  pick_idle_slot(ctx);
  int rc;
  if ((rc = ensure_ws(ctx, align_up(n * t * 48) + align_up(n * 8) + align_up(n * 32) + align_up(48) +
                               align_up(sizeof(g1_aff)) + align_up(4) + align_up(n)))) return rc;
  carve c{(char*)ctx->cur->ws};
  uint8_t* d_c = c.take<uint8_t>(n * t * 48); uint64_t* d_x = c.take<uint64_t>(n); uint8_t* d_s = c.take<uint8_t>(n * 32);
  uint8_t* d_h48 = c.take<uint8_t>(48); g1_aff* d_h = c.take<g1_aff>(1); uint32_t* d_hf = c.take<uint32_t>(1);
  uint8_t* d_v = c.take<uint8_t>(n);
  hipStream_t st = ctx->cur->stream;
  SSB_HIP(hipMemcpyAsync(d_c, commitments48, n * t * 48, hipMemcpyHostToDevice, st));
  SSB_HIP(hipMemcpyAsync(d_x, ids, n * 8, hipMemcpyHostToDevice, st));
  SSB_HIP(hipMemcpyAsync(d_s, shares32, n * 32, hipMemcpyHostToDevice, st));
  SSB_HIP(hipMemcpyAsync(d_h48, h48, 48, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_decode_pk, dim3(1), dim3(64), 0, st, 1, (const uint8_t*)d_h48, d_h, d_hf);
  { timed tm(ctx, "k_feldman_share"); launch::feldman_share(st, (int)n, (int)t, d_c, d_x, d_s, d_h, d_hf, d_v); }
  SSB_HIP(hipGetLastError());
  SSB_HIP(hipMemcpyAsync(verdicts, d_v, n, hipMemcpyDeviceToHost, st));
  SSB_SYNC_WAIT(st);
  return SSB_OK;
}

int ssb_dleq_verify_batch(ssb_ctx* ctx, size_t n, const uint8_t* points48, const uint8_t* c32, const uint8_t* r32,
                          uint8_t* verdicts) {
  if (!ctx) return SSB_EINVAL;
  SSB_SYNC_LOCK(ctx);
  if (n == 0) return SSB_OK;
  if (!points48 || !c32 || !r32 || !verdicts || n > (size_t)INT32_MAX) { ctx->err = "null pointer or n too large"; return SSB_EINVAL; }
  SSB_HIP(hipSetDevice(ctx->device));
  pick_idle_slot(ctx);
  int rc;
  if ((rc = ensure_ws(ctx, align_up(n * 192) + 2 * align_up(n * 32) + align_up(n)))) return rc;
  carve c{(char*)ctx->cur->ws};
  uint8_t* d_p = c.take<uint8_t>(n * 192); uint8_t* d_c = c.take<uint8_t>(n * 32); uint8_t* d_r = c.take<uint8_t>(n * 32);
  uint8_t* d_v = c.take<uint8_t>(n);
  hipStream_t st = ctx->cur->stream;
  SSB_HIP(hipMemcpyAsync(d_p, points48, n * 192, hipMemcpyHostToDevice, st));
  SSB_HIP(hipMemcpyAsync(d_c, c32, n * 32, hipMemcpyHostToDevice, st));
  SSB_HIP(hipMemcpyAsync(d_r, r32, n * 32, hipMemcpyHostToDevice, st));
  { timed tm(ctx, "k_dleq_verify"); launch::dleq_verify(st, (int)n, d_p, d_c, d_r, d_v); }
  SSB_HIP(hipGetLastError());
  SSB_HIP(hipMemcpyAsync(verdicts, d_v, n, hipMemcpyDeviceToHost, st));
  SSB_SYNC_WAIT(st);
  return SSB_OK;
}

int ssb_decode_wire_sigs_dev(ssb_ctx* ctx, size_t n, const uint8_t* wire, size_t stride, uint8_t* out96, int32_t* status,
                             void* stream) {
  if (!ctx) return SSB_EINVAL;
  SSB_LOCK(ctx);
  if (n == 0) return SSB_OK;
  if (!wire || !out96 || !status || stride < launch::WIRE_SIG_BYTES || n > (size_t)INT32_MAX) {
    ctx->err = "null pointer, stride < 202 or n too large"; return SSB_EINVAL;
  }
  SSB_HIP(hipSetDevice(ctx->device));
  launch::wire_sig((hipStream_t)stream, (int)n, wire, stride, out96, status);
  SSB_HIP(hipGetLastError());
  return SSB_OK;
}

int ssb_decode_wire_sigs(ssb_ctx* ctx, size_t n, const uint8_t* wire, size_t stride, uint8_t* out96, int32_t* status) {
  if (!ctx) return SSB_EINVAL;
  SSB_SYNC_LOCK(ctx);
  if (n == 0) return SSB_OK;
  if (!wire || !out96 || !status || stride < launch::WIRE_SIG_BYTES || n > (size_t)INT32_MAX) {
    ctx->err = "null pointer, stride < 202 or n too large"; return SSB_EINVAL;
  }
  SSB_HIP(hipSetDevice(ctx->device));
  pick_idle_slot(ctx);
  int rc;
  if ((rc = ensure_ws(ctx, align_up(n * stride) + align_up(n * 96) + align_up(n * 4)))) return rc;
  carve c{(char*)ctx->cur->ws};
  uint8_t* d_in = c.take<uint8_t>(n * stride); uint8_t* d_out = c.take<uint8_t>(n * 96); int32_t* d_st = c.take<int32_t>(n);
  hipStream_t st = ctx->cur->stream;
  SSB_HIP(hipMemcpyAsync(d_in, wire, n * stride, hipMemcpyHostToDevice, st));
  { timed t(ctx, "k_wire_sig"); launch::wire_sig(st, (int)n, d_in, stride, d_out, d_st); }
  SSB_HIP(hipGetLastError());
  SSB_HIP(hipMemcpyAsync(out96, d_out, n * 96, hipMemcpyDeviceToHost, st));
  SSB_HIP(hipMemcpyAsync(status, d_st, n * 4, hipMemcpyDeviceToHost, st));
  SSB_SYNC_WAIT(st);
  return SSB_OK;
}

int ssb_verify_batch(ssb_ctx* ctx, size_t n, const uint8_t* pk48, const uint8_t* sig96, const uint32_t* root_idx,
                     size_t n_roots, const uint8_t* roots32, const uint8_t* dst, size_t dst_len, uint64_t rlc_seed,
                     uint8_t* verdicts) {
  if (!ctx) return SSB_EINVAL;
  SSB_SYNC_LOCK(ctx);
  if (n == 0) return SSB_OK;
  if (!pk48 || !sig96 || !root_idx || !roots32 || !verdicts || n_roots == 0) { ctx->err = "null pointer or no roots"; return SSB_EINVAL; }
  for (size_t i = 0; i < n; ++i) if (root_idx[i] >= n_roots) { ctx->err = "root_idx out of range"; return SSB_EINVAL; }
  SSB_HIP(hipSetDevice(ctx->device));
  pick_idle_slot(ctx);
  dst_arg d; int rc = fill_dst(ctx, d, dst, dst_len); if (rc) return rc;
  size_t io = align_up(n * 48) + align_up(n * 96) + align_up(n * 4) + align_up(n_roots * 32) + align_up(n);
  if ((rc = ensure_io(ctx, io))) return rc;
  if ((rc = ensure_ws(ctx, verify_ws_bytes(n, n_roots), true))) return rc;
  carve ci{(char*)ctx->io};
  uint8_t* d_pk = ci.take<uint8_t>(n * 48); uint8_t* d_sig = ci.take<uint8_t>(n * 96);
  uint32_t* d_root = ci.take<uint32_t>(n); uint8_t* d_roots = ci.take<uint8_t>(n_roots * 32); uint8_t* d_v = ci.take<uint8_t>(n);
  hipStream_t st = ctx->cur->stream;
  SSB_HIP(hipMemcpyAsync(d_pk, pk48, n * 48, hipMemcpyHostToDevice, st));
  SSB_HIP(hipMemcpyAsync(d_sig, sig96, n * 96, hipMemcpyHostToDevice, st));
  SSB_HIP(hipMemcpyAsync(d_root, root_idx, n * 4, hipMemcpyHostToDevice, st));
  SSB_HIP(hipMemcpyAsync(d_roots, roots32, n_roots * 32, hipMemcpyHostToDevice, st));
  carve c{(char*)ctx->cur->ws};
  verify_ws w = carve_verify(c, n, n_roots);
  if ((rc = run_verify(ctx, w, n, n_roots, d_sig, d_pk, nullptr, d_root, d_roots, d, rlc_seed, d_v, [] {}, st))) return rc;
  SSB_HIP(hipMemcpyAsync(verdicts, d_v, n, hipMemcpyDeviceToHost, st));
  SSB_SYNC_WAIT(st);
  return SSB_OK;
}

}  // extern "C"

namespace {
// the body of the _dev entry points: public keys compressed (pk48) or from the cache (pk_index)
// (wire != nullptr: the shares arrive as wire records -- record i at wire + i * stride -- and sig96 is
// unused; wire_status receives each record's status, and a share whose record does not deserialize
// is absent from its job, as the reference drops it: select_job)
int aggregate_dev(ssb_ctx* ctx, size_t n_jobs, size_t n_shares, const uint32_t* share_off,
                  const uint32_t* t, const uint8_t* sig96, const uint8_t* pk48, const uint32_t* pk_index,
                  const uint64_t* ids, const uint32_t* job_root, size_t n_roots, const uint8_t* roots32,
                  const uint8_t* dst, size_t dst_len, uint64_t rlc_seed, uint8_t* out_sig96,
                  int32_t* out_status, uint64_t* out_err, uint8_t* share_verdicts, void* stream,
                  const uint8_t* wire = nullptr, size_t stride = 0, int32_t* wire_status = nullptr) {
  if (!ctx) return SSB_EINVAL;
  SSB_LOCK(ctx);
  if (n_jobs == 0) return SSB_OK;
  if (!share_off || !t || !job_root || !roots32 || !out_sig96 || !out_status || !out_err || n_roots == 0 ||
      (n_shares && (!(sig96 || wire) || !(pk48 || pk_index) || !ids))) { ctx->err = "null pointer or no roots"; return SSB_EINVAL; }
  if (wire && (!wire_status || stride < launch::WIRE_SIG_BYTES || n_shares > (size_t)INT32_MAX)) {
    ctx->err = "wire records: null status, stride < 202 or too many shares"; return SSB_EINVAL;
  }
  if (pk_index && !ctx->pkc_aff) { ctx->err = "no public-key cache (ssb_pk_cache_set)"; return SSB_EINVAL; }
  SSB_HIP(hipSetDevice(ctx->device));
  pick_slot(ctx, stream);           // pipeline slot: batches on different slots overlap
  dst_arg d; int rc = fill_dst(ctx, d, dst, dst_len); if (rc) return rc;
  const size_t n = n_shares;
  size_t need = verify_ws_bytes(n, n_roots) + align_up(n * 4) * 3 + align_up(n) + align_up(n * sizeof(fr)) +
                align_up(4 * n * sizeof(g2_jac)) + align_up(n_jobs * 4) + align_up(n_jobs * RC_TAB_BYTES) + align_up(n_jobs * sizeof(g2_jac)) + align_up(32 * n_jobs) +
                (wire ? align_up(n * 96) : 0);
  if ((rc = ensure_ws(ctx, need, true))) return rc;
  hipStream_t user = (hipStream_t)stream;
  const bool on_slot = post_on_slot(ctx->cur);
  hipStream_t st = ctx->cur->stream, sc = ctx->spec, tl = on_slot ? st : slot_tail(ctx);
  // order the engine's streams after the caller's stream, and the caller's stream after them
  if (user != st) {
    SSB_HIP(hipEventRecord(ctx->cur->ev_user, user));
    SSB_HIP(hipStreamWaitEvent(st, ctx->cur->ev_user, 0));
  }
  carve c{(char*)ctx->cur->ws};
  const bool pre = g1_pre_path(ctx, pk_index, n, n_roots);
  verify_ws w = carve_verify(c, n, n_roots, pre);
  uint32_t* share_job = c.take<uint32_t>(n);
  uint32_t* share_root = c.take<uint32_t>(n);
  uint32_t* sel = c.take<uint32_t>(n);
  uint8_t* verdict = share_verdicts ? share_verdicts : c.take<uint8_t>(n);
  fr* lam = c.take<fr>(n);
  g2_jac* term = c.take<g2_jac>(4 * n);     // k_combine_terms_gls: four digit terms per share
  uint32_t* fast = c.take<uint32_t>(n_jobs);
  // jobs whose lambda_i are ratios of small integers (registry ids; ids 1..n with a share skipped):
  // [M^-1](sum c_i sig_i) on one lane per job, lane-uniform windows (k_combine_ratio); SSB_NO_RATIO=1
  // sends them to the general combine (lambda_i by unit_lagrange_fast, four GLS lanes per share)
  const uint32_t ratio = getenv("SSB_NO_RATIO") ? 0u : 1u;
  uint8_t* rtab = c.take<uint8_t>(n_jobs * RC_TAB_BYTES);
  g2_jac* rT = c.take<g2_jac>(n_jobs);
  uint64_t* rk = c.take<uint64_t>(4 * n_jobs);
  // the ratio combine rides in the terms launch (phase T: its blocks past nbt) and the sum launch (phase K)
  const unsigned nbt = nblk(4 * n, 64), nbr = nblk(n_jobs, 64);
  const ratio_args ra{ids, rtab, ratio ? rT : nullptr, rk, nbt, w.sig_aff, getenv("SSB_RATIO_LANE_EXACT") ? 1u : 0u};
  // k_combine_sum: one thread per job, then the lane-group blocks of the fast-3 jobs (ratio jobs a wave
  // holds too few of: RATIO_LANE_PER_WAVE blocks per wave, those without a job leave at once)
  const unsigned nbsum = nblk(n_jobs, 64) * (ratio ? 1u + RATIO_LANE_PER_WAVE : 1u);
  if (wire && n) {   // the records' hex -> the 96-byte compressed form, first on the slot's stream
    uint8_t* sig_ws = c.take<uint8_t>(n * 96);
    { timed tm(ctx, "k_wire_sig", st); launch::wire_sig(st, (int)n, wire, stride, sig_ws, wire_status, 0); }
    sig96 = sig_ws;
  }
  // share -> (job, root): in the decode launch on the fused path, else a launch of its own
  const bool fmap = fused_sort_path(ctx->cur, n, n_roots, pre);
  const job_map jm{(int)n_jobs, (uint32_t)n, share_off, t, job_root, share_job, share_root};
  if (n && !fmap)
    hipLaunchKernelGGL(k_share_map, dim3(nblk(n, 64)), dim3(64), 0, st, (int)n_jobs, (uint32_t)n, share_off, t, job_root, share_job, share_root);
  // speculative combine (selection from the decode flags) on its own stream, beside the pairing chain
  auto spec = [&] {
    hipStreamWaitEvent(sc, ctx->cur->ev_dec, 0);
    { timed tm(ctx, "k_combine_fast", sc);   // select + small-integer combine + Lagrange, one launch
      hipLaunchKernelGGL(k_select_combine, dim3(nblk(n_jobs, 64)), dim3(64), 0, sc, (int)n_jobs, (uint32_t)n, share_off, t, ids,
                         (const uint8_t*)nullptr, w.flags, (const uint32_t*)nullptr, sel, out_status, out_err, w.sig_aff, fast,
                         out_sig96, lam, ratio, wire ? wire_status : (int32_t*)nullptr); }
    if (nbt + (ratio ? nbr : 0)) { timed tm(ctx, "k_combine_terms", sc); hipLaunchKernelGGL(k_combine_terms_gls, dim3(nbt + (ratio ? nbr : 0)), dim3(64), 0, sc, (int)n, (uint32_t)n_jobs, share_job, share_off, t, out_status, sel, lam, w.sig_aff, (const uint32_t*)nullptr, (const uint32_t*)fast, term, ra); }
    { timed tm(ctx, "k_combine_sum", sc); hipLaunchKernelGGL(k_combine_sum, dim3(nbsum), dim3(64), 0, sc, (int)n_jobs, share_off, t, out_status, term, (const uint32_t*)nullptr, (const uint32_t*)fast, out_sig96, 4, (const uint32_t*)sel, ra); }
    hipEventRecord(ctx->cur->ev_comb, sc);
  };
  // one-stream slots: the speculative pass rides in the window-sum launch (msm_both), no stream
  const spec_jobs sj{(int)n_jobs, (uint32_t)n, share_off, t, ids, w.flags, sel, out_status, out_err, w.sig_aff, fast,
                     out_sig96, lam, ratio, wire ? wire_status : nullptr};
  bool spec_in_window = false;
  if ((rc = run_verify(ctx, w, n, n_roots, sig96, pk48, pk_index, share_root, roots32, d, rlc_seed, verdict,
                       [&] { if (!on_slot) spec(); }, tl, on_slot ? &sj : nullptr, &spec_in_window, fmap ? &jm : nullptr)))
    return rc;
  if (!n && !on_slot) spec();
  // exact path: only if the RLC batch failed (every kernel a no-op when w.ok == 1, the speculative
  // combine stands) -- on the shared tail stream, or on the slot's stream; one-stream slots whose
  // window launch could not carry the speculative pass run the exact pass always
  const uint32_t* gate = (on_slot && !spec_in_window) ? nullptr : (const uint32_t*)w.ok;
  if (!on_slot) SSB_HIP(hipStreamWaitEvent(tl, ctx->cur->ev_comb, 0));
  st = tl;
  if (on_slot) {
    timed tm(ctx, "k_combine_fast", st);
    hipLaunchKernelGGL(k_select_combine, dim3(nblk(n_jobs, 64)), dim3(64), 0, st, (int)n_jobs, (uint32_t)n, share_off, t, ids,
                       (const uint8_t*)verdict, w.flags, gate, sel, out_status, out_err, w.sig_aff, fast, out_sig96, lam, ratio,
                       wire ? wire_status : (int32_t*)nullptr);
  } else {
    hipLaunchKernelGGL(k_select_combine, dim3(nblk(n_jobs, 64)), dim3(64), 0, st, (int)n_jobs, (uint32_t)n, share_off, t, ids,
                       (const uint8_t*)verdict, w.flags, gate, sel, out_status, out_err, w.sig_aff, fast, out_sig96, lam, ratio,
                       wire ? wire_status : (int32_t*)nullptr);
  }
  // (after a speculative pass in the window launch the general combine of the jobs the small-
  // integer path did not finish still follows here, on whichever selection stands)
  const uint32_t* gate2 = spec_in_window ? nullptr : gate;
  if (nbt + (ratio ? nbr : 0)) {
    timed tm(ctx, "k_combine_terms", st);
    hipLaunchKernelGGL(k_combine_terms_gls, dim3(nbt + (ratio ? nbr : 0)), dim3(64), 0, st, (int)n, (uint32_t)n_jobs, share_job, share_off, t, out_status, sel, lam, w.sig_aff, gate2, (const uint32_t*)fast, term, ra);
  }
  { timed tm(ctx, "k_combine_sum", st);
    hipLaunchKernelGGL(k_combine_sum, dim3(nbsum), dim3(64), 0, st, (int)n_jobs, share_off, t, out_status, term, gate2, (const uint32_t*)fast, out_sig96, 4, (const uint32_t*)sel, ra); }
  SSB_HIP(hipGetLastError());
  SSB_HIP(hipEventRecord(ctx->cur->ev_out, st));
  ctx->cur->out_pending = true;
  ctx->cur->out_on_stream = st == ctx->cur->stream;
  if (user != st) SSB_HIP(hipStreamWaitEvent(user, ctx->cur->ev_out, 0));
  return SSB_OK;
}

// the body of ssb_verify_batch_dev / _cached_dev: verdicts of (pk, sig, root) triples, device
// pointers, enqueued on the next pipeline slot (a-2; a-8 with the validators' master keys)
int verify_dev(ssb_ctx* ctx, size_t n, const uint8_t* pk48, const uint32_t* pk_index, const uint8_t* sig96,
               const uint32_t* root_idx, size_t n_roots, const uint8_t* roots32, const uint8_t* dst, size_t dst_len,
               uint64_t rlc_seed, uint8_t* verdicts, void* stream) {
  if (!ctx) return SSB_EINVAL;
  SSB_LOCK(ctx);
  if (n == 0) return SSB_OK;
  if (!(pk48 || pk_index) || !sig96 || !root_idx || !roots32 || !verdicts || n_roots == 0) {
    ctx->err = "null pointer or no roots"; return SSB_EINVAL;
  }
  if (pk_index && !ctx->pkc_aff) { ctx->err = "no public-key cache (ssb_pk_cache_set)"; return SSB_EINVAL; }
  SSB_HIP(hipSetDevice(ctx->device));
  pick_slot(ctx, stream);
  dst_arg d; int rc = fill_dst(ctx, d, dst, dst_len); if (rc) return rc;
  if ((rc = ensure_ws(ctx, verify_ws_bytes(n, n_roots), true))) return rc;
  hipStream_t user = (hipStream_t)stream, st = ctx->cur->stream;
  if (user != st) {
    SSB_HIP(hipEventRecord(ctx->cur->ev_user, user));
    SSB_HIP(hipStreamWaitEvent(st, ctx->cur->ev_user, 0));
  }
  carve c{(char*)ctx->cur->ws};
  verify_ws w = carve_verify(c, n, n_roots, g1_pre_path(ctx, pk_index, n, n_roots));
  // root indices >= n_roots: those shares are skipped by the sums and get verdict 0
  hipStream_t tl = post_on_slot(ctx->cur) ? st : slot_tail(ctx);
  if ((rc = run_verify(ctx, w, n, n_roots, sig96, pk48, pk_index, root_idx, roots32, d, rlc_seed, verdicts, [] {},
                       tl))) return rc;
  SSB_HIP(hipEventRecord(ctx->cur->ev_out, tl));
  ctx->cur->out_pending = true;
  ctx->cur->out_on_stream = tl == ctx->cur->stream;
  if (user != tl) SSB_HIP(hipStreamWaitEvent(user, ctx->cur->ev_out, 0));
  return SSB_OK;
}

}  // namespace

extern "C" {

int ssb_threshold_aggregate_batch_dev(ssb_ctx* ctx, size_t n_jobs, size_t n_shares, const uint32_t* share_off,
                                      const uint32_t* t, const uint8_t* sig96, const uint8_t* pk48, const uint64_t* ids,
                                      const uint32_t* job_root, size_t n_roots, const uint8_t* roots32,
                                      const uint8_t* dst, size_t dst_len, uint64_t rlc_seed, uint8_t* out_sig96,
                                      int32_t* out_status, uint64_t* out_err, uint8_t* share_verdicts, void* stream) {
  if (ctx && n_shares && !pk48) { ctx->err = "null pk48"; return SSB_EINVAL; }
  return aggregate_dev(ctx, n_jobs, n_shares, share_off, t, sig96, pk48, nullptr, ids, job_root, n_roots, roots32, dst,
                       dst_len, rlc_seed, out_sig96, out_status, out_err, share_verdicts, stream);
}

int ssb_threshold_aggregate_batch_cached_dev(ssb_ctx* ctx, size_t n_jobs, size_t n_shares, const uint32_t* share_off,
                                             const uint32_t* t, const uint8_t* sig96, const uint32_t* pk_index,
                                             const uint64_t* ids, const uint32_t* job_root, size_t n_roots,
                                             const uint8_t* roots32, const uint8_t* dst, size_t dst_len, uint64_t rlc_seed,
                                             uint8_t* out_sig96, int32_t* out_status, uint64_t* out_err,
                                             uint8_t* share_verdicts, void* stream) {
  if (ctx && n_shares && !pk_index) { ctx->err = "null pk_index"; return SSB_EINVAL; }
  return aggregate_dev(ctx, n_jobs, n_shares, share_off, t, sig96, nullptr, pk_index, ids, job_root, n_roots, roots32, dst,
                       dst_len, rlc_seed, out_sig96, out_status, out_err, share_verdicts, stream);
}
int ssb_threshold_aggregate_batch_wire_cached_dev(ssb_ctx* ctx, size_t n_jobs, size_t n_shares, const uint32_t* share_off,
                                                  const uint32_t* t, const uint8_t* wire, size_t stride,
                                                  const uint32_t* pk_index, const uint64_t* ids, const uint32_t* job_root,
                                                  size_t n_roots, const uint8_t* roots32, const uint8_t* dst, size_t dst_len,
                                                  uint64_t rlc_seed, uint8_t* out_sig96, int32_t* out_status,
                                                  uint64_t* out_err, uint8_t* share_verdicts, int32_t* share_wire_status,
                                                  void* stream) {
  if (ctx && n_shares && (!pk_index || !wire)) { ctx->err = "null pk_index or wire"; return SSB_EINVAL; }
  return aggregate_dev(ctx, n_jobs, n_shares, share_off, t, nullptr, nullptr, pk_index, ids, job_root, n_roots, roots32, dst,
                       dst_len, rlc_seed, out_sig96, out_status, out_err, share_verdicts, stream, wire, stride,
                       share_wire_status);
}

int ssb_verify_batch_dev(ssb_ctx* ctx, size_t n, const uint8_t* pk48, const uint8_t* sig96, const uint32_t* root_idx,
                         size_t n_roots, const uint8_t* roots32, const uint8_t* dst, size_t dst_len, uint64_t rlc_seed,
                         uint8_t* verdicts, void* stream) {
  if (ctx && n && !pk48) { ctx->err = "null pk48"; return SSB_EINVAL; }
  return verify_dev(ctx, n, pk48, nullptr, sig96, root_idx, n_roots, roots32, dst, dst_len, rlc_seed, verdicts, stream);
}

int ssb_verify_batch_cached_dev(ssb_ctx* ctx, size_t n, const uint32_t* pk_index, const uint8_t* sig96,
                                const uint32_t* root_idx, size_t n_roots, const uint8_t* roots32, const uint8_t* dst,
                                size_t dst_len, uint64_t rlc_seed, uint8_t* verdicts, void* stream) {
  if (ctx && n && !pk_index) { ctx->err = "null pk_index"; return SSB_EINVAL; }
  return verify_dev(ctx, n, nullptr, pk_index, sig96, root_idx, n_roots, roots32, dst, dst_len, rlc_seed, verdicts, stream);
}

}  // extern "C"
namespace {
void pkc_free(ssb_ctx* ctx) {
  if (ctx->pkc_aff) { hipFree(ctx->pkc_aff); ctx->pkc_aff = nullptr; }
  if (ctx->pkc_flags) { hipFree(ctx->pkc_flags); ctx->pkc_flags = nullptr; }
  if (ctx->pkc_pow) { hipFree(ctx->pkc_pow); ctx->pkc_pow = nullptr; }
  ctx->pkc_n = ctx->pkc_cap = 0;
}
// every slot and context stream idle: in-flight batches read the table through the pointers they
// were launched with
int pkc_quiesce(ssb_ctx* ctx) {
  for (int i = 0; i < ctx->nslots; ++i) sync_slot(ctx, ctx->sl[i]);
  for (hipStream_t x : {ctx->spec, ctx->tail}) if (x) SSB_HIP(hipStreamSynchronize(x));
  return SSB_OK;
}
// Key registration (pkc_reserve / pkc_fill) runs on a stream created for the call and destroyed
// after it: registering a key waits for that key's decode only, not for the batches queued on a
// slot, and holds no hardware queue between registrations.  (A context-lifetime stream
// took one of the process's GPU_MAX_HW_QUEUES from the slots: two slots then shared a queue and
// the pipelined rate fell from 12.8 M to 9.6 M partial sigs/s, round 5.)
struct reg_stream {
  hipStream_t s = nullptr;
  int open(ssb_ctx* ctx) {
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess) return SSB_OK;
    s = nullptr;
    ctx->err = "hipStreamCreate (key registration) failed";
    return SSB_EHIP;
  }
  ~reg_stream() { if (s) { hipStreamSynchronize(s); hipStreamDestroy(s); } }
};
// room for `need` rows; growing (capacity doubles) moves the live rows to the new arrays after every
// in-flight batch has finished -- registration-time work, amortised over the doublings
int pkc_reserve(ssb_ctx* ctx, size_t need) {
  if (need <= ctx->pkc_cap) return SSB_OK;
  if (int rc = pkc_quiesce(ctx)) return rc;
  const size_t cap = std::max<size_t>({need, 2 * ctx->pkc_cap, (size_t)1024});
  g1_aff* a = nullptr; uint32_t* f = nullptr; g1_aff* p = nullptr;
  if (hipMalloc(&a, cap * sizeof(g1_aff)) != hipSuccess || hipMalloc(&f, cap * 4) != hipSuccess) {
    if (a) hipFree(a);
    (void)hipGetLastError();
    ctx->err = "hipMalloc public-key cache failed";
    return SSB_ENOMEM;
  }
  // the precomputed bases of the batch path's merged G1 MSM (plan_msm g1_pre): registration-time
  // work, like the decompression; without them (allocation failed) batches use the windowed G1 MSM
  if (hipMalloc(&p, cap * PKPOW_W * sizeof(g1_aff)) != hipSuccess) { p = nullptr; (void)hipGetLastError(); }
  const size_t n = ctx->pkc_n;
  if (n) {
    reg_stream rs;
    if (int rc = rs.open(ctx)) return rc;
    hipStream_t st = rs.s;
    SSB_HIP(hipMemcpyAsync(a, ctx->pkc_aff, n * sizeof(g1_aff), hipMemcpyDeviceToDevice, st));
    SSB_HIP(hipMemcpyAsync(f, ctx->pkc_flags, n * 4, hipMemcpyDeviceToDevice, st));
    if (p && ctx->pkc_pow)
      SSB_HIP(hipMemcpyAsync(p, ctx->pkc_pow, n * PKPOW_W * sizeof(g1_aff), hipMemcpyDeviceToDevice, st));
    else if (p)
      hipLaunchKernelGGL(k_pk_pow, dim3(nblk(n, 64)), dim3(64), 0, st, (int)n, (const g1_aff*)a, (const uint32_t*)f, p);
    SSB_HIP(hipGetLastError());
    SSB_HIP(hipStreamSynchronize(st));
  }
  const size_t live = ctx->pkc_n;
  pkc_free(ctx);
  ctx->pkc_aff = a; ctx->pkc_flags = f; ctx->pkc_pow = p; ctx->pkc_n = live; ctx->pkc_cap = cap;
  return SSB_OK;
}
// decode n compressed keys into rows [row, row + n) (+ their precomputed bases); synchronous.  Runs
// on a registration stream (reg_stream): rows below `row` -- the only ones an in-flight batch can index -- are untouched.
int pkc_fill(ssb_ctx* ctx, size_t row, size_t n, const uint8_t* pk48) {
  if (!n) return SSB_OK;
  if (n * 48 > ctx->pkc_stage_bytes) {
    if (ctx->pkc_stage) { hipFree(ctx->pkc_stage); ctx->pkc_stage = nullptr; ctx->pkc_stage_bytes = 0; }
    const size_t want = std::max<size_t>(n * 48, 48 * 1024);
    if (hipMalloc(&ctx->pkc_stage, want) != hipSuccess) { ctx->pkc_stage = nullptr; ctx->err = "hipMalloc key staging failed"; return SSB_ENOMEM; }
    ctx->pkc_stage_bytes = want;
  }
  reg_stream rs;
  if (int rc = rs.open(ctx)) return rc;
  hipStream_t st = rs.s;
  SSB_HIP(hipMemcpyAsync(ctx->pkc_stage, pk48, n * 48, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_decode_pk, dim3(nblk(n, 64)), dim3(64), 0, st, (int)n, (const uint8_t*)ctx->pkc_stage,
                     ctx->pkc_aff + row, ctx->pkc_flags + row);
  if (ctx->pkc_pow)
    hipLaunchKernelGGL(k_pk_pow, dim3(nblk(n, 64)), dim3(64), 0, st, (int)n, (const g1_aff*)(ctx->pkc_aff + row),
                       (const uint32_t*)(ctx->pkc_flags + row), ctx->pkc_pow + row * PKPOW_W);
  SSB_HIP(hipGetLastError());
  SSB_HIP(hipStreamSynchronize(st));
  return SSB_OK;
}
}  // namespace
extern "C" {

int ssb_pk_cache_set(ssb_ctx* ctx, size_t n, const uint8_t* pk48) {
  if (!ctx) return SSB_EINVAL;
  SSB_LOCK(ctx);
  if (n && !pk48) { ctx->err = "null pk48"; return SSB_EINVAL; }
  if (n > (size_t)UINT32_MAX) { ctx->err = "too many keys"; return SSB_EINVAL; }
  SSB_HIP(hipSetDevice(ctx->device));
  if (int rc = pkc_quiesce(ctx)) return rc;
  pkc_free(ctx);
  ctx->pkc_map.clear();
  ctx->pkc_set_keys.clear();
  ctx->pkc_map_valid = true;
  if (!n) return SSB_OK;
  int rc;
  if ((rc = pkc_reserve(ctx, n))) return rc;
  if ((rc = pkc_fill(ctx, 0, n, pk48))) return rc;
  ctx->pkc_n = n;
  // the key -> row index for a later ssb_pk_cache_add is built from these bytes on first use
  ctx->pkc_set_keys.assign(pk48, pk48 + n * 48);
  ctx->pkc_map_valid = false;
  return SSB_OK;
}

int ssb_pk_cache_add(ssb_ctx* ctx, size_t n, const uint8_t* pk48, uint32_t* out_index) {
  if (!ctx) return SSB_EINVAL;
  SSB_LOCK(ctx);
  if (n == 0) return SSB_OK;
  if (!pk48 || !out_index) { ctx->err = "null pointer"; return SSB_EINVAL; }
  SSB_HIP(hipSetDevice(ctx->device));
  if (!ctx->pkc_map_valid) {   // after a _set: index its rows (first occurrence of each key)
    ctx->pkc_map.clear();
    ctx->pkc_map.reserve(ctx->pkc_set_keys.size() / 48);
    for (size_t r = 0; r * 48 < ctx->pkc_set_keys.size(); ++r)
      ctx->pkc_map.emplace(std::string((const char*)ctx->pkc_set_keys.data() + 48 * r, 48), (uint32_t)r);
    std::vector<uint8_t>().swap(ctx->pkc_set_keys);
    ctx->pkc_map_valid = true;
  }
  // new distinct keys of this call, in order
  std::vector<uint8_t> fresh;
  std::unordered_map<std::string, uint32_t> local;
  size_t next = ctx->pkc_n;
  for (size_t i = 0; i < n; ++i) {
    std::string k((const char*)pk48 + 48 * i, 48);
    auto it = ctx->pkc_map.find(k);
    if (it != ctx->pkc_map.end()) { out_index[i] = it->second; continue; }
    auto jt = local.find(k);
    if (jt != local.end()) { out_index[i] = jt->second; continue; }
    if (next >= (size_t)UINT32_MAX) { ctx->err = "key table full"; return SSB_EINVAL; }
    local.emplace(std::move(k), (uint32_t)next);
    out_index[i] = (uint32_t)next++;
    fresh.insert(fresh.end(), pk48 + 48 * i, pk48 + 48 * i + 48);
  }
  const size_t nf = fresh.size() / 48;
  if (!nf) return SSB_OK;
  int rc;
  if ((rc = pkc_reserve(ctx, ctx->pkc_n + nf))) return rc;
  if ((rc = pkc_fill(ctx, ctx->pkc_n, nf, fresh.data()))) return rc;
  ctx->pkc_n += nf;
  for (auto& kv : local) ctx->pkc_map.emplace(kv.first, kv.second);
  return SSB_OK;
}

}  // extern "C"
namespace {
// the body of the two submit entry points: public keys compressed (pk48) or cache indices (pk_index)
int submit_impl(ssb_ctx* ctx, size_t n_jobs, const uint32_t* share_off, const uint32_t* t, const uint8_t* sig96,
                const uint8_t* pk48, const uint32_t* pk_index, const uint64_t* ids, const uint32_t* job_root, size_t n_roots,
                const uint8_t* roots32, const uint8_t* dst, size_t dst_len, uint64_t rlc_seed, uint8_t* out_sig96,
                int32_t* out_status, uint64_t* out_err, uint8_t* share_verdicts, uint64_t* ticket) {
  if (!ctx) return SSB_EINVAL;
  SSB_LOCK(ctx);
  if (ticket) *ticket = 0;
  if (n_jobs == 0) return SSB_OK;
  if (!share_off || !t || !job_root || !roots32 || !out_sig96 || !out_status || !out_err || n_roots == 0 || !ticket) {
    ctx->err = "null pointer or no roots"; return SSB_EINVAL;
  }
  if (share_off[0] != 0) { ctx->err = "share_off[0] must be 0"; return SSB_EINVAL; }
  for (size_t j = 0; j < n_jobs; ++j) {
    if (share_off[j + 1] < share_off[j]) { ctx->err = "share_off not monotone"; return SSB_EINVAL; }
    if (t[j] == 0 || t[j] > SSB_MAX_T) { ctx->err = "t out of range [1, SSB_MAX_T]"; return SSB_EINVAL; }
    if (job_root[j] >= n_roots) { ctx->err = "job_root out of range"; return SSB_EINVAL; }
  }
  const size_t n = share_off[n_jobs];
  if (n && (!sig96 || !(pk48 || pk_index) || !ids)) { ctx->err = "null share arrays"; return SSB_EINVAL; }
  if (pk_index && !ctx->pkc_aff) { ctx->err = "no public-key cache (ssb_pk_cache_set)"; return SSB_EINVAL; }
  SSB_HIP(hipSetDevice(ctx->device));
  // the next slot round robin; its previous host batch is delivered before its staging is reused
  const int k = ctx->next;
  ssb_slot& S = ctx->sl[k];
  SSB_HIP(deliver_host(ctx, S));
  size_t o = 0;
  auto at = [&](size_t bytes) { const size_t r = o; o += align_up(bytes); return r; };
  const size_t i_sig = at(n * 96), i_pk = at(pk_index ? n * 4 : n * 48), i_ids = at(n * 8), i_off = at((n_jobs + 1) * 4), i_t = at(n_jobs * 4),
               i_jr = at(n_jobs * 4), i_roots = at(n_roots * 32), o_sig = at(n_jobs * 96), o_st = at(n_jobs * 4),
               o_err = at(n_jobs * 16), o_ver = at(n ? n : 1);
  if (o > S.hst_bytes) {
    if (S.hst) { hipHostFree(S.hst); S.hst = nullptr; S.hst_bytes = 0; }
    const size_t want = o + o / 4;
    if (hipHostMalloc((void**)&S.hst, want, hipHostMallocMapped | hipHostMallocNonCoherent) != hipSuccess) {
      S.hst = nullptr; ctx->err = "hipHostMalloc staging failed"; return SSB_ENOMEM;
    }
    S.hst_bytes = want;
  }
  uint8_t* h = S.hst;
  if (n) {
    memcpy(h + i_sig, sig96, n * 96);
    if (pk_index) memcpy(h + i_pk, pk_index, n * 4); else memcpy(h + i_pk, pk48, n * 48);
    memcpy(h + i_ids, ids, n * 8);
  }
  memcpy(h + i_off, share_off, (n_jobs + 1) * 4);
  memcpy(h + i_t, t, n_jobs * 4);
  memcpy(h + i_jr, job_root, n_jobs * 4);
  memcpy(h + i_roots, roots32, n_roots * 32);
  uint8_t* d = nullptr;
  SSB_HIP(hipHostGetDevicePointer((void**)&d, S.hst, 0));
  int rc = aggregate_dev(ctx, n_jobs, n, (const uint32_t*)(d + i_off), (const uint32_t*)(d + i_t), d + i_sig,
                         pk_index ? nullptr : d + i_pk, pk_index ? (const uint32_t*)(d + i_pk) : nullptr,
                         (const uint64_t*)(d + i_ids), (const uint32_t*)(d + i_jr), n_roots, d + i_roots, dst, dst_len,
                         rlc_seed, d + o_sig, (int32_t*)(d + o_st), (uint64_t*)(d + o_err), d + o_ver, (void*)S.stream);
  if (rc) return rc;
  SSB_HIP(hipEventRecord(S.ev_host, S.stream));
  S.ho.sig = out_sig96; S.ho.st = out_status; S.ho.err = out_err; S.ho.ver = share_verdicts;
  S.ho.nj = n_jobs; S.ho.n = n; S.ho.o_sig = o_sig; S.ho.o_st = o_st; S.ho.o_err = o_err; S.ho.o_ver = o_ver;
  S.host_ticket = (++ctx->ticket_gen << 8) | (uint64_t)k;
  *ticket = S.host_ticket;
  return SSB_OK;
}
}  // namespace
extern "C" {

int ssb_threshold_aggregate_batch_submit(ssb_ctx* ctx, size_t n_jobs, const uint32_t* share_off, const uint32_t* t,
                                         const uint8_t* sig96, const uint8_t* pk48, const uint64_t* ids,
                                         const uint32_t* job_root, size_t n_roots, const uint8_t* roots32,
                                         const uint8_t* dst, size_t dst_len, uint64_t rlc_seed, uint8_t* out_sig96,
                                         int32_t* out_status, uint64_t* out_err, uint8_t* share_verdicts,
                                         uint64_t* ticket) {
  if (ctx && n_jobs && share_off && share_off[n_jobs] && !pk48) { ctx->err = "null pk48"; return SSB_EINVAL; }
  return submit_impl(ctx, n_jobs, share_off, t, sig96, pk48, nullptr, ids, job_root, n_roots, roots32, dst, dst_len,
                     rlc_seed, out_sig96, out_status, out_err, share_verdicts, ticket);
}

int ssb_threshold_aggregate_batch_cached_submit(ssb_ctx* ctx, size_t n_jobs, const uint32_t* share_off, const uint32_t* t,
                                                const uint8_t* sig96, const uint32_t* pk_index, const uint64_t* ids,
                                                const uint32_t* job_root, size_t n_roots, const uint8_t* roots32,
                                                const uint8_t* dst, size_t dst_len, uint64_t rlc_seed, uint8_t* out_sig96,
                                                int32_t* out_status, uint64_t* out_err, uint8_t* share_verdicts,
                                                uint64_t* ticket) {
  if (ctx && n_jobs && share_off && share_off[n_jobs] && !pk_index) { ctx->err = "null pk_index"; return SSB_EINVAL; }
  return submit_impl(ctx, n_jobs, share_off, t, sig96, nullptr, pk_index, ids, job_root, n_roots, roots32, dst, dst_len,
                     rlc_seed, out_sig96, out_status, out_err, share_verdicts, ticket);
}

int ssb_batch_wait(ssb_ctx* ctx, uint64_t ticket) {
  if (!ctx) return SSB_EINVAL;
  std::unique_lock<std::recursive_mutex> ssb_lock_(ctx->mu);
  if (ticket == 0) return SSB_OK;
  const int k = (int)(ticket & 0xff);
  // only generations never issued are unknown; any issued ticket that no live slot holds was
  // delivered (its slot reused, waited before, or removed by ssb_set_pipeline_depth /
  // ssb_set_slot_streams / ssb_pk_cache_*, which deliver first) -- unless its delivery failed
  if ((ticket >> 8) == 0 || (ticket >> 8) > ctx->ticket_gen || k >= SSB_MAX_SLOTS) { ctx->err = "unknown ticket"; return SSB_EINVAL; }
  // the batch is waited for OUTSIDE the context lock (polled: each query under the lock, so the slot
  // and its event stay valid), so other threads' batches -- a collector's windows -- launch meanwhile
  // (ADVICE r5); the delivery itself (host copies) runs under the lock
  for (;;) {
    if (!(k < ctx->nslots && ctx->sl[k].host_ticket == ticket)) break;   // delivered by another call
    if (hipEventQuery(ctx->sl[k].ev_host) != hipErrorNotReady) { (void)deliver_host(ctx, ctx->sl[k]); break; }
    ssb_lock_.unlock();
    std::this_thread::sleep_for(std::chrono::microseconds(20));
    ssb_lock_.lock();
  }
  (void)hipGetLastError();   // (hipErrorNotReady of the queries)
  auto it = ctx->failed_tickets.find(ticket);
  if (it != ctx->failed_tickets.end()) {
    ctx->failed_tickets.erase(it);
    ctx->err = "the batch did not complete (HIP error); its statuses are SSB_DVF_ENGINE_ERROR";
    return SSB_EHIP;
  }
  return SSB_OK;
}

int ssb_threshold_aggregate_batch(ssb_ctx* ctx, size_t n_jobs, const uint32_t* share_off, const uint32_t* t,
                                  const uint8_t* sig96, const uint8_t* pk48, const uint64_t* ids, const uint32_t* job_root,
                                  size_t n_roots, const uint8_t* roots32, const uint8_t* dst, size_t dst_len,
                                  uint64_t rlc_seed, uint8_t* out_sig96, int32_t* out_status, uint64_t* out_err,
                                  uint8_t* share_verdicts) {
  uint64_t ticket = 0;
  const int rc = ssb_threshold_aggregate_batch_submit(ctx, n_jobs, share_off, t, sig96, pk48, ids, job_root, n_roots, roots32,
                                                      dst, dst_len, rlc_seed, out_sig96, out_status, out_err, share_verdicts,
                                                      &ticket);
  if (rc) return rc;
  return ssb_batch_wait(ctx, ticket);
}

int ssb_unsafe_aggregate_batch(ssb_ctx* ctx, size_t n_jobs, const uint32_t* share_off, const uint8_t* sig96,
                               const uint64_t* ids, uint8_t* out_sig96, int32_t* out_status) {
  if (!ctx) return SSB_EINVAL;
  SSB_SYNC_LOCK(ctx);
  if (n_jobs == 0) return SSB_OK;
  if (!share_off || !out_sig96 || !out_status) { ctx->err = "null pointer"; return SSB_EINVAL; }
  if (share_off[0] != 0) { ctx->err = "share_off[0] must be 0"; return SSB_EINVAL; }
  for (size_t j = 0; j < n_jobs; ++j) {
    if (share_off[j + 1] < share_off[j]) { ctx->err = "share_off not monotone"; return SSB_EINVAL; }
    if (share_off[j + 1] - share_off[j] > SSB_MAX_T) { ctx->err = "more than SSB_MAX_T shares in a job"; return SSB_EINVAL; }
  }
  const size_t n = share_off[n_jobs];
  if (n && (!sig96 || !ids)) { ctx->err = "null share arrays"; return SSB_EINVAL; }
  SSB_HIP(hipSetDevice(ctx->device));
  pick_idle_slot(ctx);
  int rc;
  size_t io = align_up(n * 96) + align_up(n * 8) + align_up((n_jobs + 1) * 4) + align_up(n_jobs * 96) + align_up(n_jobs * 4);
  if ((rc = ensure_io(ctx, io))) return rc;
  size_t need = align_up(n * sizeof(g2_aff)) + align_up(n * 4) * 3 + align_up(n_jobs * 4) + align_up(n_jobs * 16) +
                align_up(n * sizeof(fr)) + align_up(n * sizeof(g2_jac));
  if ((rc = ensure_ws(ctx, need))) return rc;
  carve ci{(char*)ctx->io};
  uint8_t* d_sig = ci.take<uint8_t>(n * 96); uint64_t* d_ids = ci.take<uint64_t>(n); uint32_t* d_off = ci.take<uint32_t>(n_jobs + 1);
  uint8_t* d_out = ci.take<uint8_t>(n_jobs * 96); int32_t* d_st = ci.take<int32_t>(n_jobs);
  carve c{(char*)ctx->cur->ws};
  g2_aff* sig_aff = c.take<g2_aff>(n); uint32_t* flags = c.take<uint32_t>(n); uint32_t* share_job = c.take<uint32_t>(n);
  uint32_t* sel = c.take<uint32_t>(n); uint32_t* tt = c.take<uint32_t>(n_jobs); uint64_t* err = c.take<uint64_t>(n_jobs * 2);
  fr* lam = c.take<fr>(n); g2_jac* term = c.take<g2_jac>(n);
  hipStream_t st = ctx->cur->stream;
  if (n) {
    SSB_HIP(hipMemcpyAsync(d_sig, sig96, n * 96, hipMemcpyHostToDevice, st));
    SSB_HIP(hipMemcpyAsync(d_ids, ids, n * 8, hipMemcpyHostToDevice, st));
  }
  SSB_HIP(hipMemcpyAsync(d_off, share_off, (n_jobs + 1) * 4, hipMemcpyHostToDevice, st));
  if (n) hipLaunchKernelGGL(k_share_map, dim3(nblk(n, 64)), dim3(64), 0, st, (int)n_jobs, (uint32_t)n, d_off, (const uint32_t*)nullptr, (const uint32_t*)nullptr, share_job, (uint32_t*)nullptr);
  if (n) hipLaunchKernelGGL(k_decode, dim3(nblk(n, 64)), dim3(64), 0, st, (int)n, d_sig, (const uint8_t*)nullptr, 0, sig_aff, (g1_aff*)nullptr, flags);
  hipLaunchKernelGGL(k_select_all, dim3(nblk(n_jobs, 64)), dim3(64), 0, st, (int)n_jobs, d_off, flags, sel, tt, d_st, err);
  // unsafe_aggregate does not subgroup-check its inputs (blst.rs:77-84): always the exact 255-bit path
  hipLaunchKernelGGL(k_lagrange, dim3(nblk(n_jobs, 64)), dim3(64), 0, st, (int)n_jobs, d_off, tt, d_ids, sel, d_st, (const uint32_t*)nullptr, (const uint32_t*)nullptr, lam);
  if (n) hipLaunchKernelGGL(k_combine_terms, dim3(nblk(n, 64)), dim3(64), 0, st, (int)n, (uint32_t)n_jobs, share_job, d_off, tt, d_st, sel, lam, sig_aff, (const uint32_t*)nullptr, (const uint32_t*)nullptr, term);
  hipLaunchKernelGGL(k_combine_sum, dim3(nblk(n_jobs, 64)), dim3(64), 0, st, (int)n_jobs, d_off, tt, d_st, term, (const uint32_t*)nullptr, (const uint32_t*)nullptr, d_out, 1, (const uint32_t*)nullptr, ratio_args{nullptr, nullptr, nullptr, nullptr, 0u, nullptr, 0u});
  SSB_HIP(hipGetLastError());
  SSB_HIP(hipMemcpyAsync(out_sig96, d_out, n_jobs * 96, hipMemcpyDeviceToHost, st));
  SSB_HIP(hipMemcpyAsync(out_status, d_st, n_jobs * 4, hipMemcpyDeviceToHost, st));
  SSB_SYNC_WAIT(st);
  return SSB_OK;
}

int ssb_sign_batch(ssb_ctx* ctx, size_t n, const uint8_t* sk32le, const uint32_t* root_idx, size_t n_roots,
                   const uint8_t* roots32, const uint8_t* dst, size_t dst_len, uint8_t* out_sig96) {
  if (!ctx) return SSB_EINVAL;
  SSB_SYNC_LOCK(ctx);
  if (n == 0) return SSB_OK;
  if (!sk32le || !root_idx || !roots32 || !out_sig96 || n_roots == 0) { ctx->err = "null pointer or no roots"; return SSB_EINVAL; }
  for (size_t i = 0; i < n; ++i) if (root_idx[i] >= n_roots) { ctx->err = "root_idx out of range"; return SSB_EINVAL; }
  SSB_HIP(hipSetDevice(ctx->device));
  pick_idle_slot(ctx);
  dst_arg d; int rc = fill_dst(ctx, d, dst, dst_len); if (rc) return rc;
  size_t need = align_up(n * 32) + align_up(n * 4) + align_up(n_roots * 32) + align_up(n_roots * sizeof(g2_aff)) + align_up(n * 96) +
                align_up(launch::hash_ws_bytes(n_roots));
  if ((rc = ensure_ws(ctx, need))) return rc;
  carve c{(char*)ctx->cur->ws};
  uint8_t* d_sk = c.take<uint8_t>(n * 32); uint32_t* d_ri = c.take<uint32_t>(n); uint8_t* d_roots = c.take<uint8_t>(n_roots * 32);
  g2_aff* d_h = c.take<g2_aff>(n_roots); uint8_t* d_out = c.take<uint8_t>(n * 96);
  char* hws = c.take<char>(launch::hash_ws_bytes(n_roots));
  hipStream_t st = ctx->cur->stream;
  SSB_HIP(hipMemcpyAsync(d_sk, sk32le, n * 32, hipMemcpyHostToDevice, st));
  SSB_HIP(hipMemcpyAsync(d_ri, root_idx, n * 4, hipMemcpyHostToDevice, st));
  SSB_HIP(hipMemcpyAsync(d_roots, roots32, n_roots * 32, hipMemcpyHostToDevice, st));
  launch::hash_to_g2(st, (int)n_roots, d_roots, d, d_h, hws);
  { timed tm(ctx, "k_sign"); hipLaunchKernelGGL(k_sign, dim3(nblk(n, 64)), dim3(64), 0, st, (int)n, d_sk, d_ri, d_h, d_out); }
  SSB_HIP(hipGetLastError());
  SSB_HIP(hipMemcpyAsync(out_sig96, d_out, n * 96, hipMemcpyDeviceToHost, st));
  SSB_SYNC_WAIT(st);
  return SSB_OK;
}

int ssb_sk_to_pk_batch(ssb_ctx* ctx, size_t n, const uint8_t* sk32le, uint8_t* out_pk48) {
  if (!ctx) return SSB_EINVAL;
  SSB_SYNC_LOCK(ctx);
  if (n == 0) return SSB_OK;
  if (!sk32le || !out_pk48) { ctx->err = "null pointer"; return SSB_EINVAL; }
  SSB_HIP(hipSetDevice(ctx->device));
  pick_idle_slot(ctx);
  int rc;
  size_t need = align_up(n * 32) + align_up(n * 48);
  if ((rc = ensure_ws(ctx, need))) return rc;
  carve c{(char*)ctx->cur->ws};
  uint8_t* d_sk = c.take<uint8_t>(n * 32); uint8_t* d_out = c.take<uint8_t>(n * 48);
  hipStream_t st = ctx->cur->stream;
  SSB_HIP(hipMemcpyAsync(d_sk, sk32le, n * 32, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_sk_to_pk, dim3(nblk(n, 64)), dim3(64), 0, st, (int)n, d_sk, d_out);
  SSB_HIP(hipGetLastError());
  SSB_HIP(hipMemcpyAsync(out_pk48, d_out, n * 48, hipMemcpyDeviceToHost, st));
  SSB_SYNC_WAIT(st);
  return SSB_OK;
}

int ssb_pk_validate_batch(ssb_ctx* ctx, size_t n, const uint8_t* pk48, uint8_t* out_valid, uint8_t* out_pk48) {
  if (!ctx) return SSB_EINVAL;
  SSB_SYNC_LOCK(ctx);
  if (n == 0) return SSB_OK;
  if (!pk48 || !out_valid || !out_pk48 || n > (size_t)INT32_MAX) { ctx->err = "null pointer or n too large"; return SSB_EINVAL; }
  SSB_HIP(hipSetDevice(ctx->device));
  pick_idle_slot(ctx);
  int rc;
  if ((rc = ensure_ws(ctx, 2 * align_up(n * 48) + align_up(n)))) return rc;
  carve c{(char*)ctx->cur->ws};
  uint8_t* d_in = c.take<uint8_t>(n * 48); uint8_t* d_out = c.take<uint8_t>(n * 48); uint8_t* d_v = c.take<uint8_t>(n);
  hipStream_t st = ctx->cur->stream;
  SSB_HIP(hipMemcpyAsync(d_in, pk48, n * 48, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_pk_validate, dim3(nblk(n, 64)), dim3(64), 0, st, (int)n, (const uint8_t*)d_in, d_v, d_out);
  SSB_HIP(hipGetLastError());
  SSB_HIP(hipMemcpyAsync(out_valid, d_v, n, hipMemcpyDeviceToHost, st));
  SSB_HIP(hipMemcpyAsync(out_pk48, d_out, n * 48, hipMemcpyDeviceToHost, st));
  SSB_SYNC_WAIT(st);
  return SSB_OK;
}

int ssb_lagrange_coeffs(ssb_ctx* ctx, size_t t, const uint64_t* ids, uint8_t* out32) {
  if (!ctx) return SSB_EINVAL;
  SSB_SYNC_LOCK(ctx);
  if (t == 0) return SSB_OK;
  if (!ids || !out32 || t > SSB_MAX_T) { ctx->err = "bad arguments"; return SSB_EINVAL; }
  SSB_HIP(hipSetDevice(ctx->device));
  pick_idle_slot(ctx);
  int rc;
  size_t need = align_up(8 * 4) + align_up(t * 8) + align_up(t * 4) + align_up(4) + align_up(t * sizeof(fr));
  if ((rc = ensure_ws(ctx, need))) return rc;
  carve c{(char*)ctx->cur->ws};
  uint32_t* d_off = c.take<uint32_t>(2); uint64_t* d_ids = c.take<uint64_t>(t); uint32_t* d_sel = c.take<uint32_t>(t);
  uint32_t* d_t = c.take<uint32_t>(1); int32_t* d_st = c.take<int32_t>(1); fr* d_lam = c.take<fr>(t);
  std::vector<uint32_t> sel(t); for (size_t i = 0; i < t; ++i) sel[i] = (uint32_t)i;
  uint32_t off[2] = {0, (uint32_t)t}; uint32_t tt = (uint32_t)t; int32_t st0 = 0;
  hipStream_t st = ctx->cur->stream;
  SSB_HIP(hipMemcpyAsync(d_off, off, 8, hipMemcpyHostToDevice, st));
  SSB_HIP(hipMemcpyAsync(d_ids, ids, t * 8, hipMemcpyHostToDevice, st));
  SSB_HIP(hipMemcpyAsync(d_sel, sel.data(), t * 4, hipMemcpyHostToDevice, st));
  SSB_HIP(hipMemcpyAsync(d_t, &tt, 4, hipMemcpyHostToDevice, st));
  SSB_HIP(hipMemcpyAsync(d_st, &st0, 4, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_lagrange, dim3(1), dim3(64), 0, st, 1, d_off, d_t, d_ids, d_sel, d_st, (const uint32_t*)nullptr, (const uint32_t*)nullptr, d_lam);
  SSB_HIP(hipGetLastError());
  std::vector<fr> lam(t);
  SSB_HIP(hipMemcpyAsync(lam.data(), d_lam, t * sizeof(fr), hipMemcpyDeviceToHost, st));
  SSB_SYNC_WAIT(st);
  for (size_t i = 0; i < t; ++i)
    for (int k = 0; k < 8; ++k)
      for (int b = 0; b < 4; ++b) out32[32 * i + 4 * k + b] = (uint8_t)(lam[i].l[k] >> (8 * b));
  return SSB_OK;
}

}  // extern "C"
