// collbench.cpp -- the value_collector driver (bench.py, tests/test_gpu_collector.py): native
// submitter threads feed the library's per-slot collector exactly as SafeStake's per-duty tasks
// would (one ssb_collector_submit per (validator, duty) job, HotstuffOperatorCommittee::sign,
// src/validation/impls/hotstuff.rs:165-166), and the run is timed from the first submit to the
// last job's completion callback.  Benchmark / test infrastructure, not part of libssbls.so.
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "../include/ssbls.h"

namespace {
struct run_state {
  std::atomic<uint64_t> done{0};
};
void on_done(void* user, const ssb_job_result*) {
  static_cast<run_state*>(user)->done.fetch_add(1, std::memory_order_acq_rel);
}
}  // namespace

extern "C" {

/* n_jobs jobs over a workload of V validators x n shares (job k = validator k % V): sig96[V*n*96],
 * rows[V*n] (key-table rows), ids[V*n], roots32 / job_root[V]; res[n_jobs] receives every job's
 * result.  `threads` submitters, job k on thread k % threads (so every window mixes validators).
 * Returns 0 and writes the wall time (first submit -> last completion callback) to *seconds. */
int ssb_collbench_run(ssb_collector* col, int threads, uint64_t n_jobs, uint32_t V, uint32_t n, uint32_t t,
                      const uint8_t* sig96, const uint32_t* rows, const uint64_t* ids, const uint8_t* roots32,
                      const uint32_t* job_root, ssb_job_result* res, double* seconds) {
  if (!col || threads < 1 || !V || !res || !seconds) return SSB_EINVAL;
  run_state rs;
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  std::atomic<int> fail{0};
  std::vector<std::thread> th;
  for (int i = 0; i < threads; ++i)
    th.emplace_back([&, i] {
      ready.fetch_add(1);
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      for (uint64_t k = (uint64_t)i; k < n_jobs; k += (uint64_t)threads) {
        const uint32_t v = (uint32_t)(k % V);
        const size_t s0 = (size_t)v * n;
        if (ssb_collector_submit(col, t, n, sig96 + 96 * s0, rows + s0, ids + s0, roots32 + 32 * (size_t)job_root[v],
                                 &res[k], on_done, &rs) != SSB_OK) {
          fail.fetch_add(1);
          return;
        }
      }
    });
  while (ready.load() < threads) std::this_thread::yield();
  const auto t0 = std::chrono::steady_clock::now();
  go.store(true, std::memory_order_release);
  for (auto& x : th) x.join();
  if (fail.load()) { ssb_collector_flush(col); return SSB_EINVAL; }
  // the tail of the run: the last window closes on its timer (or is full)
  while (rs.done.load(std::memory_order_acquire) < n_jobs) std::this_thread::sleep_for(std::chrono::microseconds(20));
  const auto t1 = std::chrono::steady_clock::now();
  *seconds = std::chrono::duration<double>(t1 - t0).count();
  return SSB_OK;
}

/* The same through the wire-record entry point (a SSB_COLLECTOR_WIRE collector): share s arrives as
 * the bytes a remote operator sends, wire[s * 202 .. + 202) = bincode(bls::Signature) (encoded by the
 * caller before the run), and every job is one ssb_collector_submit_wire -- no CPU deserialization. */
int ssb_collbench_run_wire(ssb_collector* col, int threads, uint64_t n_jobs, uint32_t V, uint32_t n, uint32_t t,
                           const uint8_t* wire, const uint32_t* rows, const uint64_t* ids, const uint8_t* roots32,
                           const uint32_t* job_root, ssb_job_result* res, double* seconds) {
  if (!col || threads < 1 || !V || !res || !seconds || n > 64) return SSB_EINVAL;
  run_state rs;
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  std::atomic<int> fail{0};
  std::vector<std::thread> th;
  for (int i = 0; i < threads; ++i)
    th.emplace_back([&, i] {
      const uint8_t* recs[64];
      size_t lens[64];
      ready.fetch_add(1);
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      for (uint64_t k = (uint64_t)i; k < n_jobs; k += (uint64_t)threads) {
        const uint32_t v = (uint32_t)(k % V);
        const size_t s0 = (size_t)v * n;
        for (uint32_t q = 0; q < n; ++q) { recs[q] = wire + 202 * (s0 + q); lens[q] = 202; }
        if (ssb_collector_submit_wire(col, t, n, recs, lens, rows + s0, ids + s0, roots32 + 32 * (size_t)job_root[v],
                                      &res[k], on_done, &rs) != SSB_OK) {
          fail.fetch_add(1);
          return;
        }
      }
    });
  while (ready.load() < threads) std::this_thread::yield();
  const auto t0 = std::chrono::steady_clock::now();
  go.store(true, std::memory_order_release);
  for (auto& x : th) x.join();
  if (fail.load()) { ssb_collector_flush(col); return SSB_EINVAL; }
  while (rs.done.load(std::memory_order_acquire) < n_jobs) std::this_thread::sleep_for(std::chrono::microseconds(20));
  const auto t1 = std::chrono::steady_clock::now();
  *seconds = std::chrono::duration<double>(t1 - t0).count();
  return SSB_OK;
}

}  // extern "C"
