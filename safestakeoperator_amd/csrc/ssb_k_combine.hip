// ssb_k_combine.hip -- kernels (gfx950): reference scan/selection, Lagrange coefficients, combine.
// Launched from ssbls.hip (declarations in ssb_kernels.h); one TU per kernel family so the
// library compiles in parallel.
// Two waves per SIMD (256 registers, the rest spilled inside the queue primer's segment): the
// general and registry combines' digit chains measured registry C2 2.42 -> 2.93 M partial sigs/s
// against one wave (round 4, gpurun_out/r04cw2*), the all-valid path unchanged within run-to-run noise
#ifndef SSB_WAVES_PER_EU
#define SSB_WAVES_PER_EU 2
#endif
#include "ssb_kernels.h"
#include "ssb_blocks.h"

namespace ssb {
namespace k {

__global__ void k_select(int n_jobs, uint32_t n_shares, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                         const uint64_t* __restrict__ ids, const uint8_t* __restrict__ verdict,
                         const uint32_t* __restrict__ flags, const uint32_t* __restrict__ skip_if_ok,
                         uint32_t* __restrict__ sel, int32_t* __restrict__ status, uint64_t* __restrict__ err) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_jobs) return;
  if (skip_if_ok && *skip_if_ok) return;
  select_job(j, n_shares, off, tt, ids, verdict, flags, sel, status, err);
}
__global__ void k_select_all(int n_jobs, const uint32_t* __restrict__ off, const uint32_t* __restrict__ flags,
                             uint32_t* __restrict__ sel, uint32_t* __restrict__ tt, int32_t* __restrict__ status,
                             uint64_t* __restrict__ err) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_jobs) return;
  const uint32_t b = off[j], e = off[j + 1];
  tt[j] = e - b;
  int32_t st = SSB_DVF_OK;
  for (uint32_t s = b; s < e; ++s) {
    sel[s] = s;
    if (!(flags[s] & DEC_OK)) st = SSB_DVF_BAD_SIGNATURE_ENCODING;
  }
  status[j] = st; err[2 * j] = 0; err[2 * j + 1] = 0;
}
__global__ void k_lagrange(int n_jobs, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                           const uint64_t* __restrict__ ids, const uint32_t* __restrict__ sel,
                           const int32_t* __restrict__ status, const uint32_t* __restrict__ skip_if_ok,
                           const uint32_t* __restrict__ fast, fr* __restrict__ lam) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_jobs || status[j] != SSB_DVF_OK) return;
  if (skip_if_ok && *skip_if_ok) return;
  if (fast && fast[j]) return;
  lagrange_job(j, off, tt, ids, sel, lam);
}
__global__ void SSB_LB(64) k_combine_terms(int n, uint32_t n_jobs, const uint32_t* __restrict__ share_job,
                                                      const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                                                      const int32_t* __restrict__ status, const uint32_t* __restrict__ sel,
                                                      const fr* __restrict__ lam, const g2_aff* __restrict__ sig_aff,
                                                      const uint32_t* __restrict__ skip_if_ok, const uint32_t* __restrict__ fast,
                                                      g2_jac* __restrict__ term) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  if (skip_if_ok && *skip_if_ok) return;
  const uint32_t j = share_job[s];
  if (j >= n_jobs) return;   // outside every well-formed job (k_share_map's sentinel)
  if (fast && fast[j]) return;
  const uint32_t k = (uint32_t)s - off[j];
  if (status[j] != SSB_DVF_OK || k >= tt[j]) return;
  const fr l = lam[s];
  g2_jac r;
  unit_combine_term(r, sig_aff[sel[s]], l.l);  // blst_p2_mult(.., 255 bits)
  term[s] = r;
}
// The general combine's terms and phase T of the ratio combine, in one launch.
// Blocks [0, nbt): verified candidates only, four lanes per share, one base-u digit each
// (unit_combine_term_gls); term[4 s + q].  Jobs combine_job finished (fast 1) or left to the ratio
// combine (fast 2) are skipped.
// Blocks [nbt, ..): one lane per job of the ratio combine (fast 2: lambda_i = c_i / M), phase T --
// T = sum c_i sig_i, lane-uniform joint windows (unit_ratio_T), into rT[j]; tables in the job's
// RC_TAB_BYTES region of `tabs`.  Every lane of the wave takes part in the window count's maximum
// before any returns, so the doubling chain is the wave's.
__global__ void SSB_LB(64) k_combine_terms_gls(int n, uint32_t n_jobs, const uint32_t* __restrict__ share_job,
                                              const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                                              const int32_t* __restrict__ status, const uint32_t* __restrict__ sel,
                                              const fr* __restrict__ lam, const g2_aff* __restrict__ sig_aff,
                                              const uint32_t* __restrict__ skip_if_ok, const uint32_t* __restrict__ fast,
                                              g2_jac* __restrict__ term, ratio_args ra) {
  if (blockIdx.x >= ra.nbt) {
    const int j = (blockIdx.x - ra.nbt) * blockDim.x + threadIdx.x;
    const bool act = (uint32_t)j < n_jobs && !(skip_if_ok && *skip_if_ok) && fast && fast[j] == 2u;
    int64_t c[FAST_T];
    uint64_t M = 1;
    int W = 1;
    if (act) {
      ratio_coeffs(j, off, tt, sel, ra.ids, c, &M);
      W = rc_windows(c, tt[j]);
    }
    for (int o = 32; o >= 1; o >>= 1) { const int x = __shfl_xor(W, o, 64); W = x > W ? x : W; }
    W = __builtin_amdgcn_readfirstlane(W);
    if (!act) return;
    unit_ratio_T(ra.rT + j, ra.rk + 4 * (size_t)j, sig_aff, sel + off[j], c, tt[j], M, W, ra.tabs + (size_t)j * RC_TAB_BYTES);
    return;
  }
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= 4 * n) return;
  if (skip_if_ok && *skip_if_ok) return;
  const int s = g >> 2, q = g & 3;
  const uint32_t j = share_job[s];
  if (j >= n_jobs) return;   // outside every well-formed job (k_share_map's sentinel)
  if (fast && fast[j]) return;
  const uint32_t k = (uint32_t)s - off[j];
  if (status[j] != SSB_DVF_OK || k >= tt[j]) return;
  const fr l = lam[s];
  g2_jac r;
  unit_combine_term_gls(r, sig_aff[sel[s]], l.l, q);
  term[4 * (size_t)s + q] = r;
}
// stride: terms per share (1: k_combine_terms, 4: k_combine_terms_gls).  Jobs of the ratio combine
// (fast 2; ra.rT != nullptr) run its phase K here: [M^-1] T from rT[j], compressed (unit_ratio_K).
__global__ void SSB_LB(64) k_combine_sum(int n_jobs, const uint32_t* __restrict__ off,
                                                    const uint32_t* __restrict__ tt, const int32_t* __restrict__ status,
                                                    const g2_jac* __restrict__ term, const uint32_t* __restrict__ skip_if_ok,
                                                    const uint32_t* __restrict__ fast, uint8_t* __restrict__ out96, int stride,
                                                    const uint32_t* __restrict__ sel, ratio_args ra) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_jobs) return;
  if (skip_if_ok && *skip_if_ok) return;
  if (fast && fast[j] == 2u && ra.rT) {
    unit_ratio_K(out96 + 96 * (size_t)j, ra.rT + j, ra.rk + 4 * (size_t)j, ra.tabs + (size_t)j * RC_TAB_BYTES);
    return;
  }
  if (fast && fast[j]) return;   // finished by combine_job (1)
  uint8_t o[96];
  if (status[j] == SSB_DVF_OK) {
    unit_combine_sum(o, term + (size_t)stride * off[j], (uint32_t)stride * tt[j]);  // infinity(t) start (blst.rs:74)
  } else {
    for (int k = 0; k < 96; ++k) o[k] = 0;
  }
  for (int k = 0; k < 96; ++k) out96[96 * (size_t)j + k] = o[k];
}
__global__ void SSB_LB(64) k_combine_fast(int n_jobs, const uint32_t* __restrict__ off,
                                                     const uint32_t* __restrict__ tt, const int32_t* __restrict__ status,
                                                     const uint32_t* __restrict__ sel, const uint64_t* __restrict__ ids,
                                                     const g2_aff* __restrict__ sig_aff,
                                                     const uint32_t* __restrict__ skip_if_ok, uint32_t* __restrict__ fast,
                                                     uint8_t* __restrict__ out96) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_jobs) return;
  if (skip_if_ok && *skip_if_ok) return;
  fast[j] = combine_job(j, off, tt, status, sel, ids, sig_aff, out96, 0u);
}
// k_select + k_combine_fast + k_lagrange of one job in one thread (one launch instead of three)
__global__ void SSB_LB(64) k_select_combine(int n_jobs, uint32_t n_shares, const uint32_t* __restrict__ off,
                                            const uint32_t* __restrict__ tt, const uint64_t* __restrict__ ids,
                                            const uint8_t* __restrict__ verdict, const uint32_t* __restrict__ flags,
                                            const uint32_t* __restrict__ skip_if_ok, uint32_t* __restrict__ sel,
                                            int32_t* __restrict__ status, uint64_t* __restrict__ err,
                                            const g2_aff* __restrict__ sig_aff, uint32_t* __restrict__ fast,
                                            uint8_t* __restrict__ out96, fr* __restrict__ lam, uint32_t ratio,
                                            int32_t* __restrict__ wst) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_jobs) return;
  if (skip_if_ok && *skip_if_ok) return;
  select_job(j, n_shares, off, tt, ids, verdict, flags, sel, status, err, wst);
  const uint32_t f = ratio_by_wave(combine_job(j, off, tt, status, sel, ids, sig_aff, out96, ratio));
  fast[j] = f;
  if (!f && status[j] == SSB_DVF_OK) lagrange_job(j, off, tt, ids, sel, lam);
}

__global__ void k_hold(const uint32_t* flag, uint32_t max_polls) {
  for (uint32_t i = 0; i < max_polls; ++i) {
    if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) break;
    __builtin_amdgcn_s_sleep(127);
  }
}
// Scratch primer: a private array as large as the largest private segment of the slot kernels
// (runtime-indexed, so it lives in scratch), over a full-device grid.  Run once per new queue,
// one queue at a time (launch::prime_queue): the queue acquires its scratch while the others are
// idle.  Twenty queues acquiring scratch at once on their first batches intermittently failed with
// HSA_STATUS_ERROR_OUT_OF_RESOURCES (about 1 run in 10 at 20 slots); primed one by one, 0 in 14.
constexpr int PRIME_WORDS = 640;   // 2560 B per lane >= k_msm_window2's 2080 B (the largest)
__global__ void SSB_LB(64) k_scratch_prime(uint32_t* __restrict__ out, uint32_t seed) {
  uint32_t buf[PRIME_WORDS];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  for (int i = 0; i < PRIME_WORDS; ++i) buf[(i * 37u + t) % PRIME_WORDS] = (uint32_t)i ^ seed;
  if (seed == 0xffffffffu) out[t & 63u] = buf[(t * 13u) % PRIME_WORDS];   // never taken: keeps buf
}
__global__ void k_copy_u8(int n, const uint8_t* __restrict__ a, uint8_t* __restrict__ b) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i];
}

}  // namespace k

namespace launch {
int prime_queue(hipStream_t st) {
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  hipLaunchKernelGGL(k::k_scratch_prime, dim3((unsigned)(ncu * 32)), dim3(64), 0, st, (uint32_t*)nullptr, 0u);
  if (hipGetLastError() != hipSuccess) return -1;
  return hipStreamSynchronize(st) == hipSuccess ? 0 : -1;
}
}  // namespace launch
}  // namespace ssb
