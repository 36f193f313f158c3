// ssb_k_combine.hip -- kernels (gfx950): reference scan/selection, Lagrange coefficients, combine.
// Launched from ssbls.hip (declarations in ssb_kernels.h); one TU per kernel family so the
// library compiles in parallel.
#include "ssb_kernels.h"

namespace ssb {
namespace k {

// A job the engine cannot run -- t == 0, t > SSB_MAX_T, share_off[j + 1] < share_off[j] or past the
// batch's n_shares (only the *_dev entry points can pass one: the host wrapper refuses them) --
// gets SSB_DVF_INVALID_JOB and is never selected, so no later kernel indexes its fixed t-arrays or
// its share range.  (k_share_map clamps the ranges the same way.)
SSB_INL bool job_ok(uint32_t b, uint32_t e, uint32_t t, uint32_t n_shares) {
  return t >= 1 && t <= SSB_MAX_T && b <= e && e <= n_shares;
}
SSB_INL void select_job(int j, uint32_t n_shares, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                        const uint64_t* __restrict__ ids, const uint8_t* __restrict__ verdict,
                        const uint32_t* __restrict__ flags, uint32_t* __restrict__ sel, int32_t* __restrict__ status,
                        uint64_t* __restrict__ err) {
  const uint32_t b = off[j], e = off[j + 1], t = tt[j];
  if (!job_ok(b, e, t, n_shares)) { status[j] = SSB_DVF_INVALID_JOB; err[2 * j] = t; err[2 * j + 1] = e - b; return; }
  const uint32_t n = e - b;
  if (n < t) { status[j] = SSB_DVF_INSUFFICIENT_SIGNATURES; err[2 * j] = n; err[2 * j + 1] = t; return; }
  uint32_t cnt = 0;
  for (uint32_t s = b; s < e; ++s) {
    const uint64_t id = ids[s];
    if (id == 0) { status[j] = SSB_DVF_INVALID_OPERATOR_ID; err[2 * j] = 0; err[2 * j + 1] = 0; return; }
    bool dup = false;
    for (uint32_t k = 0; k < cnt; ++k) dup = dup || (ids[sel[b + k]] == id);
    if (dup) continue;
    if (verdict ? (verdict[s] != 0) : ((flags[s] & FLAG_CANDIDATE) != 0)) {
      sel[b + cnt] = s;
      ++cnt;
      if (cnt >= t) break;
    }
  }
  if (cnt < t) { status[j] = SSB_DVF_INSUFFICIENT_VALID_SIGNATURES; err[2 * j] = cnt; err[2 * j + 1] = t; return; }
  status[j] = SSB_DVF_OK; err[2 * j] = 0; err[2 * j + 1] = 0;
}
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
SSB_INL void lagrange_job(int j, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                          const uint64_t* __restrict__ ids, const uint32_t* __restrict__ sel, fr* __restrict__ lam) {
  const uint32_t b = off[j], t = tt[j];
  uint64_t x[SSB_MAX_T];
  for (uint32_t i = 0; i < t; ++i) x[i] = ids[sel[b + i]];
  unit_lagrange(lam + b, x, t);
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
__global__ void SSB_LB(64) k_combine_terms(int n, const uint32_t* __restrict__ share_job,
                                                      const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                                                      const int32_t* __restrict__ status, const uint32_t* __restrict__ sel,
                                                      const fr* __restrict__ lam, const g2_aff* __restrict__ sig_aff,
                                                      const uint32_t* __restrict__ skip_if_ok, const uint32_t* __restrict__ fast,
                                                      g2_jac* __restrict__ term) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  if (skip_if_ok && *skip_if_ok) return;
  const uint32_t j = share_job[s];
  if (fast && fast[j]) return;
  const uint32_t k = (uint32_t)s - off[j];
  if (status[j] != SSB_DVF_OK || k >= tt[j]) return;
  const fr l = lam[s];
  g2_jac r;
  unit_combine_term(r, sig_aff[sel[s]], l.l);  // blst_p2_mult(.., 255 bits)
  term[s] = r;
}
// verified candidates only: four lanes per share, one base-u digit each (unit_combine_term_gls);
// term[4 s + q]
__global__ void SSB_LB(64) k_combine_terms_gls(int n, const uint32_t* __restrict__ share_job,
                                              const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                                              const int32_t* __restrict__ status, const uint32_t* __restrict__ sel,
                                              const fr* __restrict__ lam, const g2_aff* __restrict__ sig_aff,
                                              const uint32_t* __restrict__ skip_if_ok, const uint32_t* __restrict__ fast,
                                              g2_jac* __restrict__ term) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= 4 * n) return;
  if (skip_if_ok && *skip_if_ok) return;
  const int s = g >> 2, q = g & 3;
  const uint32_t j = share_job[s];
  if (fast && fast[j]) return;
  const uint32_t k = (uint32_t)s - off[j];
  if (status[j] != SSB_DVF_OK || k >= tt[j]) return;
  const fr l = lam[s];
  g2_jac r;
  unit_combine_term_gls(r, sig_aff[sel[s]], l.l, q);
  term[4 * (size_t)s + q] = r;
}
// stride: terms per share (1: k_combine_terms, 4: k_combine_terms_gls)
__global__ void SSB_LB(64) k_combine_sum(int n_jobs, const uint32_t* __restrict__ off,
                                                    const uint32_t* __restrict__ tt, const int32_t* __restrict__ status,
                                                    const g2_jac* __restrict__ term, const uint32_t* __restrict__ skip_if_ok,
                                                    const uint32_t* __restrict__ fast, uint8_t* __restrict__ out96, int stride) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_jobs) return;
  if (skip_if_ok && *skip_if_ok) return;
  if (fast && fast[j]) return;
  uint8_t o[96];
  if (status[j] == SSB_DVF_OK) {
    unit_combine_sum(o, term + (size_t)stride * off[j], (uint32_t)stride * tt[j]);  // infinity(t) start (blst.rs:74)
  } else {
    for (int k = 0; k < 96; ++k) o[k] = 0;
  }
  for (int k = 0; k < 96; ++k) out96[96 * (size_t)j + k] = o[k];
}
// Small-integer Lagrange fast path (unit_lagrange_small), for t <= FAST_T (larger thresholds take
// the 255-bit path; the per-lane arrays stay small -- this kernel's private segment sets the
// scratch the runtime reserves on every slot's hardware queue): every selected share is a verified
// (hence order-r) point, so sum c_i sig_i with the integer c_i == lambda_i mod r is the reference's
// combination.  fast[j] = 1 when the job was finished here; the 255-bit path skips those jobs.
constexpr uint32_t FAST_T = 16;
// fast[j] = 1 when the job was finished here
SSB_INL uint32_t combine_fast_job(int j, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                                  const int32_t* __restrict__ status, const uint32_t* __restrict__ sel,
                                  const uint64_t* __restrict__ ids, const g2_aff* __restrict__ sig_aff,
                                  uint8_t* __restrict__ out96) {
  if (status[j] != SSB_DVF_OK || tt[j] > FAST_T) return 0u;
  const uint32_t t = tt[j], b = off[j];
  uint64_t x[FAST_T];
  int64_t c[FAST_T];
  const g2_aff* pts[FAST_T];
  for (uint32_t i = 0; i < t; ++i) { x[i] = ids[sel[b + i]]; pts[i] = &sig_aff[sel[b + i]]; }
  if (!unit_lagrange_small(c, x, t)) return 0u;
  uint8_t o[96];
  unit_combine_small(o, pts, c, t);
  for (int k = 0; k < 96; ++k) out96[96 * (size_t)j + k] = o[k];
  return 1u;
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
  fast[j] = combine_fast_job(j, off, tt, status, sel, ids, sig_aff, out96);
}
// k_select + k_combine_fast + k_lagrange of one job in one thread (one launch instead of three)
__global__ void SSB_LB(64) k_select_combine(int n_jobs, uint32_t n_shares, const uint32_t* __restrict__ off,
                                            const uint32_t* __restrict__ tt, const uint64_t* __restrict__ ids,
                                            const uint8_t* __restrict__ verdict, const uint32_t* __restrict__ flags,
                                            const uint32_t* __restrict__ skip_if_ok, uint32_t* __restrict__ sel,
                                            int32_t* __restrict__ status, uint64_t* __restrict__ err,
                                            const g2_aff* __restrict__ sig_aff, uint32_t* __restrict__ fast,
                                            uint8_t* __restrict__ out96, fr* __restrict__ lam) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_jobs) return;
  if (skip_if_ok && *skip_if_ok) return;
  select_job(j, n_shares, off, tt, ids, verdict, flags, sel, status, err);
  const uint32_t f = combine_fast_job(j, off, tt, status, sel, ids, sig_aff, out96);
  fast[j] = f;
  if (!f && status[j] == SSB_DVF_OK) lagrange_job(j, off, tt, ids, sel, lam);
}

__global__ void k_hold(const uint32_t* flag, uint32_t max_polls) {
  for (uint32_t i = 0; i < max_polls; ++i) {
    if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) break;
    __builtin_amdgcn_s_sleep(127);
  }
}
__global__ void k_copy_u8(int n, const uint8_t* __restrict__ a, uint8_t* __restrict__ b) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i];
}

}  // namespace k
}  // namespace ssb
