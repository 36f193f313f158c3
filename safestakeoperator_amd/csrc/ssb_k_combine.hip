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
#include "ssb_lane_ops.h"

namespace ssb {
namespace k {

// ---- fast 3: the ratio combine of a job on one workgroup's eight lane groups ----
// (ratio jobs in a wave holding fewer than RATIO_MIN_JOBS of them; lambda_i = c_i / M)
//   T = sum c_i sig_i       group i (< 8, then i + 8, ..) [c_i] sig_i, signed 4-bit windows (the job's
//                           window count), the groups' terms summed by a tree through LDS;
//   [M^-1] T                the four base-u digits k_q of M^-1 mod r (rc_digits): group q (< 4)
//                           [k_q] (-1)^q psi^q(T), 16 windows, the tree again;
//   affine + compress       lane 0.
// Every product of a point operation is spread over the group's 8 lanes (the G2 lane programs,
// ssb_lane_ops.h), so no lane runs a whole scalar chain.  All groups run the same program (the
// window count is the job's); an inactive group works on a stand-in and its result and checks are
// dropped.  An exceptional addition in an active group (an input at infinity, equal or opposite
// points: degenerate or adversarial shares) sends the job to the exact single-lane combine
// (unit_combine_ratio_w4 in the job's table region) -- as does ra.exact (SSB_RATIO_LANE_EXACT=1).
namespace rl {
using namespace ssb::lane;
constexpr int NG = 8;
constexpr int S0 = G2_ADD_SCRATCH;
static_assert(S0 >= G2_MADD_SCRATCH && S0 >= G2_DBL_SCRATCH && S0 >= G2_PSI_SCRATCH, "program scratch");
// group-relative slots: BASE, the table of odd multiples, ACC, TMP, X (a partner's point), SUM
constexpr int BASE = S0, TAB = BASE + 6, ACC = TAB + 48, TMP = ACC + 6, X = TMP + 6, SUM = X + 6, GS = SUM + 6;
struct lds { lslot s[LP_NCODE_CONST + NG * GS]; uint32_t flg[NG]; };

// dst = sign(d) (|d|) B from the table (d odd)
SSB_INL void pick(grp& g, int d, int dst) {
  const int e = TAB + 6 * (((d < 0 ? -d : d) - 1) >> 1);
  LP_FOR(8) {
    if (role < 6) {
      lv v = lp_get(g.s + e + role);
      if (d < 0 && (role == 2 || role == 3)) lv_neg(v);
      lp_put(g.s + dst + role, v);
    }
  }
  LP_SYNC();
}
// ACC = [m] BASE for an odd m < 2^(4W) (per group; W uniform): table of the odd multiples, regular
// signed windows (sw4_digit, as rc_joint_sum)
SSB_FN void mul_odd(grp& g, uint64_t m, int W, uint32_t& exc) {
  g2_dbl(g, BASE, TMP);
  lg_copy<8>(g, BASE, TAB, 6);
  for (int j = 1; j < 8; ++j) g2_add(g, TAB + 6 * (j - 1), TMP, TAB + 6 * j, exc);
  pick(g, sw4_digit(m, W - 1, W), ACC);
  for (int w = W - 2; w >= 0; --w) {
    g2_dbl(g, ACC, ACC); g2_dbl(g, ACC, ACC); g2_dbl(g, ACC, ACC); g2_dbl(g, ACC, ACC);
    pick(g, sw4_digit(m, w, W), TMP);
    g2_add(g, ACC, TMP, ACC, exc);
  }
}
// ACC = [a] BASE, negated when neg, for a != 0 (even a: [a | 1] BASE - BASE; the subtraction runs in
// every group when any active group needs it, kept where needed)
SSB_FN void mul_signed(grp& g, uint64_t a, bool neg, bool act, int W, uint32_t& exc) {
  uint32_t e = 0;
  mul_odd(g, a | 1ull, W, e);
  const bool even = !(a & 1ull);
  if (__syncthreads_or(even && act ? 1 : 0)) {   // uniform
    LP_FOR(8) {
      if (role < 6) {
        lv v = lp_get(g.s + BASE + role);
        if (role == 2 || role == 3) lv_neg(v);
        lp_put(g.s + TMP + role, v);
      }
    }
    LP_SYNC();
    uint32_t e2 = 0;
    g2_add(g, ACC, TMP, X, e2);
    if (even) {
      e |= e2;
      LP_FOR(8) { if (role < 6) g.s[ACC + role] = g.s[X + role]; }
    }
    LP_SYNC();
  }
  if (neg) {
    LP_FOR(8) { if (role == 2 || role == 3) { lv v = lp_get(g.s + ACC + role); lv_neg(v); lp_put(g.s + ACC + role, v); } }
  }
  LP_SYNC();
  if (act) exc |= e;
}
// slot S of groups 0 .. n-1 summed into group 0's (a tree: round h adds group gi + h into gi)
SSB_FN void tree(grp& g, lfp* groups, int gi, int n, int S, uint32_t& exc) {
  for (int h = 1; h < n; h <<= 1) {
    const bool has = (gi % (2 * h)) == 0 && gi + h < n;
    LP_FOR(8) { if (role < 6) g.s[X + role] = has ? groups[(gi + h) * GS + S + role] : g.s[S + role]; }
    LP_SYNC();
    uint32_t e = 0;
    g2_add(g, S, X, TMP, e);
    if (has) {
      exc |= e;
      LP_FOR(8) { if (role < 6) g.s[S + role] = g.s[TMP + role]; }
    }
    LP_SYNC();
  }
}
}  // namespace rl

// coefficient c_i of job j, its window count W and M (the coefficient array in this frame only)
SSB_FN int64_t ratio_ci(int j, uint32_t i, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                        const uint32_t* __restrict__ sel, const uint64_t* __restrict__ ids, int* W, uint64_t* M) {
  int64_t c[FAST_T];
  ratio_coeffs(j, off, tt, sel, ids, c, M);
  *W = rc_windows(c, tt[j]);
  return c[i < tt[j] ? i : 0u];
}
// the exact single-lane ratio combine of job j, phase T into rT[j] / rk[j] (phase K follows in the
// kernel: the two phases' frames are never on one call chain)
SSB_FN void ratio_lane_exact_T(int j, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                               const uint32_t* __restrict__ sel, const ratio_args& ra) {
  int64_t c[FAST_T];
  uint64_t M;
  ratio_coeffs(j, off, tt, sel, ra.ids, c, &M);
  unit_ratio_T(ra.rT + j, ra.rk + 4 * (size_t)j, ra.sig, sel + off[j], c, tt[j], M, rc_windows(c, tt[j]),
               ra.tabs + (size_t)j * RC_TAB_BYTES);
}
// the fast-3 job of extra block b (wave b % nw, its (b / nw)-th fast-3 job), or nothing; returns the
// job when it must be redone exactly (ratio_lane_exact_T + phase K, called by the kernel: the frames are
// never on one call chain), else -1.  Uniform.
SSB_FN int ratio_lane_job(rl::lds& L, int b, int nw, int n_jobs, const uint32_t* __restrict__ off,
                           const uint32_t* __restrict__ tt, const uint32_t* __restrict__ sel,
                           const uint32_t* __restrict__ fast, uint8_t* __restrict__ out96, const ratio_args& ra) {
  using namespace ssb::lane;
  const int w = b % nw, slot = b / nw, lane_ = threadIdx.x;
  const int jl = 64 * w + lane_;
  uint64_t m = __ballot(jl < n_jobs && fast[jl] == 3u);
  if (__popcll(m) <= slot) return -1;   // uniform
  for (int i = 0; i < slot; ++i) m &= m - 1;
  const int j = 64 * w + __builtin_ctzll(m);
  const uint32_t t = tt[j], b0 = off[j];
  uint32_t exc = 0;
  if (!ra.exact) {
    const int gi = lane_ >> 3;
    lfp* groups = (lfp*)L.s + LP_NCODE_CONST;
    grp g{(lfp*)L.s, groups + gi * rl::GS, 0, 0, 0, (lu32*)&L.flg[gi], lane_ & 7};
    lp_init_consts(g);
    // T
    int W = 1;
    uint64_t M = 1;
    for (uint32_t p = 0; p * rl::NG < t; ++p) {
      const uint32_t i = p * rl::NG + (uint32_t)gi;
      const bool act = i < t;
      const int64_t ci = ratio_ci(j, i, off, tt, sel, ra.ids, &W, &M);   // (W, M: the job's, every lane)
      {
        const g2_aff q = ra.sig[sel[b0 + (act ? i : 0u)]];
        if (g.role < 4) lp_put(g.s + rl::BASE + g.role, lv_in(((const fp*)&q)[g.role]));
        else if (g.role < 6) lp_put(g.s + rl::BASE + g.role, g.role == 4 ? lv_one() : lv_zero());
      }
      __syncthreads();
      rl::mul_signed(g, (uint64_t)(ci < 0 ? -ci : ci), ci < 0, act, W, exc);
      if (p == 0) {
        lg_copy<8>(g, rl::ACC, rl::SUM, 6);
      } else {
        uint32_t e = 0;
        g2_add(g, rl::SUM, rl::ACC, rl::TMP, e);
        if (act) {
          exc |= e;
          if (g.role < 6) g.s[rl::SUM + g.role] = g.s[rl::TMP + g.role];
        }
        __syncthreads();
      }
    }
    rl::tree(g, groups, gi, (int)(t < (uint32_t)rl::NG ? t : (uint32_t)rl::NG), rl::SUM, exc);
    // [M^-1] T: group q's base (-1)^q psi^q(T)
    uint64_t kk[4];
    rc_digits(kk, M);
    const int q = gi & 3;
    if (g.role < 6) g.s[rl::BASE + g.role] = groups[rl::SUM + g.role];
    __syncthreads();
    for (int r = 1; r < 4; ++r) {
      g2_psi(g, rl::BASE, rl::TMP);
      if (q >= r && g.role < 6) g.s[rl::BASE + g.role] = g.s[rl::TMP + g.role];
      __syncthreads();
    }
    if ((q & 1) && (g.role == 2 || g.role == 3)) { lv v = lp_get(g.s + rl::BASE + g.role); lv_neg(v); lp_put(g.s + rl::BASE + g.role, v); }
    __syncthreads();
    rl::mul_signed(g, kk[q], false, gi < 4, 16, exc);
    rl::tree(g, groups, gi, 4, rl::ACC, exc);
  }
  if (ra.exact || __syncthreads_or(exc ? 1 : 0)) return j;
  if (lane_ == 0) {
    g2_jac R;
    for (int k = 0; k < 6; ++k) ((fp*)&R)[k] = slot_out(L.s[LP_NCODE_CONST + rl::ACC + k]);
    g2_aff a;
    jac_to_aff(a, R);
    g2_compress(out96 + 96 * (size_t)j, a);
  }
  return -1;
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
  // (the term written in place: jac_mul_aff stores its result once, at the end -- a local point here
  // would sit in the kernel's frame, under the chain of the ratio jobs' phase T)
  unit_combine_term_gls(term[4 * (size_t)s + q], sig_aff[sel[s]], lam[s].l, q);
}
// stride: terms per share (1: k_combine_terms, 4: k_combine_terms_gls).  Jobs of the ratio combine
// (fast 2; ra.rT != nullptr) run its phase K here: [M^-1] T from rT[j], compressed (unit_ratio_K);
// blocks past the jobs' (RATIO_LANE_PER_WAVE per wave of 64 jobs) run the fast-3 jobs whole
// (ratio_lane_job; ra.sig != nullptr).
__global__ void SSB_LB(64) k_combine_sum(int n_jobs, const uint32_t* __restrict__ off,
                                                    const uint32_t* __restrict__ tt, const int32_t* __restrict__ status,
                                                    const g2_jac* __restrict__ term, const uint32_t* __restrict__ skip_if_ok,
                                                    const uint32_t* __restrict__ fast, uint8_t* __restrict__ out96, int stride,
                                                    const uint32_t* __restrict__ sel, ratio_args ra) {
  const int nbs = (n_jobs + 63) / 64;
  if ((int)blockIdx.x >= nbs) {   // extra blocks: the fast-3 jobs, one workgroup each (uniform)
    if (!fast || !ra.sig || !ra.rT || (skip_if_ok && *skip_if_ok)) return;
    __shared__ rl::lds L;
    const int jx = ratio_lane_job(L, (int)blockIdx.x - nbs, nbs, n_jobs, off, tt, sel, fast, out96, ra);
    if (jx >= 0 && threadIdx.x == 0) {
      ratio_lane_exact_T(jx, off, tt, sel, ra);
      unit_ratio_K(out96 + 96 * (size_t)jx, ra.rT + jx, ra.rk + 4 * (size_t)jx, ra.tabs + (size_t)jx * RC_TAB_BYTES);
    }
    return;
  }
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
