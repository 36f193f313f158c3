// ssb_k_pair.hip -- kernels (gfx950): lane-program Miller loops, Fp12 products and the final exponentiation.
// Launched from ssbls.hip (declarations in ssb_kernels.h); one TU per kernel family so the
// library compiles in parallel.
// lane-program kernels at two waves per SIMD (256 registers, the rest spilled within the queue
// primer's private segment): under load they no longer wait for a whole SIMD's register file
#ifndef SSB_WAVES_PER_EU
#define SSB_WAVES_PER_EU 2
#endif
#include "ssb_kernels.h"
#include "ssb_blocks.h"
#include "ssb_lane_ops.h"

namespace ssb {
namespace k {

// the speculative a-1 scan + combine of job j (candidate flags as verdicts), out of line: its
// temporaries live in its own frame, not in the Miller blocks' (every kernel's private segment sets
// the scratch each slot queue reserves)
SSB_FN void spec_job(int j, const spec_jobs& sj) {
  select_job(j, sj.n_shares, sj.off, sj.tt, sj.ids, (const uint8_t*)nullptr, sj.flags, sj.sel, sj.status, sj.err, sj.wst);
  const uint32_t fj = ratio_by_wave(combine_job(j, sj.off, sj.tt, sj.status, sj.sel, sj.ids, sj.sig_aff, sj.out96, sj.ratio));
  sj.fast[j] = fj;
  if (!fj && sj.status[j] == SSB_DVF_OK) lagrange_job(j, sj.off, sj.tt, sj.ids, sj.sel, sj.lam);
}

// ---- lane-program versions (straight-line programs of gen_lane_progs.py, G = 64) ----
constexpr int ML_S0 = lane::MILLER_ITER_SCRATCH > lane::MILLER_ADDSTEP_SCRATCH ? lane::MILLER_ITER_SCRATCH
                                                                               : lane::MILLER_ADDSTEP_SCRATCH;
constexpr int ML_SLOTS = ML_S0 + 18 + 6;
// one Miller loop per pair (P[p], Q[p]), one workgroup each: the roots' (S_r, H(root r)) and the
// G2 MSM windows' ([2^(c w)](-g1), W_w)
__global__ void SSB_LB(64) k_miller_pairs(int npairs, const g1_aff* __restrict__ Pa,
                                                     const g2_aff* __restrict__ Qa, fp12* __restrict__ f, spec_jobs sj) {
  using namespace ssb::lane;
  __shared__ lslot lds[LP_NCODE_CONST + ML_SLOTS];
  __shared__ uint32_t flg;
  const int p = blockIdx.x, lane_ = threadIdx.x;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST, 0, 0, 0, (lu32*)&flg, lane_};
  if (p >= npairs) {   // the speculative a-1 scan + combine, 64 jobs per block (candidate flags as verdicts)
    const int j = (p - npairs) * 64 + lane_;
    if (j >= sj.n_jobs) return;
    spec_job(j, sj);
    return;
  }
  const g1_aff P = Pa[p];
  const g2_aff Q = Qa[p];
  if (P.inf || Q.inf) {  // e(O, Q) = e(P, O) = 1  (uniform per workgroup)
    if (lane_ == 0) f[p] = fp12_one();
    return;
  }
  lp_init_consts(g);
  const int F = ML_S0, B = F + 18;
  if (lane_ < 4) lp_put(g.s + B + lane_, lv_in(((const fp*)&Q)[lane_]));
  if (lane_ == 4) lp_put(g.s + B + 4, lv_in(P.x));
  if (lane_ == 5) lp_put(g.s + B + 5, lv_in(P.y));
  __syncthreads();
  f12_miller(g, F, B);
  if (lane_ < 12) ((fp*)&f[p])[lane_] = lv_out(lp_get(g.s + F + lane_));
}

// Exact per-share verification e(pk, H(m)) * e(-g1, sig) == 1, run when the RLC batch check
// failed (a no-op otherwise).  A bounded grid of 64-lane workgroups strides over the shares; each
// candidate runs two lane-program Miller loops, one Fp12 product and one final exponentiation out of
// LDS (the single-lane form needs ~9 KB of scratch per lane, which a full-size grid cannot reserve
// on every hardware queue).  The two Miller loops run as one two-pair loop (f12_miller2).
constexpr int fb_max(int a, int b) { return a > b ? a : b; }
constexpr int FB_S0 = fb_max(fb_max(ML_S0, fb_max(lane::MILLER_ITER2_SCRATCH, lane::MILLER_ADDSTEP2_SCRATCH)),
                             lane::FP12_MUL_SCRATCH);
constexpr int FB_SLOTS = FB_S0 + 24 + 12 + 4 + 84;
__global__ void SSB_LB(64) k_fallback_lane(int n, const uint32_t* __restrict__ ok,
                                                      const uint32_t* __restrict__ flags,
                                                      const uint32_t* __restrict__ share_root,
                                                      const g2_aff* __restrict__ H, const g2_aff* __restrict__ sig_aff,
                                                      const g1_aff* __restrict__ pk_aff, uint8_t* __restrict__ verdict) {
  using namespace ssb::lane;
  if (*ok) return;  // uniform: the batch passed
  __shared__ lslot lds[LP_NCODE_CONST + FB_SLOTS];
  __shared__ uint32_t flg;
  const int lane_ = threadIdx.x;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST, 0, 0, 0, (lu32*)&flg, lane_};
  lp_init_consts(g);
  const int F1 = FB_S0, B = F1 + 24, BP = B + 12, TMP = BP + 4;
  for (int s = blockIdx.x; s < n; s += gridDim.x) {
    if (!(flags[s] & FLAG_CANDIDATE)) continue;  // uniform per workgroup; verdict written by k_final_lane
    const g1_aff pk = pk_aff[s];
    const g2_aff h = H[share_root[s]], sg = sig_aff[s];
    const g1_aff ng = g1_neg_generator();
    // e(pk, H(m)) e(-g1, sig) before the final exponentiation (candidates: pk, sig not infinity)
    if (lane_ < 4) { lp_put(g.s + B + lane_, lv_in(((const fp*)&h)[lane_])); lp_put(g.s + B + 6 + lane_, lv_in(((const fp*)&sg)[lane_])); }
    if (lane_ == 4) { lp_put(g.s + B + 4, lv_in(pk.x)); lp_put(g.s + B + 10, lv_in(ng.x)); }
    if (lane_ == 5) { lp_put(g.s + B + 5, lv_in(pk.y)); lp_put(g.s + B + 11, lv_in(ng.y)); }
    __syncthreads();
    f12_miller2(g, F1, B, BP);
    f12_final_exp(g, F1, TMP);
    if (lane_ == 0) {
      fp12 e;
      ld12(e, g.s + F1);
      verdict[s] = fp12_is_one(e) ? 1 : 0;
    }
    __syncthreads();
  }
}

// out[w] = prod of in[8w .. 8w+7]
__global__ void SSB_LB(64) k_fp12_prod8(int n, const fp12* __restrict__ in, fp12* __restrict__ out) {
  using namespace ssb::lane;
  __shared__ lslot lds[LP_NCODE_CONST + FP12_MUL_SCRATCH + 24];
  __shared__ uint32_t flg;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST, 0, 0, 0, (lu32*)&flg, (int)threadIdx.x};
  lp_init_consts(g);
  const int ACC = FP12_MUL_SCRATCH, IN = ACC + 12;
  const int b = blockIdx.x * 8, e = min(n, b + 8);
  if (threadIdx.x < 12) lp_put(g.s + ACC + threadIdx.x, lv_in(((const fp*)&in[b])[threadIdx.x]));
  __syncthreads();
  for (int i = b + 1; i < e; ++i) {
    if (threadIdx.x < 12) lp_put(g.s + IN + threadIdx.x, lv_in(((const fp*)&in[i])[threadIdx.x]));
    __syncthreads();
    f12_mul(g, ACC, IN, ACC);
  }
  if (threadIdx.x < 12) ((fp*)&out[blockIdx.x])[threadIdx.x] = lv_out(lp_get(g.s + ACC + threadIdx.x));
}

// product of the n values, then ONE final exponentiation -> batch verdict
constexpr int FE_S0 = lane::FP12_MUL_SCRATCH;
// (with verdict != nullptr it also writes the verdicts of a passing batch and of the non-candidates
// -- the candidates of a failed batch are left to the exact fallback)
__global__ void SSB_LB(64) k_final_lane(int n, const fp12* __restrict__ in, uint32_t* __restrict__ ok, int nv,
                                        const uint32_t* __restrict__ flags, uint8_t* __restrict__ verdict) {
  using namespace ssb::lane;
  __shared__ lslot lds[LP_NCODE_CONST + FE_S0 + 12 + 12 + 84];
  __shared__ uint32_t flg;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST, 0, 0, 0, (lu32*)&flg, (int)threadIdx.x};
  lp_init_consts(g);
  const int ACC = FE_S0, IN = ACC + 12, TMP = IN + 12;
  if (threadIdx.x < 12) lp_put(g.s + ACC + threadIdx.x, lv_in(((const fp*)&in[0])[threadIdx.x]));
  __syncthreads();
  for (int i = 1; i < n; ++i) {
    if (threadIdx.x < 12) lp_put(g.s + IN + threadIdx.x, lv_in(((const fp*)&in[i])[threadIdx.x]));
    __syncthreads();
    f12_mul(g, ACC, IN, ACC);
  }
  f12_final_exp(g, ACC, TMP);
  if (threadIdx.x == 0) {  // == 1, read slot by slot (an fp12 local would sit in scratch)
    bool one = true;
    for (int k = 0; k < 12; ++k) {
      const fp v = lv_out(lp_get(g.s + ACC + k));
      one = one && (k == 0 ? fp_eq(v, fp_one()) : fp_is_zero(v));
    }
    *ok = one ? 1u : 0u;
    flg = one ? 1u : 0u;
  }
  if (!verdict) return;
  __syncthreads();
  const bool pass = flg != 0;
  for (int s = threadIdx.x; s < nv; s += 64) {
    const bool cand = (flags[s] & FLAG_CANDIDATE) != 0;
    if (pass || !cand) verdict[s] = cand ? 1 : 0;
  }
}

// Miller loops, the product tree and ONE final exponentiation in one launch (the fused one-stream
// path; k_miller_pairs + k_fp12_prod8 x 2 + k_final_lane in the other paths).  Block p computes pair
// p's Miller value; the last block of each group of 8 to finish multiplies that group's values;
// the last group to finish multiplies the group products and runs the final exponentiation -> *ok.
// Completion tickets (tk[0]: groups done, tk[1 + i]: blocks of group i done), no block ever waits:
// a block continues only with work whose inputs are complete, so the grid drains in every
// schedule; the last block zeroes the tickets for the slot's next batch.  Saves three launches and
// their dispatch gaps on the batch's latency-bound tail.  Blocks [npairs, ..) run the speculative
// a-1 scan + combine, as in k_miller_pairs.  (The verdicts of a passing batch are written grid-wide
// by the next launch, k_fb_rlc.)
constexpr int MF_FE = FE_S0 + 12 + 12 + 84;
constexpr int MF_SLOTS = ML_SLOTS > MF_FE ? ML_SLOTS : MF_FE;
__global__ void SSB_LB(64) k_miller_final(int npairs, const g1_aff* __restrict__ Pa, const g2_aff* __restrict__ Qa,
                                          fp12* __restrict__ f, spec_jobs sj, uint32_t* __restrict__ tk,
                                          uint32_t* __restrict__ ok) {
  using namespace ssb::lane;
  __shared__ lslot lds[LP_NCODE_CONST + MF_SLOTS];
  __shared__ uint32_t flg, last;
  SSB_TRACE_T0();
  const int p = blockIdx.x, lane_ = threadIdx.x;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST, 0, 0, 0, (lu32*)&flg, lane_};
  if (p >= npairs) {   // the speculative a-1 scan + combine, 64 jobs per block (candidate flags as verdicts)
    const int j = (p - npairs) * 64 + lane_;
    if (j >= sj.n_jobs) return;
    spec_job(j, sj);
    return;
  }
  lp_init_consts(g);
  {
    const g1_aff P = Pa[p];
    const g2_aff Q = Qa[p];
    if (P.inf || Q.inf) {  // e(O, Q) = e(P, O) = 1  (uniform per workgroup)
      if (lane_ == 0) f[p] = fp12_one();
    } else {
      const int F = ML_S0, B = F + 18;
      if (lane_ < 4) lp_put(g.s + B + lane_, lv_in(((const fp*)&Q)[lane_]));
      if (lane_ == 4) lp_put(g.s + B + 4, lv_in(P.x));
      if (lane_ == 5) lp_put(g.s + B + 5, lv_in(P.y));
      __syncthreads();
      f12_miller(g, F, B);
      if (lane_ < 12) ((fp*)&f[p])[lane_] = lv_out(lp_get(g.s + F + lane_));
    }
  }
  SSB_TRACE(TR_MF_MILLER);
  const int ng = (npairs + 7) / 8, gi = p / 8, gb = gi * 8, ge = min(npairs, gb + 8);
  __threadfence();
  __syncthreads();
  if (lane_ == 0) last = atomicAdd(&tk[1 + gi], 1u) == (uint32_t)(ge - gb - 1) ? 1u : 0u;
  __syncthreads();
  if (!last) return;
  __threadfence();
  const int ACC = FE_S0, IN = ACC + 12, TMP = IN + 12;
  if (lane_ < 12) lp_put(g.s + ACC + lane_, lv_in(((const fp*)&f[gb])[lane_]));
  __syncthreads();
  for (int i = gb + 1; i < ge; ++i) {
    if (lane_ < 12) lp_put(g.s + IN + lane_, lv_in(((const fp*)&f[i])[lane_]));
    __syncthreads();
    f12_mul(g, ACC, IN, ACC);
  }
  if (lane_ < 12) ((fp*)&f[npairs + gi])[lane_] = lv_out(lp_get(g.s + ACC + lane_));
  SSB_TRACE(TR_MF_GROUP);
  __threadfence();
  __syncthreads();
  if (lane_ == 0) last = atomicAdd(&tk[0], 1u) == (uint32_t)(ng - 1) ? 1u : 0u;
  __syncthreads();
  if (!last) return;
  __threadfence();
  if (lane_ < 12) lp_put(g.s + ACC + lane_, lv_in(((const fp*)&f[npairs])[lane_]));
  __syncthreads();
  for (int i = 1; i < ng; ++i) {
    if (lane_ < 12) lp_put(g.s + IN + lane_, lv_in(((const fp*)&f[npairs + i])[lane_]));
    __syncthreads();
    f12_mul(g, ACC, IN, ACC);
  }
  SSB_TRACE(TR_MF_PRODUCT);
  // the product before the final exponentiation, for the exclusion check of a failed batch
  // (k_fb_excl: the batch check without its suspect shares, by bilinearity from this value)
  if (lane_ < 12) ((fp*)&f[npairs + ng])[lane_] = lv_out(lp_get(g.s + ACC + lane_));
  f12_final_exp(g, ACC, TMP);
  if (lane_ == 0) {  // == 1, read slot by slot (an fp12 local would sit in scratch)
    bool one = true;
    for (int k = 0; k < 12; ++k) {
      const fp v = lv_out(lp_get(g.s + ACC + k));
      one = one && (k == 0 ? fp_eq(v, fp_one()) : fp_is_zero(v));
    }
    *ok = one ? 1u : 0u;
  }
  for (int i = lane_; i <= ng; i += 64) tk[i] = 0u;   // every block has passed its tickets
  SSB_TRACE(TR_MF_FINAL);
}

}  // namespace k
}  // namespace ssb

SSB_TRACE_READER(pair)
