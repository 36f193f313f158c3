// ssb_blocks.h -- workgroup bodies of the kernels that the one-stream slot path also runs FUSED:
// a fused launch gives each body its own range of blocks (block index and LDS passed explicitly),
// so independent stages of a batch -- the G2 and G1 MSMs, the hash_to_G2 stages beside the
// per-share kernels -- overlap on the device although the slot has a single stream
// (ssb_k_fused.hip).  The stand-alone kernels (ssb_k_msm.hip, ssb_k_hash.hip) wrap the same bodies.
#pragma once
#include <type_traits>
#include "ssb_kernels.h"
#include "ssb_lane_ops.h"

namespace ssb {
namespace k {

SSB_INL bool share_decodable(uint32_t sf, uint32_t pf) {
  return (sf & DEC_OK) && !(sf & DEC_INF) && (pf & DEC_OK) && !(pf & DEC_INF);
}

template <bool SCATTER>
SSB_INL void msm_entries(int i, uint64_t k, uint32_t g, const msm_cfg& c, uint32_t* __restrict__ cnt,
                         uint32_t* __restrict__ ent) {
  const uint64_t mask = (1ull << c.c) - 1ull;
  if (c.merged) {
    // every window of the share's group shares the group's buckets: the windows holding the same
    // digit d go to bucket d with ONE cursor atomic (and consecutive entries), not one per window --
    // 16 windows of 4-bit digits hold ~9.7 distinct digits.  (The sort's HBM writes are mostly
    // these device-scope atomics: ~99 MB per 8 x C2 count pass, against ~26 MB of decoded points.)
    uint32_t done = 0;
    for (uint32_t w = 0; w < c.W; ++w) {
      const uint32_t d = (uint32_t)((k >> (c.c * w)) & mask);
      if (!d || ((done >> d) & 1u)) continue;
      done |= 1u << d;
      uint32_t m = 0;
      for (uint32_t v = w; v < c.W; ++v) m += (uint32_t)((k >> (c.c * v)) & mask) == d ? 1u : 0u;
      const uint32_t key = c.base + (g << c.c) + d;
      if (SCATTER) {
        uint32_t p = atomicAdd(&cnt[key], m);
        for (uint32_t v = w; v < c.W; ++v)
          if ((uint32_t)((k >> (c.c * v)) & mask) == d) ent[p++] = ((uint32_t)i << 4) | v;
      } else {
        atomicAdd(&cnt[key], m);
      }
    }
    return;
  }
  for (uint32_t w = 0; w < c.W; ++w) {
    const uint32_t d = (uint32_t)((k >> (c.c * w)) & mask);
    if (!d) continue;
    // merged: all windows of the group share its buckets; the entry names the window's base
    const uint32_t key = c.merged ? c.base + (g << c.c) + d : c.base + ((g * c.W + w) << c.c) + d;
    const uint32_t e = c.merged ? ((uint32_t)i << 4) | w : (uint32_t)i;
    if (SCATTER) ent[atomicAdd(&cnt[key], 1u)] = e;
    else atomicAdd(&cnt[key], 1u);
  }
}

// one share's entries of both MSMs (the count pass, or with SCATTER the scatter pass of the sort);
// a share whose root index is out of range has none (it cannot enter the batch)
template <bool SCATTER>
SSB_INL void msm_sort_lane_root(int i, uint32_t g, const rlc_key& key, const msm_cfg& c2, const msm_cfg& c1,
                                uint32_t* __restrict__ cnt, uint32_t* __restrict__ ent) {
  if (g >= c1.ngroups) return;
  const uint64_t k = rlc_scalar_odd(key, (uint64_t)i);
  msm_entries<SCATTER>(i, k, 0u, c2, cnt, ent);
  msm_entries<SCATTER>(i, k, g, c1, cnt, ent);
}
template <bool SCATTER>
SSB_INL void msm_sort_lane(int i, const rlc_key& key, const uint32_t* __restrict__ share_root, const msm_cfg& c2,
                           const msm_cfg& c1, uint32_t* __restrict__ cnt, uint32_t* __restrict__ ent) {
  msm_sort_lane_root<SCATTER>(i, share_root[i], key, c2, c1, cnt, ent);
}

// ---- bucket sums: J = 2^lj lanes per bucket, 64/J buckets per workgroup, buckets in `order` ----
// (block bodies take their block index and LDS explicitly, so one launch can run the G2 and the
// G1 side's blocks side by side: k_msm_bucket2 / k_msm_window2 below)
// (pow != nullptr: a merged MSM -- entry = share << 4 | window, point = pow[pidx[share] * PKPOW_W + window],
// the cached key's precomputed base [2^(4 window)] pk)
template <class F>
SSB_INL void msm_bucket_block(uint32_t bid, jac<F>* sh, uint32_t nb, uint32_t base, int lj, const uint32_t* __restrict__ order,
                              const uint32_t* __restrict__ start, const uint32_t* __restrict__ end,
                              const uint32_t* __restrict__ ent, const uint32_t* __restrict__ flags,
                              const aff<F>* __restrict__ pts, jac<F>* __restrict__ bsum,
                              const aff<F>* __restrict__ pow = nullptr, const uint32_t* __restrict__ pidx = nullptr) {
  const int lane = threadIdx.x, J = 1 << lj, j = lane & (J - 1);
  const uint32_t ob = bid * (64u >> lj) + (uint32_t)(lane >> lj);
  const uint32_t key = ob < nb ? order[base + ob] : 0u, b = key - base;
  jac<F> acc;
  jac_set_inf(acc);
  if (ob < nb) {
    // end[key]: the scatter's cursor, start + count after the scatter (the counts themselves are
    // zeroed by the scan for the slot's next batch)
    const uint32_t s = start[key], e = end[key];
    // one point live: with the tree's addition inlined too, the body fits 256 registers and the
    // bucket launch runs two waves per SIMD, which hide each other's latency (round 2: the former
    // software-pipelined loop, two points live, held 256 VGPRs + 165 AGPRs = one wave per SIMD;
    // C2 at 20 steps 11.2 -> 12.1 M partial sigs/s)
    if (pow) {
#if defined(SSB_MSM_R28)
      if constexpr (std::is_same<F, fp>::value) {   // (experiment knob) G1 in the reduced radix
        r28::pt1 a;
        a.inf = true;
        for (uint32_t x = s + j; x < e; x += J) {
          const uint32_t en = ent[x], i = en >> 4;
          if (flags[i] & FLAG_CANDIDATE) r28::pt1_madd(a, pow[(size_t)pidx[i] * PKPOW_W + (en & 15u)]);
        }
        r28::pt1_to_engine(acc, a);
      } else
#endif
      for (uint32_t x = s + j; x < e; x += J) {
        const uint32_t en = ent[x], i = en >> 4;
        if (flags[i] & FLAG_CANDIDATE) jac_madd_at(acc, pow + ((size_t)pidx[i] * PKPOW_W + (en & 15u)));
      }
#if defined(SSB_MSM_R28)
    } else if constexpr (std::is_same<F, fp2>::value) {
      // (experiment knob, SSB_VARIANT_DEFS=-DSSB_MSM_R28) G2 in the reduced radix (ssb_f28.h pt2_madd),
      // the accumulator's X / Y parked in the block's tree LDS while an addition's products run (the
      // tree below starts after every lane's loop).  A/B on one box (gpurun_out/r06k): the bucket
      // launch 2.10 -> 2.05 ms mean, 20 steps 13.9-14.0 -> 14.3-14.4 M, 1,000 steps 17.7 -> 17.3-17.4 M
      // -- the launch is bound by its G1 side and the point loads, not by the G2 products: not default
      r28::pt2 a;
      r28::pt2_set_inf(a);
      r28::keep_t* keep = (r28::keep_t*)(uint32_t*)sh + lane;
      static_assert(64 * sizeof(jac<F>) >= sizeof(uint32_t) * r28::KEEP_WORDS * 64, "keep in the tree's LDS");
      for (uint32_t x = s + j; x < e; x += J) {
        const uint32_t i = ent[x];
        if (flags[i] & FLAG_CANDIDATE) r28::pt2_madd<64>(a, pts[i], keep);
      }
      r28::pt2_to_engine(acc, a);
#endif
    } else {
      for (uint32_t x = s + j; x < e; x += J) {
        const uint32_t i = ent[x];
        if (flags[i] & FLAG_CANDIDATE) jac_madd_at(acc, pts + i);
      }
    }
  }
  __syncthreads();   // (every lane's loop, and its parked words, are done before the tree's LDS use)
  for (int h = J >> 1; h >= 1; h >>= 1) {
    sh[lane] = acc;
    __syncthreads();
    if (j < h) { jac<F> o = sh[lane + h]; jac_add_inl(acc, acc, o); }
    __syncthreads();
  }
  if (j == 0 && ob < nb) bsum[b] = acc;
}
// ---- window sums  sum_d d * B_d  (one workgroup per (group, window)) ----
// G1: out_jac[gw] (Jacobian, for the Horner combine).  G2: the window is affine pair gw of the
// multi-pairing: out_q[gw] = W_gw, out_p[gw] = [2^(c gw)](-g1) from negg1_pow.
// (redo != nullptr: the lane-group kernel below already summed the window into lane_sum, and
// only the windows it flagged -- an exceptional addition, e.g. an empty bucket -- are recomputed
// here; the others just take lane_sum[w] to the outputs)
template <class F>
SSB_INL void msm_window_block(uint32_t bid, jac<F>* sh, int c, const jac<F>* __restrict__ bsum, jac<F>* __restrict__ out_jac,
                              aff<F>* __restrict__ out_q, g1_aff* __restrict__ out_p,
                              const g1_aff* __restrict__ negg1_pow, const uint32_t* __restrict__ redo,
                              const jac<F>* __restrict__ lane_sum) {
  const int t = threadIdx.x, B = 1 << c, L = B < 64 ? B : 64, m = B / L;
  const jac<F>* bk = bsum + (size_t)bid * B;
  if (redo && !redo[bid]) {
    if (t == 0) {
      const jac<F> U = lane_sum[bid];
      if (out_jac) out_jac[bid] = U;
      if (out_q) {
        aff<F> a;
        jac_to_aff(a, U);
        out_q[bid] = a;
        out_p[bid] = negg1_pow[c * bid];
      }
    }
    return;
  }
  jac<F> S, U;
  jac_set_inf(S);
  jac_set_inf(U);
  if (t < L) {
    for (int e = m - 1; e >= 1; --e) { jac<F> o = bk[t * m + e]; jac_add(S, S, o); jac_add(U, U, S); }
    jac<F> o = bk[t * m]; jac_add(S, S, o);
  }
  // suffix scan over the lanes: S_t <- sum_{t' >= t} S_t'  (blocks wider than 64 lanes: the lanes
  // past 64 only keep the barriers)
  for (int off = 1; off < L; off <<= 1) {
    if (t < 64) sh[t] = S;
    __syncthreads();
    if (t + off < L) { jac<F> o = sh[t + off]; jac_add(S, S, o); }
    __syncthreads();
  }
  if (t >= 1 && t < L) {
    for (int q = m; q > 1; q >>= 1) jac_dbl(S, S);
    jac_add(U, U, S);
  }
  for (int h = L >> 1; h >= 1; h >>= 1) {
    if (t < 64) sh[t] = U;
    __syncthreads();
    if (t < h) { jac<F> o = sh[t + h]; jac_add(U, U, o); }
    __syncthreads();
  }
  if (t == 0) {
    if (out_jac) out_jac[bid] = U;
    if (out_q) {
      aff<F> a;
      jac_to_aff(a, U);
      out_q[bid] = a;
      out_p[bid] = negg1_pow[c * bid];
    }
  }
}

// ---- window sums for narrow windows (2^c <= 16 buckets): one lane per (group, window), the
// sequential running sum  R += B_d, U += R  for d = 2^c - 1 .. 1  (2 (2^c - 1) additions) ----
template <class F>
SSB_INL void msm_window_seq_block(uint32_t bid, uint32_t ngw, int c, const jac<F>* __restrict__ bsum,
                                  jac<F>* __restrict__ out_jac) {
  const uint32_t gw = bid * blockDim.x + threadIdx.x;
  if (gw >= ngw) return;
  const int B = 1 << c;
  const jac<F>* bk = bsum + (size_t)gw * B;
  jac<F> R, U;
  jac_set_inf(R);
  jac_set_inf(U);
  for (int d = B - 1; d >= 1; --d) {
    jac<F> o = bk[d];
    jac_add(R, R, o);
    jac_add(U, U, R);
  }
  out_jac[gw] = U;
}
// 2: simplified SWU, one lane per (root, u_j, candidate x1 / x2): both square roots run at once
// instead of one after the other; then the 3-isogeny.  Lanes 4i+2j+c, 16 roots per block.
struct h2c_cand { fp2 x, y; uint32_t ok; };
constexpr size_t H2C_MAP_LDS = 64 * sizeof(h2c_cand);
SSB_INL void h2c_map_block(uint32_t bid, h2c_cand* cs, int n, const fp2* __restrict__ u, g2_aff* __restrict__ q) {
  const int t = bid * 64 + threadIdx.x;
  const int i = t >> 2, j = (t >> 1) & 1, c = t & 1;
  const bool act = i < n;
  fp2 uu = act ? u[2 * i + j] : fp2_one();
  fp2 x, y;
  const bool ok = sswu_candidate(x, y, uu, c);
  cs[threadIdx.x].x = x; cs[threadIdx.x].y = y; cs[threadIdx.x].ok = ok ? 1u : 0u;
  __syncthreads();
  if (act && c == 0) {
    const h2c_cand o = cs[threadIdx.x + 1];
    g2_aff r;
    sswu_finish(r, uu, ok ? x : o.x, ok ? y : o.y);
    q[2 * i + j] = r;
  }
}

// 3: q0 + q1 and the cofactor clearing as lane-group programs (8 lanes per root, 8 roots per block)
constexpr int H2C_S0 = lane::G2_ADD_SCRATCH > lane::G2_MADD_SCRATCH ? lane::G2_ADD_SCRATCH : lane::G2_MADD_SCRATCH;
constexpr int H2C_GS = H2C_S0 + 6 + 4 + 6 + 30;
constexpr size_t H2C_CLEAR_LDS = (lane::LP_NCODE_CONST + 8 * H2C_GS) * sizeof(lane::lslot) + 8 * sizeof(uint32_t);
SSB_INL void h2c_clear_block(uint32_t bid, lane::lslot* lds, int n, const g2_aff* __restrict__ q, g2_jac* __restrict__ hj,
                             uint32_t* __restrict__ exc_out) {
  using namespace ssb::lane;
  uint32_t* flg = (uint32_t*)(lds + LP_NCODE_CONST + 8 * H2C_GS);
  const int gi = threadIdx.x / 8, role = threadIdx.x % 8;
  const int i = bid * 8 + gi;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST + gi * H2C_GS, 0, 0, 0, (lu32*)&flg[gi], role};
  lp_init_consts(g);
  const bool act = i < n;
  const int P = H2C_S0, Q1 = P + 6, R = Q1 + 4, W = R + 6;
  {
    g2_aff a0, a1;
    if (act) { a0 = q[2 * i]; a1 = q[2 * i + 1]; } else { a0.x = fp2_zero(); a0.y = fp2_one(); a1 = a0; a1.x = fp2_one(); }
    if (role < 4) { lp_put(g.s + P + role, lv_in(((const fp*)&a0)[role])); lp_put(g.s + Q1 + role, lv_in(((const fp*)&a1)[role])); }
    if (role == 4) lp_put(g.s + P + 4, lv_one());
    if (role == 5) lp_put(g.s + P + 5, lv_zero());
  }
  __syncthreads();
  uint32_t exc = 0;
  g2_madd(g, P, Q1, P, exc);      // q0 + q1 (q0, q1 never infinity: iso3_map of the SWU points)
  g2_clear_cofactor(g, P, R, W, exc);
  if (act) {
    if (role < 6) ((fp*)&hj[i])[role] = lv_out(lp_get(g.s + R + role));
    if (role == 0) exc_out[i] = exc;
  }
}

// 4: affine output; a root whose lane-group stage met an exceptional addition (or every root,
// with exact_all: the test knob SSB_H2C_EXACT) is redone exactly, hj[i] serving as its temporary
SSB_INL void h2c_affine_block(uint32_t bid, int n, const g2_aff* __restrict__ q, g2_jac* __restrict__ hj,
                              const uint32_t* __restrict__ exc, int exact_all, g2_aff* __restrict__ out) {
  const int i = bid * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2_jac s;
  if (exc[i] || exact_all) {
    h2c_clear_exact(s, q[2 * i], q[2 * i + 1], &hj[i]);
  } else {
    s = hj[i];
  }
  g2_aff a;
  jac_to_aff(a, s);
  out[i] = a;
}

// ---- per-job bodies of the a-1 scan and the combine (ssb_k_combine.hip; the one-stream path also
// runs them speculatively beside the window sums) ----
// A job the engine cannot run -- t == 0, t > SSB_MAX_T, share_off[j + 1] < share_off[j] or past the
// batch's n_shares (only the *_dev entry points can pass one: the host wrapper refuses them) --
// gets SSB_DVF_INVALID_JOB and is never selected, so no later kernel indexes its fixed t-arrays or
// its share range.  (k_share_map clamps the ranges the same way.)
SSB_INL bool job_ok(uint32_t b, uint32_t e, uint32_t t, uint32_t n_shares) {
  return t >= 1 && t <= SSB_MAX_T && b <= e && e <= n_shares;
}
// share -> (job, root): job j = the last j with off[j] <= s (binary search over off[0..n_jobs]).  A
// share outside every well-formed job's range -- share_off not monotone, off[0] > 0,
// off[n_jobs] < n_shares, or its job fails job_ok -- gets the sentinel 0xffffffff for both (no
// H(root): never a candidate; the combine kernels skip it), so no kernel reads a stale entry of the
// reused workspace or indexes a job array past n_jobs.  (tt == nullptr: no job_ok check.)
SSB_INL void share_lookup(uint32_t s, const job_map& jm, uint32_t& job, uint32_t& root) {
  int lo = 0, hi = jm.n_jobs;   // invariant (monotone off): off[lo] <= s < off[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (jm.off[mid] <= s) lo = mid; else hi = mid;
  }
  const uint32_t b = jm.off[lo], e = jm.off[lo + 1];
  const bool in = jm.n_jobs > 0 && b <= s && s < e && (!jm.tt || job_ok(b, e, jm.tt[lo], jm.n_shares));
  job = in ? (uint32_t)lo : 0xffffffffu;
  root = in ? (jm.job_root ? jm.job_root[lo] : 0u) : 0xffffffffu;
}
// wst != nullptr (the wire-record path, ssb_threshold_aggregate_batch_wire_cached_dev): a share whose
// record did not deserialize -- a format error (wst[s] 1..3) or bytes that do not decompress (DEC_OK
// clear; wst[s] := 4 here) -- is ABSENT, as the reference drops it before the call
// (RemoteOperator::sign, operator.rs:108-131, then `.flatten()` in HotstuffOperatorCommittee::sign,
// hotstuff.rs:150-155): it does not count towards sigs.len() (InsufficientSignatures{got: present,
// expected: t}) and the scan never meets it.
SSB_INL void select_job(int j, uint32_t n_shares, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                        const uint64_t* __restrict__ ids, const uint8_t* __restrict__ verdict,
                        const uint32_t* __restrict__ flags, uint32_t* __restrict__ sel, int32_t* __restrict__ status,
                        uint64_t* __restrict__ err, int32_t* __restrict__ wst = nullptr) {
  const uint32_t b = off[j], e = off[j + 1], t = tt[j];
  if (!job_ok(b, e, t, n_shares)) { status[j] = SSB_DVF_INVALID_JOB; err[2 * j] = t; err[2 * j + 1] = e - b; return; }
  uint32_t n = e - b;
  if (wst) {
    for (uint32_t s = b; s < e; ++s)
      if (!(flags[s] & DEC_OK)) {
        if (wst[s] == 0) wst[s] = 4;
        --n;
      }
  }
  if (n < t) { status[j] = SSB_DVF_INSUFFICIENT_SIGNATURES; err[2 * j] = n; err[2 * j + 1] = t; return; }
  uint32_t cnt = 0;
  for (uint32_t s = b; s < e; ++s) {
    if (wst && !(flags[s] & DEC_OK)) continue;   // absent
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
SSB_FN void lagrange_job(int j, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                          const uint64_t* __restrict__ ids, const uint32_t* __restrict__ sel, fr* __restrict__ lam) {
  const uint32_t b = off[j], t = tt[j];
  uint64_t x[SSB_MAX_T];
  for (uint32_t i = 0; i < t; ++i) x[i] = ids[sel[b + i]];
  unit_lagrange_fast(lam + b, x, t);
}
// Small-integer Lagrange fast path (unit_lagrange_small), for t <= FAST_T (larger thresholds take
// the 255-bit path; the per-lane arrays stay small -- this kernel's private segment sets the
// scratch the runtime reserves on every slot's hardware queue): every selected share is a verified
// (hence order-r) point, so sum c_i sig_i with the integer c_i == lambda_i mod r is the reference's
// combination.  fast[j] = 1 when the job was finished here; the 255-bit path skips those jobs.
constexpr uint32_t FAST_T = 16;
// The combine of job j after its selection: small-integer Lagrange coefficients (ids 1..n:
// unit_lagrange_small) finish the job here (returns 1, out96 written); coefficients that are ratios
// of small integers (registry ids, and ids 1..n with a share skipped: unit_lagrange_ratio) return 2
// -- k_combine_ratio finishes the job, one lane each (unit_combine_ratio_w4); else 0 (the general
// path: lambda_i, k_combine_terms_gls, k_combine_sum).  `ratio` = 0 (SSB_NO_RATIO): never 2.
// One function for both, out of line: one set of per-lane arrays in its own frame.
// The coefficients' kind, a leaf (no calls: a function that calls out keeps its values in the
// callee-saved VGPRs and saves ~110 of them in its frame -- combine_job did, 736 B, round 5):
// 1 with c[] the small-integer coefficients, 2 (ratio != 0) ratio coefficients, else 0.
SSB_FN uint32_t lagrange_kind(int64_t* __restrict__ c, const uint64_t* __restrict__ ids, const uint32_t* __restrict__ sel,
                              uint32_t t, uint32_t ratio) {
  uint64_t x[FAST_T];
  for (uint32_t i = 0; i < t; ++i) x[i] = ids[sel[i]];
  if (unit_lagrange_small(c, x, t)) return 1u;
  uint64_t M;
  return ratio && unit_lagrange_ratio(c, &M, x, t) ? 2u : 0u;
}
// the small-integer combine of a job lagrange_kind classed 1 (its coefficients recomputed here, so
// no array of them lives in combine_job's frame across a call)
SSB_FN void combine_small_job(uint8_t* __restrict__ out96, const g2_aff* __restrict__ sig_aff,
                              const uint64_t* __restrict__ ids, const uint32_t* __restrict__ sel, uint32_t t) {
  int64_t c[FAST_T];
  lagrange_kind(c, ids, sel, t, 0u);
  unit_combine_small_at(out96, sig_aff, sel, c, t);
}
SSB_FN uint32_t lagrange_class(const uint64_t* __restrict__ ids, const uint32_t* __restrict__ sel, uint32_t t,
                               uint32_t ratio) {
  int64_t c[FAST_T];
  return lagrange_kind(c, ids, sel, t, ratio);
}
SSB_FN uint32_t combine_job(int j, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                            const int32_t* __restrict__ status, const uint32_t* __restrict__ sel,
                            const uint64_t* __restrict__ ids, const g2_aff* __restrict__ sig_aff,
                            uint8_t* __restrict__ out96, uint32_t ratio) {
  if (status[j] != SSB_DVF_OK || tt[j] > FAST_T) return 0u;
  const uint32_t t = tt[j], b = off[j];
  const uint32_t kind = lagrange_class(ids, sel + b, t, ratio);
  if (kind == 1u) combine_small_job(out96 + 96 * (size_t)j, sig_aff, ids, sel + b, t);
  return kind;
}
// Ratio jobs take the lane-uniform ratio combine only where they fill a wave: with fewer than
// RATIO_MIN_JOBS of a wave's 64 jobs marked 2 (ids 1..n with a share skipped -- the jobs an invalid
// share leaves behind -- are ratio jobs too, a few per wave), the wave would run the whole ratio
// chain (~9k dependent Fp products on ONE lane) for them, and its latency set the batch's tail: at
// 1e-2 invalid shares k_combine_sum averaged 11.6 ms and k_combine_terms_gls 4.9 ms per launch
// (round 5).  Those jobs are marked 3: each runs on a workgroup of its own, its products spread
// over eight lane groups (k_combine_sum's extra blocks, ratio_lane_job) -- the general combine
// they took before (four GLS lanes per share, each a ~2.9k-product chain on one lane) still set a
// 7.7-9.9 ms k_combine_terms_gls on the 1e-2 batch's chain (round 5, depth-1 trace).
// Every lane of the wave must call this (a ballot); the wave's 64 jobs are 64 consecutive js.
constexpr uint32_t RATIO_MIN_JOBS = 16;
static_assert(RATIO_MIN_JOBS - 1 == RATIO_LANE_PER_WAVE, "k_combine_sum's extra blocks per wave");
SSB_INL uint32_t ratio_by_wave(uint32_t f) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t m = __ballot(f == 2u);
  if (f == 2u && (uint32_t)__popcll(m) < RATIO_MIN_JOBS) return 3u;
#endif
  return f;
}
// the ratio coefficients of a job combine_job marked 2 (recomputed: a few 64-bit operations)
SSB_INL void ratio_coeffs(int j, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                          const uint32_t* __restrict__ sel, const uint64_t* __restrict__ ids, int64_t* c,
                          uint64_t* M) {
  const uint32_t t = tt[j], b = off[j];
  uint64_t x[FAST_T];
  for (uint32_t i = 0; i < t; ++i) x[i] = ids[sel[b + i]];
  unit_lagrange_ratio(c, M, x, t);
}
}  // namespace k
}  // namespace ssb
