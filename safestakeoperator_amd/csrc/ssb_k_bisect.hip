// ssb_k_bisect.hip -- kernels (gfx950): exact per-share verdicts after a failed RLC batch check,
// by group testing instead of one pairing check per share.
//
// "on batch failure, bisect deterministically until each share's verdict equals
// the single-verify result".  The shares of a failed batch are ordered by signing root (counting
// sort) and tested in root-aligned groups on a B-ary tree (B = 16 by default): level 0 holds groups of
// Gs_0 = B^(L-1) >= n shares (one group per root), level l groups of Gs_0 / B^l, the last level single
// shares.  B = 16 rather than 4: the fallback runs on a shared tail stream and is latency bound
// (each level is one pairing check deep), so fewer, wider levels win -- at one invalid share per C2
// batch 3 tested levels instead of 5.
// A group g of root r passes when
//     e(sum_{i in g} k_i pk_i, H(r)) * e(-g1, sum_{i in g} k_i sig_i) == 1
// with the batch's own odd 64-bit RLC scalars k_i: every candidate of a passing group gets verdict 1
// (the batch check's soundness, 2^-63 per group); a failing single-share group is exactly the
// reference's verify (k_i != 0 mod r), so it gets verdict 0.  Children of a passing group are not
// tested; a group whose share range equals its failed parent's inherits the failure untested.
// Launches (all on the slot's stream, each a uniform no-op when the batch passed):
//   k_fb_rlc     verdicts the batch check decides, the candidates' scalars k_i, counting sort by root,
//                the committee relations (suspect jobs)
//   k_fb_excl    the committee stage: exclusion check + suspects alone, or the group-test mode
//   k_fb_root    level 0, one check per root (or the committee stage's verdicts / deductions): S_r = sum k_i sig_i as a 4-bit-digit bucket sum (no
//                per-share products); e(PK_r, H(r)) is the batch check's own Miller value
//   k_fb_single  <= FB_SINGLE_MAX shares in failing roots: each checked alone (no products, one
//                pairing check deep) -- one invalid share per C2 batch: 256 single checks
//                otherwise (same launch): k_i sig_i, k_i pk_i for the failing roots' candidates, then
//   k_fb_level l the 16-ary levels below the root (work at 1% invalid shares, C2: ~3.5k group checks
//                instead of 16,384 per-share checks)
// lane-program kernels at two waves per SIMD (256 registers, the rest spilled within the queue
// primer's private segment): under load they no longer wait for a whole SIMD's register file
#ifndef SSB_WAVES_PER_EU
#define SSB_WAVES_PER_EU 2
#endif
#include "ssb_kernels.h"
#include "ssb_lane_ops.h"

namespace ssb {
namespace k {

using launch::fb_jobs;
// committee stage: at most this many suspect shares are checked one by one (beyond it the tree decides)
constexpr uint32_t FB_SUSPECT_MAX = 2048;
constexpr unsigned EX_SINGLE_BLOCKS = 512;
// the exclusion check's parts of X: slices of at most this many suspects (EX_X_PARTS of them cover all)
constexpr uint32_t EX_X_SHARES = (FB_SUSPECT_MAX + launch::EX_X_PARTS - 1) / launch::EX_X_PARTS;
// grid of the fallback launches that stride over their work (k_fb_single, k_fb_level):
// most failed batches leave them at their first test, and a grid of thousands of blocks waited
// milliseconds for free slots behind the other pipeline slots' waves (round 4 profile of the 1e-2
// workload: k_fb_single 6.0 ms, the former k_fb_group 2.9 ms per launch while doing nothing)
constexpr unsigned FB_GRID_MAX = 512;

// One workgroup (the last block of k_fb_rlc's grid): counting sort of the shares by (root, operator-id
// bucket) -- key = root * NB + bucket(id), NB = fb_nbuckets(n_roots) -- into perm, the per-key
// segments (kcnt, kstart) and the per-root ones they nest in (cnt, start), and the group starts of
// every tree level (gst[l][r], n_roots + 1 words per level); it also zeroes k_fb_root's per-root
// tickets.  Inside a root the shares of one operator id are contiguous: the committee stage's group
// tests (a faulty operator's shares fail together) and the tree's level groups (any order is valid
// for them) use the same permutation.  Phases separated by workgroup barriers (global atomics and
// stores of one workgroup are ordered by them).
struct fb_prep_args { int n_roots, L, lb; const uint32_t* share_root; uint32_t* cnt; uint32_t* start; uint32_t* cursor;
                      uint32_t* gst; uint32_t* perm; uint32_t* rtk; uint32_t* nfail; const uint64_t* ids;
                      uint32_t* kcnt; uint32_t* kstart; uint32_t* klist; uint32_t* ictr; };
SSB_INL uint32_t fb_bucket(uint64_t id, int nb) {
  return nb > 1 ? (uint32_t)((id * 0x9E3779B97F4A7C15ull) >> 60) & (uint32_t)(nb - 1) : 0u;
}
SSB_INL void fb_prep_block(int n, const fb_prep_args& a) {
  const int t = threadIdx.x, NT = blockDim.x, n_roots = a.n_roots, L = a.L, lb = a.lb;
  const int NB = a.ids && a.kcnt ? launch::fb_nbuckets(n_roots) : 1;
  const int K = n_roots * NB;
  const uint32_t* __restrict__ share_root = a.share_root;
  uint32_t* __restrict__ cnt = a.cnt;
  uint32_t* __restrict__ start = a.start;
  uint32_t* __restrict__ cursor = a.cursor;
  uint32_t* __restrict__ gst = a.gst;
  uint32_t* __restrict__ perm = a.perm;
  uint32_t* __restrict__ kc = NB > 1 ? a.kcnt : cnt;       // per-key counts (the roots' when NB == 1)
  uint32_t* __restrict__ ks = NB > 1 ? a.kstart : start;
  auto key = [&](int s) { return share_root[s] * (uint32_t)NB + (NB > 1 ? fb_bucket(a.ids[s], NB) : 0u); };
  for (int k = t; k < K; k += NT) kc[k] = 0u;
  for (int r = t; r < n_roots; r += NT) a.rtk[r] = 0u;
  if (t == 0) *a.nfail = 0u;
  if (t == 0 && a.ictr) *a.ictr = 0u;   // k_fb_excl's group-test item counter (the next launch on the stream)
  __syncthreads();
  for (int s = t; s < n; s += NT)
    if (share_root[s] < (uint32_t)n_roots) atomicAdd(&kc[key(s)], 1u);
  __syncthreads();
  if (t == 0) {
    uint32_t acc = 0;
    uint32_t m = 0;
    for (int k = 0; k < K; ++k) {
      ks[k] = acc; cursor[k] = acc; acc += kc[k];
      if (a.klist && kc[k]) a.klist[m++] = (uint32_t)k;
    }
    if (a.klist) a.klist[K] = m;   // (the group-test items: four per listed key)
  }
  __syncthreads();
  if (NB > 1)
    for (int r = t; r < n_roots; r += NT) {
      uint32_t c = 0;
      for (int b = 0; b < NB; ++b) c += kc[r * NB + b];
      cnt[r] = c;
      start[r] = ks[r * NB];
    }
  __syncthreads();
  if (t < L) {
    const int l = t;
    const uint32_t lg = (uint32_t)(lb * (L - 1 - l));   // Gs_l = 2^lg
    uint32_t* g = gst + (size_t)l * (n_roots + 1);
    uint32_t acc = 0;
    for (int r = 0; r < n_roots; ++r) {
      g[r] = acc;
      acc += (uint32_t)(((uint64_t)cnt[r] + (1ull << lg) - 1) >> lg);
    }
    g[n_roots] = acc;
  }
  for (int s = t; s < n; s += NT)
    if (share_root[s] < (uint32_t)n_roots) perm[atomicAdd(&cursor[key(s)], 1u)] = (uint32_t)s;
}
// ---- committee stage (aggregate batches): consistency of each job's shares ------------------------
// All valid shares of a job lie on one polynomial of degree t - 1 (generic_threshold.rs:59-80: the
// key split; src/crypto/impls/blst.rs:19-39: the combine relies on it), so any t + 1 of them satisfy
// the t-th divided difference  sum_i sig_i / prod_{j != i} (x_i - x_j) = O, i.e. with integer
// coefficients c_i = L / prod_{j != i} (x_i - x_j)  (L the lcm of the denominators; ids 1..4:
// -1, 3, -3, 1)  sum_i c_i sig_i = O.  A job whose shares break one of its relations holds an
// invalid share: its candidates become SUSPECT (checked one by one) and the rest of the batch is
// re-checked at once by excluding them from the batch check (k_fb_excl).  The relation is only a
// partition heuristic -- every verdict still comes from a pairing check (an adversary who makes
// invalid shares satisfy it only sends them into the exclusion check, which then fails, and the
// tree below decides).  Ids whose coefficients overflow 63 bits, duplicates and t > REL_TMAX give
// no relation (the job is left to the exclusion check).
constexpr int REL_TMAX = 16;
SSB_INL int64_t rel_gcd(int64_t a, int64_t b) {
  if (a < 0) a = -a;
  if (b < 0) b = -b;
  while (b) { const int64_t t = a % b; a = b; b = t; }
  return a;
}
SSB_INL bool rel_coeffs(int64_t* c, const uint64_t* x, int m) {
  int64_t L = 1;
  for (int i = 0; i < m; ++i) {
    if (x[i] >= (1ull << 62)) return false;
    int64_t d = 1;
    for (int j = 0; j < m; ++j) {
      if (j == i) continue;
      const int64_t df = (int64_t)x[i] - (int64_t)x[j];
      if (df == 0 || __builtin_mul_overflow(d, df, &d)) return false;
    }
    c[i] = d;
    const int64_t a = d < 0 ? -d : d, g = rel_gcd(L, a);
    if (__builtin_mul_overflow(L / g, a, &L)) return false;
  }
  for (int i = 0; i < m; ++i) c[i] = L / c[i];
  return true;
}
// job j: the relations over its first t candidates plus each further candidate; on a broken one
// every candidate of the job is marked SUSPECT and listed (slist, nS)
SSB_INL void consist_job(int j, uint32_t n, const fb_jobs& jb, uint32_t* __restrict__ flags,
                         const g2_aff* __restrict__ sig_aff, uint32_t* __restrict__ slist, uint32_t* __restrict__ nS) {
  const uint32_t b = jb.off[j], e = jb.off[j + 1], t = jb.tt[j];
  if (e < b || e > n || t == 0 || t > (uint32_t)REL_TMAX) return;
  uint32_t base[REL_TMAX];
  uint64_t x[REL_TMAX + 1];
  int64_t c[REL_TMAX + 1];
  uint32_t nb = 0;
  bool sus = false;
  for (uint32_t s = b; s < e && !sus; ++s) {
    if (!(flags[s] & FLAG_CANDIDATE)) continue;
    if (nb < t) { base[nb++] = s; continue; }
    for (uint32_t i = 0; i < t; ++i) x[i] = jb.ids[base[i]];
    x[t] = jb.ids[s];
    if (!rel_coeffs(c, x, (int)t + 1)) continue;
    uint64_t mx = 0;
    for (uint32_t i = 0; i <= t; ++i) { const uint64_t m = (uint64_t)(c[i] < 0 ? -c[i] : c[i]); mx = m > mx ? m : mx; }
    const int nbits = mx ? 64 - __builtin_clzll(mx) : 0;
    g2_jac acc;
    jac_set_inf(acc);
    for (int bit = nbits - 1; bit >= 0; --bit) {
      jac_dbl(acc, acc);
      for (uint32_t i = 0; i <= t; ++i) {
        const uint64_t m = (uint64_t)(c[i] < 0 ? -c[i] : c[i]);
        if ((m >> bit) & 1ull) {
          g2_aff q = sig_aff[i < t ? base[i] : s];
          if (c[i] < 0) fp2_neg(q.y, q.y);
          jac_add_aff(acc, acc, q);
        }
      }
    }
    sus = !jac_is_inf(acc);
  }
  if (!sus) return;
  for (uint32_t s = b; s < e; ++s)
    if (flags[s] & FLAG_CANDIDATE) {
      atomicOr(&flags[s], (uint32_t)FLAG_SUSPECT);
      const uint32_t k = atomicAdd(nS, 1u);
      if (k < FB_SUSPECT_MAX) slist[k] = s;
    }
}

// sum_i c_i P_i == O for the points P_i = pts[i < m - 1 ? base[i] : extra] (signed binary, shared
// doublings) -- a committee relation over t + 1 shares, in G1 (public keys) or G2 (signatures)
template <class F>
SSB_INL bool rel_holds(const aff<F>* __restrict__ pts, const uint32_t* base, uint32_t extra, const int64_t* c, int m) {
  uint64_t mx = 0;
  for (int i = 0; i < m; ++i) { const uint64_t v = (uint64_t)(c[i] < 0 ? -c[i] : c[i]); mx = v > mx ? v : mx; }
  const int nbits = mx ? 64 - __builtin_clzll(mx) : 0;
  jac<F> acc;
  jac_set_inf(acc);
  for (int bit = nbits - 1; bit >= 0; --bit) {
    jac_dbl(acc, acc);
    for (int i = 0; i < m; ++i) {
      const uint64_t v = (uint64_t)(c[i] < 0 ? -c[i] : c[i]);
      if ((v >> bit) & 1ull) {
        aff<F> q = pts[i < m - 1 ? base[i] : extra];
        if (c[i] < 0) f_neg(q.y, q.y);
        jac_add_aff(acc, acc, q);
      }
    }
  }
  return jac_is_inf(acc);
}
// Group-test mode, after the group tests: job j's undecided candidates from the relations.  With t
// shares of the job PROVEN valid (passing groups: sig_i = s_i H, pk_i = s_i g1) and the public-key
// relation over them and share u holding (pk_u = s'_u g1 with s'_u the interpolated share), share u is
// valid -- e(pk_u, H) == e(g1, sig_u) -- exactly when sig_u = s'_u H, i.e. when the signature relation
// holds (c_u != 0 mod r: |c_u| < 2^62).  So the verdict of u follows without a pairing; a faulty
// operator's share in every committee is decided this way.  Without t proven shares, or when the
// key relation fails, u is left to its single check.
SSB_FN void deduce_job(int j, uint32_t n, const fb_jobs& jb, uint32_t* __restrict__ flags, uint8_t* __restrict__ verdict,
                       const g2_aff* __restrict__ sig_aff, const g1_aff* __restrict__ pk_aff) {
  const uint32_t b = jb.off[j], e = jb.off[j + 1], t = jb.tt[j];
  if (e < b || e > n || t == 0 || t > (uint32_t)REL_TMAX) return;
  uint32_t base[REL_TMAX];
  uint32_t nb = 0;
  bool open = false;
  for (uint32_t s = b; s < e; ++s) {
    const uint32_t f = flags[s];
    if (!(f & FLAG_CANDIDATE)) continue;
    if (!(f & FLAG_DECIDED)) { open = true; continue; }
    if (verdict[s] && nb < t) base[nb++] = s;
  }
  if (!open || nb < t) return;
  uint64_t x[REL_TMAX + 1];
  int64_t c[REL_TMAX + 1];
  for (uint32_t i = 0; i < t; ++i) x[i] = jb.ids[base[i]];
  for (uint32_t s = b; s < e; ++s) {
    const uint32_t f = flags[s];
    if (!(f & FLAG_CANDIDATE) || (f & FLAG_DECIDED)) continue;
    x[t] = jb.ids[s];
    if (!rel_coeffs(c, x, (int)t + 1)) continue;
    if (!rel_holds<fp>(pk_aff, base, s, c, (int)t + 1)) continue;
    verdict[s] = rel_holds<fp2>(sig_aff, base, s, c, (int)t + 1) ? 1 : 0;
    atomicOr(&flags[s], (uint32_t)FLAG_DECIDED);
  }
}

// Threads [0, n): the candidates' RLC scalars k64[s] (the main check's own, rlc_scalar_odd).  With
// `verdict` it also writes, grid-wide, the verdicts the batch check decides: every share of a
// passing batch, the non-candidates of a failing one (the candidates' follow from the group tests).
// Blocks after the shares' (jobs given): the committee consistency of 64 jobs each (consist_job).
// The grid's last block runs the counting sort by root (fb_prep_block).
__global__ void SSB_LB(64) k_fb_rlc(int n, rlc_key key, const uint32_t* __restrict__ ok,
                                   uint32_t* __restrict__ flags, uint64_t* __restrict__ k64,
                                   uint8_t* __restrict__ verdict, fb_prep_args prep, fb_jobs jobs,
                                   const g2_aff* __restrict__ sig_aff, uint32_t* __restrict__ slist,
                                   uint32_t* __restrict__ nS) {
  const uint32_t pass = *ok;
  if (blockIdx.x == gridDim.x - 1) {   // uniform per block
    if (!pass) fb_prep_block(n, prep);
    return;
  }
  const int nbs = (n + 63) / 64;
  if ((int)blockIdx.x >= nbs) {        // committee consistency
    const int j = ((int)blockIdx.x - nbs) * 64 + (int)threadIdx.x;
    if (!pass && j < jobs.n_jobs) consist_job(j, (uint32_t)n, jobs, flags, sig_aff, slist, nS);
    return;
  }
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const bool cand = (flags[g] & FLAG_CANDIDATE) != 0;
  if (verdict && (pass || !cand)) verdict[g] = cand ? 1 : 0;
  if (!pass && cand) k64[g] = rlc_scalar_odd(key, (uint64_t)g);
}

// Level 0 of the tree (one group per root) without per-share products: the root's group check is
//     e(PK_r, H(r)) * e(-g1, S_r) == 1,   PK_r = sum_{i in r} k_i pk_i,  S_r = sum_{i in r} k_i sig_i
// over the root's candidates -- and e(PK_r, H(r)) before the final exponentiation is the main check's
// own Miller value f[r] (pair r of the batch check is (PK_r, H(r)), ssbls.hip run_verify), so only S_r
// is new: a Pippenger sum with 4-bit digits, 16 windows x 15 buckets per root, ~16 mixed additions
// per share instead of a 64-bit double-and-add in G2 AND G1 per share (the former k_fb_rlc).
// Block (r, q) owns windows 4q .. 4q+3 of root r, lane (w, d) = bucket d of window 4q + w: the
// root's shares are sorted into the 64 buckets in LDS (chunks of FR_CHUNK shares), each lane sums
// its bucket, a 16-lane suffix scan and tree give W_w = sum_d d B_{w,d}, and
// X_q = sum_w 2^(4w) W_{4q+w}.  The last of the root's four blocks (completion ticket rtk[r], zeroed
// by fb_prep_block) forms S_r = sum_q 2^(16q) X_q and runs the check: one lane-program Miller loop
// e(-g1, S_r), times f[r], final exponentiation.  gv0[group of r] and, on a pass, the verdicts of
// the root's candidates.  Product-free: the failing roots' per-share products follow in k_fb_single's
// launch (sparse_product).
constexpr int FR_CHUNK = 512;
// at most this many shares in failing roots after level 0: k_fb_single checks them one by one
constexpr uint32_t FB_SINGLE_MAX = 384;
constexpr int bs_max(int a, int b) { return a > b ? a : b; }
constexpr int BS_S0 = bs_max(bs_max(bs_max(lane::MILLER_ITER_SCRATCH, lane::MILLER_ADDSTEP_SCRATCH),
                                    bs_max(lane::MILLER_ITER2_SCRATCH, lane::MILLER_ADDSTEP2_SCRATCH)),
                             lane::FP12_MUL_SCRATCH);
// F: f | T1 | T2 (24), B: the pairs (12), BP: 4 work slots, TMP: the final exponentiation's 84
constexpr int BS_SLOTS = BS_S0 + 24 + 12 + 4 + 84;

// The per-share products the levels below 0 sum, for the candidates of the roots whose level-0
// check failed only: items [0, n) rsig[s] = k_s sig_s, [n, 2n) rpk[s] = k_s pk_s (run by
// k_fb_single's blocks when the failing roots hold more than FB_SINGLE_MAX shares).
// Binary double-and-add (no window table): the private segment stays small -- every slot queue
// reserves scratch for the largest kernel it has run, and this one is launched on every batch.
SSB_FN void sparse_product(int g, int n, int n_roots, const uint32_t* __restrict__ flags, const uint32_t* __restrict__ share_root,
                           const uint32_t* __restrict__ gst0, const uint8_t* __restrict__ gv0, const uint64_t* __restrict__ k64,
                           const g2_aff* __restrict__ sig_aff, const g1_aff* __restrict__ pk_aff, g2_jac* __restrict__ rsig,
                           g1_jac* __restrict__ rpk) {
  const int s = g < n ? g : g - n;
  if (s >= n || !(flags[s] & FLAG_CANDIDATE)) return;
  const uint32_t r = share_root[s];
  if (r >= (uint32_t)n_roots || gv0[gst0[r]]) return;   // the root passed: its shares are decided
  const uint64_t k = k64[s];
  const uint32_t kw[2] = {(uint32_t)k, (uint32_t)(k >> 32)};
  if (g < n) { g2_jac o; jac_mul_aff(o, sig_aff[s], kw, 2); rsig[s] = o; }
  else { g1_jac o; jac_mul_aff(o, pk_aff[s], kw, 2); rpk[s] = o; }
}

// the Fp12 value in slots F .. F+11 == 1, one slot per lane (an fp12 local would take 144 registers);
// a workgroup-wide vote, so every lane gets the answer (and the slots are free again on return)
SSB_INL bool f12_slots_one(const lane::grp& g, int F) {
  __syncthreads();
  const int lane_ = threadIdx.x;
  bool one = true;
  if (lane_ < 12) { const fp v = lane::lv_out(lane::lp_get(g.s + F + lane_)); one = lane_ == 0 ? fp_eq(v, fp_one()) : fp_is_zero(v); }
  return __syncthreads_and(one ? 1 : 0) != 0;
}

// e(P, h) * e(-g1, Q) == 1 with the workgroup's lane programs (one two-pair loop when both pairs are
// finite; e(O, .) = e(., O) = 1), then the final exponentiation.  Uniform per workgroup.
SSB_FN bool pair_check(lane::grp& g, const g1_aff& P, const g2_aff& Q, const g2_aff& h, int F1, int B, int BP, int TMP) {
  using namespace ssb::lane;
  const int lane_ = threadIdx.x;
  const g1_aff ng = g1_neg_generator();
  if (!P.inf && !Q.inf) {                  // e(S_pk, H(r)) e(-g1, S_sig), one two-pair loop
    if (lane_ < 4) { lp_put(g.s + B + lane_, lv_in(((const fp*)&h)[lane_])); lp_put(g.s + B + 6 + lane_, lv_in(((const fp*)&Q)[lane_])); }
    if (lane_ == 4) { lp_put(g.s + B + 4, lv_in(P.x)); lp_put(g.s + B + 10, lv_in(ng.x)); }
    if (lane_ == 5) { lp_put(g.s + B + 5, lv_in(P.y)); lp_put(g.s + B + 11, lv_in(ng.y)); }
    __syncthreads();
    f12_miller2(g, F1, B, BP);
  } else if (!P.inf || !Q.inf) {           // one pair at infinity
    const g2_aff q = P.inf ? Q : h;
    if (lane_ < 4) lp_put(g.s + B + lane_, lv_in(((const fp*)&q)[lane_]));
    if (lane_ == 4) lp_put(g.s + B + 4, lv_in(P.inf ? ng.x : P.x));
    if (lane_ == 5) lp_put(g.s + B + 5, lv_in(P.inf ? ng.y : P.y));
    __syncthreads();
    f12_miller(g, F1, B);
  } else {
    const fp12 one = fp12_one();
    if (lane_ < 12) lp_put(g.s + F1 + lane_, lv_in(((const fp*)&one)[lane_]));
    __syncthreads();
  }
  f12_final_exp(g, F1, TMP);
  return f12_slots_one(g, F1);
}

// LDS of k_fb_root: the root's bucket lists (the point trees move through cross-lane shuffles, so
// the block's LDS stays small enough for two waves per SIMD)
struct fr_bucket_lds { uint32_t list[4 * FR_CHUNK]; uint32_t cnt[64], off[64], cur[64]; };
union fr_lds { fr_bucket_lds b; lane::lslot s[lane::LP_NCODE_CONST + BS_SLOTS]; };
template <class P> SSB_INL P shfl_down_pt(const P& p, int off) {
  P r;
  const int* a = (const int*)&p;
  int* b = (int*)&r;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(P) / 4); ++i) b[i] = __shfl_down(a[i], (unsigned)off, 64);
  return r;
}
SSB_INL g2_jac shfl_down_g2(const g2_jac& p, int off) { return shfl_down_pt(p, off); }

// X_q = sum_w 2^(4w) W_{4q+w} over the listed shares (bits 16q .. 16q+15 of their scalars k64):
// the shares are sorted into 64 buckets (4 windows x 16 digits) in LDS, chunk by chunk; lane (w, d)
// sums bucket d of window w; a 16-lane suffix scan and tree give W = sum_d d B_d; lanes 0, 16, 32, 48
// shift and add.  Result in lane 0.  Shares without `need` in their flags are skipped.
template <class F>
SSB_FN jac<F> quarter_sum(fr_bucket_lds& ub, const uint32_t* __restrict__ list, uint32_t nr,
                          const uint32_t* __restrict__ flags, uint32_t need, const uint64_t* __restrict__ k64,
                          const aff<F>* __restrict__ pts, int q) {
  const int lane_ = threadIdx.x, wl = lane_ >> 4, d = lane_ & 15;
  jac<F> acc;
  jac_set_inf(acc);
  for (uint32_t c0 = 0; c0 < nr; c0 += FR_CHUNK) {
    const uint32_t m = nr - c0 < (uint32_t)FR_CHUNK ? nr - c0 : (uint32_t)FR_CHUNK;
    ub.cnt[lane_] = 0u;
    __syncthreads();
    for (uint32_t x = lane_; x < m; x += 64) {
      const uint32_t s = list[c0 + x];
      if ((flags[s] & need) != need) continue;
      const uint32_t kq = (uint32_t)(k64[s] >> (16 * q));
      for (int w = 0; w < 4; ++w) { const uint32_t dg = (kq >> (4 * w)) & 15u; if (dg) atomicAdd(&ub.cnt[w * 16 + dg], 1u); }
    }
    __syncthreads();
    if (lane_ == 0) {
      uint32_t a = 0;
      for (int i = 0; i < 64; ++i) { ub.off[i] = a; ub.cur[i] = a; a += ub.cnt[i]; }
    }
    __syncthreads();
    for (uint32_t x = lane_; x < m; x += 64) {
      const uint32_t s = list[c0 + x];
      if ((flags[s] & need) != need) continue;
      const uint32_t kq = (uint32_t)(k64[s] >> (16 * q));
      for (int w = 0; w < 4; ++w) {
        const uint32_t dg = (kq >> (4 * w)) & 15u;
        if (dg) ub.list[atomicAdd(&ub.cur[w * 16 + dg], 1u)] = s;
      }
    }
    __syncthreads();
    const uint32_t e = ub.off[lane_] + ub.cnt[lane_];
    for (uint32_t i = ub.off[lane_]; i < e; ++i) { const aff<F> p = pts[ub.list[i]]; jac_add_aff_inl(acc, acc, p); }
    __syncthreads();
  }
  // W_w = sum_d d B_{w,d}: suffix sums S_d = sum_{d' >= d} B_{w,d'} over the window's 16 lanes (lane
  // d = 0 holds no bucket), then the sum of S_1 .. S_15
  for (int off = 1; off < 16; off <<= 1) {
    const jac<F> o = shfl_down_pt(acc, off);
    if (d + off < 16) jac_add_inl(acc, acc, o);
  }
  if (d == 0) jac_set_inf(acc);
  for (int h = 8; h >= 1; h >>= 1) {
    const jac<F> o = shfl_down_pt(acc, h);
    if (d < h) jac_add_inl(acc, acc, o);
  }
  // X_q = sum_w 2^(4w) W_{4q+w}  (lanes 0, 16, 32, 48)
  if (d == 0) for (int i = 0; i < 4 * wl; ++i) jac_dbl_inl(acc, acc);
  for (int h = 32; h >= 16; h >>= 1) {
    const jac<F> o = shfl_down_pt(acc, h);
    if (lane_ < h && d == 0) jac_add_inl(acc, acc, o);
  }
  return acc;
}
// quarter_sum stored by lane 0 at *out: one call per group sum, from the kernel (a function that held
// both group sums' results held both in its frame)
template <class F>
SSB_FN void quarter_sum_to(fr_bucket_lds& ub, const uint32_t* __restrict__ list, uint32_t nr,
                           const uint32_t* __restrict__ flags, uint32_t need, const uint64_t* __restrict__ k64,
                           const aff<F>* __restrict__ pts, int q, jac<F>* __restrict__ out) {
  const jac<F> a = quarter_sum<F>(ub, list, nr, flags, need, k64, pts, q);
  if (threadIdx.x == 0) *out = a;
}
// sum_q 2^(16q) X[q] (q < 4), affine, in lane 0 (infinity on the other lanes)
template <class F>
SSB_FN aff<F> combine_quarters(const jac<F>* __restrict__ X) {
  const int lane_ = threadIdx.x;
  jac<F> t;
  jac_set_inf(t);
  if (lane_ < 4) { t = X[lane_]; for (int i = 0; i < 16 * lane_; ++i) jac_dbl_inl(t, t); }
  for (int h = 2; h >= 1; h >>= 1) {
    const jac<F> o = shfl_down_pt(t, h);
    if (lane_ < h) jac_add_inl(t, t, o);
  }
  aff<F> Q;
  Q.inf = true;
  if (lane_ == 0) jac_to_aff(Q, t);
  return Q;
}
// Miller value m(P, Q) (lane program) into slots F1 .. F1+11 of the workgroup's LDS, or 1 when P or
// Q is infinity.  P, Q are read from lane 0; uniform.
SSB_FN void miller_one(lane::grp& g, const g1_aff& P, const g2_aff& Q, int F1, int B, uint32_t& flg) {
  using namespace ssb::lane;
  const int lane_ = threadIdx.x;
  if (lane_ == 0) {
    flg = (P.inf || Q.inf) ? 1u : 0u;
    if (!(P.inf || Q.inf)) {
      lp_put(g.s + B + 0, lv_in(Q.x.c0)); lp_put(g.s + B + 1, lv_in(Q.x.c1)); lp_put(g.s + B + 2, lv_in(Q.y.c0)); lp_put(g.s + B + 3, lv_in(Q.y.c1));
      lp_put(g.s + B + 4, lv_in(P.x)); lp_put(g.s + B + 5, lv_in(P.y));
    }
  }
  __syncthreads();
  const bool one = flg != 0;
  __syncthreads();
  if (one) {
    const fp12 o = fp12_one();
    if (lane_ < 12) lp_put(g.s + F1 + lane_, lv_in(((const fp*)&o)[lane_]));
    __syncthreads();
  } else {
    f12_miller(g, F1, B);
  }
}

// S_r = sum_q 2^(16q) X_q, then the root's check FE(f[r] * e(-g1, S_r)) == 1 (k_fb_root's last block of
// the root); out of line, so the root's point is not in the kernel's frame under the other chains
SSB_FN bool root_check(fr_lds& u, uint32_t& flg, const g2_jac* __restrict__ Xr, const fp12* __restrict__ fr) {
  using namespace ssb::lane;
  const int lane_ = threadIdx.x;
  const g2_aff Q = combine_quarters<fp2>(Xr);
  __syncthreads();   // (the bucket lists are dead: the LDS becomes the lane programs' slots)
  grp g{(lfp*)u.s, (lfp*)u.s + LP_NCODE_CONST, 0, 0, 0, (lu32*)&flg, lane_};
  lp_init_consts(g);
  const int F1 = BS_S0, B = F1 + 24, TMP = B + 12 + 4, FR = TMP + 72;
  miller_one(g, g1_neg_generator(), Q, F1, B, flg);   // e(-g1, O) = 1: the root's value is f[r] alone
  if (lane_ < 12) lp_put(g.s + FR + lane_, lv_in(((const fp*)fr)[lane_]));
  __syncthreads();
  f12_mul(g, F1, FR, F1);
  f12_final_exp(g, F1, TMP);
  return f12_slots_one(g, F1);
}
__global__ void SSB_LB2(64) k_fb_root(int L, int n_roots, const uint32_t* __restrict__ ok,
                                     const uint32_t* __restrict__ start, const uint32_t* __restrict__ cnt,
                                     const uint32_t* __restrict__ perm, const uint32_t* __restrict__ gst,
                                     const uint32_t* __restrict__ flags, const uint64_t* __restrict__ k64,
                                     const g2_aff* __restrict__ sig_aff, const fp12* __restrict__ froot,
                                     g2_jac* __restrict__ X, uint32_t* __restrict__ rtk, uint8_t* __restrict__ gv0,
                                     uint32_t* __restrict__ nfail, uint8_t* __restrict__ verdict, int n,
                                     const uint32_t* __restrict__ xok, uint32_t* __restrict__ nS, fb_jobs jobs,
                                     const g1_aff* __restrict__ pk_aff) {
  using namespace ssb::lane;
  if (*ok) return;   // uniform: the batch passed
  if (nS && blockIdx.x == 0 && threadIdx.x == 0) *nS = 0u;   // (k_fb_excl, the last reader, has finished)
  const uint32_t xv = xok ? *xok : 0u;
  if (xv == 1u) {   // the exclusion check passed: the non-suspects are valid (the suspects were checked alone)
    for (int s = blockIdx.x * 64 + threadIdx.x; s < n; s += gridDim.x * 64)
      if ((flags[s] & (FLAG_CANDIDATE | FLAG_SUSPECT)) == FLAG_CANDIDATE) verdict[s] = 1;
    return;
  }
  if (xv == 2u) {   // group-test mode: the undecided shares of every job from its relations
    for (int j = blockIdx.x * 64 + threadIdx.x; j < jobs.n_jobs; j += gridDim.x * 64)
      deduce_job(j, (uint32_t)n, jobs, (uint32_t*)flags, verdict, sig_aff, pk_aff);
    return;
  }
  const int r = blockIdx.x >> 2, q = blockIdx.x & 3;
  if (r >= n_roots) return;
  const uint32_t nr = cnt[r], sb = start[r];
  if (!nr) return;   // no group (the root's four blocks all leave here: no ticket)
  __shared__ fr_lds u;
  __shared__ uint32_t flg, last;
  const int lane_ = threadIdx.x;
  const g2_jac acc = quarter_sum<fp2>(u.b, perm + sb, nr, flags, FLAG_CANDIDATE, k64, sig_aff, q);
  if (lane_ == 0) X[4 * r + q] = acc;
  __threadfence();
  __syncthreads();
  if (lane_ == 0) last = atomicAdd(&rtk[r], 1u) == 3u ? 1u : 0u;
  __syncthreads();
  if (!last) return;
  __threadfence();
  const bool pass = root_check(u, flg, X + 4 * r, froot + r);
  if (lane_ == 0) {
    gv0[gst[r]] = pass ? 1 : 0;
    if (!pass) atomicAdd(nfail, nr);   // shares in failing roots
    rtk[r] = 0u;
  }
  if (pass || L == 1)   // (L == 1: level 0 is the single-share level)
    for (uint32_t k = sb + lane_; k < sb + nr; k += 64) {
      const uint32_t s = perm[k];
      if (flags[s] & FLAG_CANDIDATE) verdict[s] = pass ? 1 : 0;
    }
}

// The committee stage's checks (after k_fb_rlc's consistency pass listed the suspects, nS <=
// FB_SUSPECT_MAX; otherwise a no-op and the tree decides):
//   * the EXCLUSION check -- the batch check without the suspects:
//       FE( ftot * prod_r m(-E_r, H(r)) * m(g1, X) ) == 1,
//       E_r = sum_{suspects of root r} k_i pk_i = sum_q 2^16q E_{r,q}  (blocks 4r + q),
//       X   = sum_{suspects} k_i sig_i   = sum_{p,q} 2^16q X_{p,q}  (blocks 4 n_roots + 4p + q: parts p of the suspects),
//     the quarters' 4-bit-digit bucket sums, each paired on its own (ex_root_quarter, ex_quarter_point:
//     the same value after the exponentiation), where ftot is the batch check's own Miller product
//     (k_miller_final) -- by bilinearity this is the RLC check over every non-suspect candidate with
//     the batch's own scalars (soundness 2^-63), at the cost of four Miller loops per root holding
//     suspects: *xok = 1 decides them all valid;
//   * every suspect checked alone, e(pk_s, H(r)) e(-g1, sig_s) == 1, exactly the reference's verify
//     (blocks ex_pairs(n_roots) ..).
// The pair blocks finish with completion tickets (ex_pair_ticket: per root, then xtk[0]); the last
// multiplies ftot by the root products and the X values (those without suspects skipped: 1) and runs
// ONE final exponentiation.
// (the roles of k_fb_excl are out of line: each role's temporaries live in its own frame, and the
// kernel's private segment is the largest role's, not their sum)
struct ex_lds { fr_lds u; uint32_t flg, last, ncand, item; g1_aff sP; g2_aff sQ; };
SSB_FN void ex_singles(ex_lds& L, int first, uint32_t ns, const uint32_t* __restrict__ slist,
                       const uint32_t* __restrict__ share_root, const g2_aff* __restrict__ sig_aff,
                       const g1_aff* __restrict__ pk_aff, const g2_aff* __restrict__ H, uint8_t* __restrict__ verdict) {
  using namespace ssb::lane;
  const int lane_ = threadIdx.x;
  grp g{(lfp*)L.u.s, (lfp*)L.u.s + LP_NCODE_CONST, 0, 0, 0, (lu32*)&L.flg, lane_};
  const int F1 = BS_S0, B = F1 + 24, BP = B + 12, TMP = BP + 4;
  bool init = false;
  for (uint32_t x = (uint32_t)(blockIdx.x - first); x < ns; x += gridDim.x - (unsigned)first) {
    const uint32_t s = slist[x];
    if (!init) { lp_init_consts(g); init = true; }
    const bool pass = pair_check(g, pk_aff[s], sig_aff[s], H[share_root[s]], F1, B, BP, TMP);
    if (lane_ == 0) verdict[s] = pass ? 1 : 0;
  }
}
// The exclusion pairs, one block each (k_fb_excl's blocks 0 .. ex_pairs(n_roots) - 1): the Miller value
// into fex[pair], then ex_pair_ticket.  Root r's E_r and X are both split into the quarters of the
// scalars (bits 16q .. 16q+15: quarter_sum's 4-bit-digit bucket sums on the block's lanes), and X
// also into parts, P slices of the suspect list (P = ceil(nS / EX_X_SHARES) <= EX_X_PARTS):
//   block 4r + q                  m(-[2^16q] E_{r,q}, H(r))        (ex_root_quarter),
//   block 4 n_roots + 4p + q      m([2^16q] g1, X_{p,q})           (ex_quarter_point; p >= P: 1),
// whose product is m(-E_r, H(r)), resp. m(g1, X), after the final exponentiation.  No block runs a
// 64-bit scalar product on one lane (the one-invalid batch's chain, round-5 trace: the root pair
// holding its suspect ended at 6.9 ms, the X quarters at 2.8 ms), nor a bucket sum over hundreds of
// suspects (1e-2 invalid: ~650 suspects, the four X quarter sums ended at 4.3-6.2 ms).  Each role
// ends with the pair's points in L.sP / L.sQ and the block synchronised (the bucket lists dead),
// then ex_pair_lds.
// (roles out of line, called one after the other from the kernel: the quarter sum's frame and the
// Miller loop's are never on the call chain together)
SSB_FN void ex_root_quarter(ex_lds& L, int r, int q, const uint32_t* __restrict__ start, const uint32_t* __restrict__ cnt,
                            const uint32_t* __restrict__ perm, const uint32_t* __restrict__ flags,
                            const uint64_t* __restrict__ k64, const g1_aff* __restrict__ pk_aff,
                            const g2_aff* __restrict__ H) {
  const uint32_t* list = perm + start[r];
  const uint32_t nr = cnt[r];
  bool any = false;
  for (uint32_t x = threadIdx.x; x < nr; x += 64) any |= (flags[list[x]] & FLAG_SUSPECT) != 0u;
  if (!__syncthreads_or(any ? 1 : 0)) {   // uniform: no suspect in the root -- m(O, H(r)) = 1
    if (threadIdx.x == 0) { g1_aff P; P.inf = true; L.sP = P; L.sQ = H[r]; }
    __syncthreads();
    return;
  }
  const g1_jac a = quarter_sum<fp>(L.u.b, list, nr, flags, FLAG_SUSPECT, k64, pk_aff, q);
  if (threadIdx.x == 0) {
    g1_jac t = a;
    for (int i = 0; i < 16 * q; ++i) jac_dbl_inl(t, t);   // (infinity stays infinity: Z = 0)
    g1_aff P;
    jac_to_aff(P, t);
    if (!P.inf) fp_neg(P.y, P.y);   // -[2^16q] E_{r,q}
    L.sP = P;
    L.sQ = H[r];
  }
  __syncthreads();
}
// X's quarter q (ex_quarter_point, then ex_pair_lds): X_q = sum over the suspects of (bits 16q .. 16q+15 of k_i) sig_i, paired with
// [2^16q] g1 -- m(g1, X) is replaced by the product of the four m([2^16q] g1, X_q), equal after the
// final exponentiation (X = sum_q 2^16q X_q).  Each quarter's block runs its own Miller loop: no
// block waits for the other quarters, and the 48 doublings that combined them on one lane (with an
// inversion and the combined Miller loop after them: the one-invalid batch's exclusion chain, 7.6 of
// its 9.4 ms, round-5 trace) leave the critical path.
// (two functions called one after the other from the kernel: the quarter sum's frame and the Miller
// loop's are never on the call chain together)
// (the quarter sum stored by quarter_sum_to, then its affine form and the pair's G1 point into LDS)
SSB_FN void ex_quarter_point(ex_lds& L, int q, const g2_jac* __restrict__ Xq, const g1_aff* __restrict__ negg1_pow) {
  if (threadIdx.x == 0) {
    g2_aff Q;
    { const g2_jac x = *Xq; jac_to_aff(Q, x); }
    L.sQ = Q;
    g1_aff P = negg1_pow[16 * q];
    fp_neg(P.y, P.y);   // [2^16q] g1
    L.sP = P;
  }
}
SSB_FN void ex_pair_lds(ex_lds& L) {
  using namespace ssb::lane;
  grp g{(lfp*)L.u.s, (lfp*)L.u.s + LP_NCODE_CONST, 0, 0, 0, (lu32*)&L.flg, (int)threadIdx.x};
  const int F1 = BS_S0, B = F1 + 24;
  lp_init_consts(g);
  miller_one(g, L.sP, L.sQ, F1, B, L.flg);
}
// ACC *= prod of fex[first + k * stride] (k < count), the values equal to 1 skipped (a quarter without
// suspects contributed m(O, Q) = 1).  Lane i tests value k = base + i, a ballot lists the others;
// every product is a lane-program Fp12 product on this block.
SSB_FN void ex_mul_values(lane::grp& g, const fp12* __restrict__ fex, int first, int count, int stride, int ACC, int IN) {
  using namespace ssb::lane;
  const int lane_ = threadIdx.x;
  const fp one = fp_one();
  for (int base = 0; base < count; base += 64) {
    bool keep = false;
    if (base + lane_ < count) {
      const fp* v = (const fp*)&fex[first + (base + lane_) * stride];
      keep = !fp_eq(v[0], one);
      for (int k = 1; k < 12 && !keep; ++k) keep = !fp_is_zero(v[k]);
    }
    for (uint64_t m = __ballot(keep); m; m &= m - 1) {   // uniform
      const int i = first + (base + __builtin_ctzll(m)) * stride;
      if (lane_ < 12) lp_put(g.s + IN + lane_, lv_in(((const fp*)&fex[i])[lane_]));
      __syncthreads();
      f12_mul(g, ACC, IN, ACC);
    }
  }
}
// The pair's Miller value into fex[pair], then the tickets: a root's four quarter blocks first meet on
// rtk[r] (zeroed by fb_prep_block, zeroed again here for k_fb_root), the last multiplies the four
// values into fex[4r]; the root products and the X blocks then meet on xtk[0] -- true in the block
// that runs the final product.  (ex_final then multiplies n_roots + 4 EX_X_PARTS values, not every
// quarter's: with 1e-2 invalid shares ~60 of 64 roots hold suspects.)
SSB_FN bool ex_pair_ticket(ex_lds& L, int n_roots, int pair, fp12* __restrict__ fex, uint32_t* __restrict__ xtk,
                           uint32_t* __restrict__ rtk) {
  using namespace ssb::lane;
  const int lane_ = threadIdx.x;
  if (lane_ < 12) ((fp*)&fex[pair])[lane_] = lane::slot_out(L.u.s[LP_NCODE_CONST + BS_S0 + lane_]);   // (g.s + F1 of the roles)
  __threadfence();
  __syncthreads();
  if (pair < 4 * n_roots) {   // uniform
    const int r = pair >> 2;
    if (lane_ == 0) L.last = atomicAdd(&rtk[r], 1u) == 3u ? 1u : 0u;
    __syncthreads();
    if (!L.last) return false;
    __threadfence();
    grp g{(lfp*)L.u.s, (lfp*)L.u.s + LP_NCODE_CONST, 0, 0, 0, (lu32*)&L.flg, lane_};
    const int ACC = BS_S0, IN = BS_S0 + 12;
    if (lane_ < 12) lp_put(g.s + ACC + lane_, lane_ == 0 ? lv_one() : lv_zero());
    __syncthreads();
    ex_mul_values(g, fex, 4 * r, 4, 1, ACC, IN);
    if (lane_ < 12) ((fp*)&fex[4 * r])[lane_] = lv_out(lp_get(g.s + ACC + lane_));
    if (lane_ == 0) rtk[r] = 0u;
    __threadfence();
    __syncthreads();
  }
  if (lane_ == 0) L.last = atomicAdd(&xtk[0], 1u) == (uint32_t)(n_roots + 4 * launch::EX_X_PARTS - 1) ? 1u : 0u;
  __syncthreads();
  return L.last != 0;
}
// ftot * prod of the exclusion values (the root products fex[4r], the X blocks'), ONE final
// exponentiation -> *xok
SSB_FN void ex_final(ex_lds& L, int n_roots, const fp12* __restrict__ ftot, const fp12* __restrict__ fex,
                     uint32_t* __restrict__ xtk, uint32_t* __restrict__ xok) {
  using namespace ssb::lane;
  const int lane_ = threadIdx.x;
  __threadfence();
  grp g{(lfp*)L.u.s, (lfp*)L.u.s + LP_NCODE_CONST, 0, 0, 0, (lu32*)&L.flg, lane_};
  const int F1 = BS_S0, B = F1 + 24, BP = B + 12, TMP = BP + 4;
  const int ACC = F1, IN = F1 + 12;
  if (lane_ < 12) lp_put(g.s + ACC + lane_, lv_in(((const fp*)ftot)[lane_]));
  __syncthreads();
  ex_mul_values(g, fex, 0, n_roots, 4, ACC, IN);
  ex_mul_values(g, fex, 4 * n_roots, 4 * launch::EX_X_PARTS, 1, ACC, IN);
  f12_final_exp(g, ACC, TMP);
  const bool pass = f12_slots_one(g, ACC);
  if (lane_ == 0) { *xok = pass ? 1u : 0u; xtk[0] = 0u; }
}

// GROUP-TEST mode of the committee stage (more suspects than FB_SUSPECT_MAX,
// e.g. a faulty operator in every committee): one RLC check per (root, operator-id bucket) group of
// candidates with the batch's own scalars,
//     e(S1, H(r)) * e(-g1, S2) == 1,   S1 = sum k_i pk_i,   S2 = sum k_i sig_i  over the group,
// a passing group decides its candidates valid (soundness 2^-63), a one-candidate group is exactly that
// share's verify.  Items (key, q), the layout of k_fb_root: item q sums quarter q of the scalars
// (bits 16q .. 16q+15) of both sums into gX2 / gX1 (the tree's per-share product buffers, unused in
// this mode: sized for 4 fb_keys entries); the last of the key's four items -- ticket: the scatter's
// cursor, which fb_prep_block left at kstart + kcnt -- combines the quarters and runs the check.
// k_fb_root then deduces the rest of every job from its committee relations (deduce_job) and
// k_fb_single checks what is left.  (Run by k_fb_excl's blocks in that mode: one launch less in
// every failed batch's chain -- a launch that leaves at once still waits for a free wave slot
// behind the other pipeline slots' waves.)
// (the group tests' roles out of line: the quarter sums' and the combines' point temporaries live in
// their own frames, not in the kernel's beside the pairing check's)
// the last item of a group: its quarters combined into L.sQ / L.sP (lane 0), then (ex_group_check)
// ONE RLC check and the candidates' verdicts on a pass (or for a one-candidate group).  Two functions
// called one after the other from the kernel: the combines' frame and the pairing check's frame are
// never on the call chain together (private segment: the deeper of the two, not their sum).
// sum_q 2^(16q) X[q] by Horner (16 doublings and an addition per quarter) as lane programs: every
// group of the wave runs the same operation on the same values in the same slots (one wave in
// lockstep: identical stores), so the 48-doubling chain costs 48 programs, not 48 one-lane
// doublings (round-5 trace of the faulty-operator batch: the one-lane combine took 3.2 ms of every
// group's 9 ms chain).  Result in slots ACC (Jacobian); returns the additions' exception flags
// (an infinite quarter, equal or opposite partial sums: the caller's one-lane combine then).
SSB_FN uint32_t gc_horner_g2(ex_lds& L, const g2_jac* __restrict__ X, int ACC, int TMP) {
  using namespace ssb::lane;
  const int role = threadIdx.x % G2_ADD_G;
  grp g{(lfp*)L.u.s, (lfp*)L.u.s + LP_NCODE_CONST, 0, 0, 0, (lu32*)&L.flg, role};
  uint32_t exc = 0;
  if (role < 6) lp_put(g.s + ACC + role, lv_in(((const fp*)&X[3])[role]));
  __syncthreads();
  for (int q = 2; q >= 0; --q) {
    for (int i = 0; i < 16; ++i) g2_dbl(g, ACC, ACC);
    if (role < 6) lp_put(g.s + TMP + role, lv_in(((const fp*)&X[q])[role]));
    __syncthreads();
    g2_add(g, ACC, TMP, ACC, exc);
  }
  return exc;
}
SSB_FN uint32_t gc_horner_g1(ex_lds& L, const g1_jac* __restrict__ X, int ACC, int TMP) {
  using namespace ssb::lane;
  const int role = threadIdx.x % G1_ADD_G;
  grp g{(lfp*)L.u.s, (lfp*)L.u.s + LP_NCODE_CONST, 0, 0, 0, (lu32*)&L.flg, role};
  uint32_t exc = 0;
  if (role < 3) lp_put(g.s + ACC + role, lv_in(((const fp*)&X[3])[role]));
  __syncthreads();
  for (int q = 2; q >= 0; --q) {
    for (int i = 0; i < 16; ++i) g1_dbl(g, ACC, ACC);
    if (role < 3) lp_put(g.s + TMP + role, lv_in(((const fp*)&X[q])[role]));
    __syncthreads();
    g1_add(g, ACC, TMP, ACC, exc);
  }
  return exc;
}
// the lane programs' Jacobian result (slots S0 ..) to affine in L.sQ / L.sP (lane 0), or the one-lane
// combine after an exception -- each step out of line, so group_combine's frame holds no point
SSB_FN void gc_store_g2(ex_lds& L, int S0) {
  if (threadIdx.x != 0) return;
  g2_jac R;
  for (int k = 0; k < 6; ++k) ((fp*)&R)[k] = lane::slot_out(L.u.s[lane::LP_NCODE_CONST + S0 + k]);
  g2_aff Q;
  jac_to_aff(Q, R);
  L.sQ = Q;
}
SSB_FN void gc_store_g1(ex_lds& L, int S0) {
  if (threadIdx.x != 0) return;
  g1_jac R;
  for (int k = 0; k < 3; ++k) ((fp*)&R)[k] = lane::slot_out(L.u.s[lane::LP_NCODE_CONST + S0 + k]);
  g1_aff P;
  jac_to_aff(P, R);
  L.sP = P;
}
SSB_FN void gc_exact_g2(ex_lds& L, const g2_jac* __restrict__ X2) {
  const g2_aff Q = combine_quarters<fp2>(X2);
  if (threadIdx.x == 0) L.sQ = Q;
}
SSB_FN void gc_exact_g1(ex_lds& L, const g1_jac* __restrict__ X1) {
  const g1_aff P = combine_quarters<fp>(X1);
  if (threadIdx.x == 0) L.sP = P;
}
SSB_FN void group_combine(ex_lds& L, const g2_jac* __restrict__ X2, const g1_jac* __restrict__ X1) {
  using namespace ssb::lane;
  constexpr int S0 = lane::G2_ADD_SCRATCH > lane::G1_ADD_SCRATCH ? lane::G2_ADD_SCRATCH : lane::G1_ADD_SCRATCH;
  static_assert(S0 >= lane::G2_DBL_SCRATCH && S0 >= lane::G1_DBL_SCRATCH && S0 + 12 <= BS_SLOTS, "slots");
  {
    grp g{(lfp*)L.u.s, (lfp*)L.u.s + LP_NCODE_CONST, 0, 0, 0, (lu32*)&L.flg, (int)threadIdx.x};
    lp_init_consts(g);
    __syncthreads();
  }
  if (gc_horner_g2(L, X2, S0, S0 + 6)) gc_exact_g2(L, X2);   // uniform (every lane reads the one flag word)
  else gc_store_g2(L, S0);
  __syncthreads();
  if (gc_horner_g1(L, X1, S0, S0 + 3)) gc_exact_g1(L, X1);
  else gc_store_g1(L, S0);
}
SSB_FN void ex_group_check(ex_lds& L, const uint32_t* __restrict__ list, uint32_t gn, uint32_t m,
                           uint32_t* __restrict__ flags, const g2_aff& h, uint8_t* __restrict__ verdict) {
  using namespace ssb::lane;
  const int lane_ = threadIdx.x;
  grp g{(lfp*)L.u.s, (lfp*)L.u.s + LP_NCODE_CONST, 0, 0, 0, (lu32*)&L.flg, lane_};
  lp_init_consts(g);
  const int F1 = BS_S0, B = F1 + 24, BP = B + 12, TMP = BP + 4;
  const bool pass = pair_check(g, L.sP, L.sQ, h, F1, B, BP, TMP);   // (the points read from LDS)
  if (pass || m == 1)
    for (uint32_t x = lane_; x < gn; x += 64) {
      const uint32_t s = list[x];
      if (!(flags[s] & FLAG_CANDIDATE)) continue;
      verdict[s] = pass ? 1 : 0;
      atomicOr(&flags[s], (uint32_t)FLAG_DECIDED);
    }
  __syncthreads();
}
// The committee stage's checks, after k_fb_rlc's consistency pass listed the suspects (nS of them):
//   nS <= FB_SUSPECT_MAX -- the EXCLUSION check, the batch check without the suspects:
//       FE( ftot * prod_r m(-E_r, H(r)) * m(g1, X) ) == 1,
//       E_r and X split into the quarters of the scalars, one pair block per quarter (blocks 4r + q,
//       then 4 n_roots + 4p + q for the parts of X: see ex_root_quarter), ftot the batch check's own Miller product
//       (k_miller_final) -- by bilinearity the RLC check over every non-suspect candidate with the
//       batch's own scalars (soundness 2^-63): *xok = 1 decides them all valid;
//     and every suspect checked alone, e(pk_s, H(r)) e(-g1, sig_s) == 1, exactly the reference's
//     verify (blocks ex_pairs(n_roots) ..).  The pair blocks finish with a completion ticket (xtk[0]); the
//     last pair runs the product and ONE final exponentiation;
//   nS > FB_SUSPECT_MAX -- GROUP-TEST mode (e.g. a faulty operator in every committee): *xok = 2, and
//     the blocks run one RLC check per (root, operator-id bucket) group of candidates, k_fb_root
//     deduces the rest from the committee relations (deduce_job), k_fb_single checks what is left;
//   nS == 0 (no relation broken: the invalid shares sit in jobs without redundancy) -- *xok = 0, the tree.
__global__ void SSB_LB2(64) k_fb_excl(int n_roots, const uint32_t* __restrict__ ok, const uint32_t* __restrict__ nS,
                                     const uint32_t* __restrict__ slist, const uint32_t* __restrict__ start,
                                     const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ perm,
                                     uint32_t* __restrict__ flags, const uint32_t* __restrict__ share_root,
                                     const uint64_t* __restrict__ k64, const g2_aff* __restrict__ sig_aff,
                                     const g1_aff* __restrict__ pk_aff, const g2_aff* __restrict__ H,
                                     const fp12* __restrict__ ftot, fp12* __restrict__ fex, g2_jac* __restrict__ X4,
                                     uint32_t* __restrict__ xtk, uint32_t* __restrict__ xok, uint8_t* __restrict__ verdict,
                                     const uint32_t* __restrict__ kcnt, const uint32_t* __restrict__ kstart,
                                     uint32_t* __restrict__ cursor, g2_jac* __restrict__ gX2, g1_jac* __restrict__ gX1,
                                     const g1_aff* __restrict__ negg1_pow, uint32_t* __restrict__ rtk,
                                     const uint32_t* __restrict__ klist) {
  if (*ok) return;   // uniform: the batch passed
  SSB_TRACE_T0();
  const uint32_t ns = *nS;
  const int blk = blockIdx.x, lane_ = threadIdx.x;
  const bool gmode = ns > FB_SUSPECT_MAX && kcnt && klist;
  if (ns == 0 || (ns > FB_SUSPECT_MAX && !gmode)) {   // nothing to exclude / no group keys: the tree decides
    if (blk == 0 && lane_ == 0) *xok = 0u;
    return;
  }
  __shared__ ex_lds L;
  if (gmode) {   // group-test mode: blocks take (key, quarter) items from a counter
    if (blk == 0 && lane_ == 0) *xok = 2u;
    const uint32_t NB = (uint32_t)launch::fb_nbuckets(n_roots);
    // four items per non-empty key (klist: fb_prep_block), handed out in order by an item counter
    // (xtk[1], zeroed by fb_prep_block in k_fb_rlc, the previous launch on the stream): a block that
    // finishes an item takes the next one, so a block busy with a key's combine and check holds up no
    // items, and a key's four quarters run on four blocks at once.  (Static strides: over all n_roots x
    // NB keys in key order a quarter of the blocks got every busy item, 30.9 ms against a 7 ms median;
    // over the non-empty keys 14.2 ms, round-5 traces.)  The item index travels from lane 0 to the
    // wave through LDS (L.item, outside the union the item's bucket lists reuse), and is checked
    // against `items` before any item-indexed access; the counter overshoots by one fetch per block,
    // harmlessly (nothing reads it past `items`).
    const uint32_t items = 4u * klist[n_roots * NB];
    uint32_t* ictr = xtk + 1;
    for (;;) {
      if (lane_ == 0) L.item = atomicAdd(ictr, 1u);
      __syncthreads();
      const uint32_t it = __builtin_amdgcn_readfirstlane(L.item);
      __syncthreads();   // (every lane has read L.item before lane 0 writes the next)
      if (it >= items) break;   // uniform
      const uint32_t key = klist[it >> 2], q = it & 3;
#ifdef SSB_FB_CHECKS
      if (key >= (uint32_t)n_roots * NB || (it >> 2) >= klist[n_roots * NB]) {
        if (lane_ == 0) printf("[fb-check] k_fb_excl block %u: item %u of %u -> key %u (keys %u)\n", blockIdx.x, it, items,
                               key, (uint32_t)n_roots * NB);
        break;
      }
#endif
      const uint32_t gn = kcnt[key];
      if (!gn) continue;   // (uniform: the four items of an empty key all skip: no ticket)
      const uint32_t* list = perm + kstart[key];
      quarter_sum_to<fp2>(L.u.b, list, gn, flags, FLAG_CANDIDATE, k64, sig_aff, (int)q, gX2 + 4 * key + q);
      quarter_sum_to<fp>(L.u.b, list, gn, flags, FLAG_CANDIDATE, k64, pk_aff, (int)q, gX1 + 4 * key + q);
#ifndef SSB_TRACE_NO_LOOP   // (experiment: the fault bisection of round 6)
      SSB_TRACE(TR_EX_ITEM);
#endif
      __threadfence();
      __syncthreads();
      if (lane_ == 0) L.last = atomicAdd(&cursor[key], 1u) == kstart[key] + gn + 3u ? 1u : 0u;
      __syncthreads();
      if (!L.last) continue;
      __threadfence();
      if (lane_ == 0) L.ncand = 0u;
      __syncthreads();
      uint32_t nc = 0;
      for (uint32_t x = lane_; x < gn; x += 64) nc += (flags[list[x]] & FLAG_CANDIDATE) ? 1u : 0u;
      if (nc) atomicAdd(&L.ncand, nc);
      __syncthreads();
      const uint32_t m = L.ncand;
      if (!m) continue;   // uniform
      group_combine(L, gX2 + 4 * key, gX1 + 4 * key);
      __syncthreads();   // (the bucket lists are dead: the LDS becomes the lane programs' slots)
#ifndef SSB_TRACE_NO_LOOP   // (experiment: the fault bisection of round 6)
      SSB_TRACE(TR_EX_GCOMB);
#endif
      ex_group_check(L, list, gn, m, flags, H[key / NB], verdict);
#ifndef SSB_TRACE_NO_LOOP   // (experiment: the fault bisection of round 6)
      SSB_TRACE(TR_EX_GCHECK);
#endif
    }
    return;
  }
  const int npairs = launch::ex_pairs(n_roots);
  if (blk >= npairs) {   // the suspects, one pairing check each
    ex_singles(L, npairs, ns, slist, share_root, sig_aff, pk_aff, H, verdict);
    SSB_TRACE(TR_EX_SINGLE);
    return;
  }
  if (blk < 4 * n_roots) {
    ex_root_quarter(L, blk >> 2, blk & 3, start, cnt, perm, flags, k64, pk_aff, H);
    ex_pair_lds(L);
    SSB_TRACE(TR_EX_ROOTPAIR);
  } else {
    const int x = blk - 4 * n_roots, q = x & 3, part = x >> 2;
    const uint32_t P = (ns + EX_X_SHARES - 1) / EX_X_SHARES, per = (ns + P - 1) / P;   // (ns >= 1)
    const uint32_t b0 = (uint32_t)part * per;
    if ((uint32_t)part < P && b0 < ns) {   // uniform
      quarter_sum_to<fp2>(L.u.b, slist + b0, ns - b0 < per ? ns - b0 : per, flags, FLAG_SUSPECT, k64, sig_aff, q, X4 + x);
      SSB_TRACE(TR_EX_QSUM);
      ex_quarter_point(L, q, X4 + x, negg1_pow);   // (lane 0 wrote X4[x] and reads it back)
    } else if (lane_ == 0) {
      g1_aff P0; P0.inf = true; L.sP = P0;   // (no part: m(O, .) = 1)
    }
    __syncthreads();   // (the bucket lists are dead: the LDS becomes the lane programs' slots)
    ex_pair_lds(L);
    SSB_TRACE(TR_EX_PAIR);
  }
  if (ex_pair_ticket(L, n_roots, blk, fex, xtk, rtk)) {
    ex_final(L, n_roots, ftot, fex, xtk, xok);
    SSB_TRACE(TR_EX_FINAL);
  }
}

// Few shares in failing roots (<= FB_SINGLE_MAX after level 0): each of them checked alone,
// e(pk_s, H(r)) * e(-g1, sig_s) == 1 -- exactly the reference's verify, no RLC scalar, no per-share
// products, one pairing check deep instead of the products + the levels below the root.  Blocks
// stride over the root-sorted order (a failing root's shares are contiguous there: one per block).
__global__ void SSB_LB(64) k_fb_single(int n_roots, const uint32_t* __restrict__ ok, const uint32_t* __restrict__ nfail,
                                      const uint32_t* __restrict__ start, const uint32_t* __restrict__ cnt,
                                      const uint32_t* __restrict__ perm, const uint32_t* __restrict__ gst0,
                                      const uint8_t* __restrict__ gv0, const uint32_t* __restrict__ flags,
                                      const uint32_t* __restrict__ share_root, const g2_aff* __restrict__ H,
                                      const g2_aff* __restrict__ sig_aff, const g1_aff* __restrict__ pk_aff,
                                      uint8_t* __restrict__ verdict, const uint32_t* __restrict__ xok, int n,
                                      const uint64_t* __restrict__ k64, g2_jac* __restrict__ rsig, g1_jac* __restrict__ rpk) {
  using namespace ssb::lane;
  if (*ok) return;   // uniform
  const uint32_t xv = xok ? *xok : 0u;
  if (xv == 1u) return;   // the exclusion check decided the batch
  if (xv == 0u && *nfail > FB_SINGLE_MAX) {   // the tree's per-share products instead (one launch for both)
    for (int g = (int)(blockIdx.x * 64 + threadIdx.x); g < 2 * n; g += (int)(gridDim.x * 64))
      sparse_product(g, n, n_roots, flags, share_root, gst0, gv0, k64, sig_aff, pk_aff, rsig, rpk);
    return;
  }
  // (xv == 2: group-test mode's leftovers)
  __shared__ lslot lds[LP_NCODE_CONST + BS_SLOTS];
  __shared__ uint32_t flg;
  const int lane_ = threadIdx.x;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST, 0, 0, 0, (lu32*)&flg, lane_};
  bool init = false;
  const int F1 = BS_S0, B = F1 + 24, BP = B + 12, TMP = BP + 4;
  const uint32_t total = start[n_roots - 1] + cnt[n_roots - 1];
  for (uint32_t x = blockIdx.x; x < total; x += gridDim.x) {
    const uint32_t s = perm[x];
    const uint32_t r = share_root[s];
    if (!(flags[s] & FLAG_CANDIDATE)) continue;
    if (xv == 2u ? (flags[s] & FLAG_DECIDED) != 0 : gv0[gst0[r]] != 0) continue;
    if (!init) { lp_init_consts(g); init = true; }
    const bool pass = pair_check(g, pk_aff[s], sig_aff[s], H[r], F1, B, BP, TMP);
    if (lane_ == 0) verdict[s] = pass ? 1 : 0;
  }
}

// One level of the group tree.  Workgroups (one wave) stride over the level's groups (control
// flow uniform per group): sums of the group's k_i pk_i and k_i sig_i (lane-strided, LDS tree),
// affine, then ONE two-pair lane-program Miller loop (f12_miller2: e(S_pk, H(r)) and e(-g1, S_sig)
// share the squarings of f; 1.33 single loops of latency instead of 2), final exponentiation.  (A
// two-wave variant running the two loops on two waves halved the resident workgroups and measured
// slower.)
// gv_prev / gv_cur: per-group results of the previous / this level (1 pass, 0 fail).
constexpr int LV_THREADS = 64;
// the group's sums S_sig = sum k_i sig_i, S_pk = sum k_i pk_i over its candidates [a, b) of perm (lane-
// strided, LDS tree), affine into *sQ / *sP, the candidate count into *ncand; out of line, so the
// points it holds are not in the kernel's frame under the pairing check's chain
SSB_FN void level_group_sums(uint64_t a, uint64_t b, const uint32_t* __restrict__ perm, const uint32_t* __restrict__ flags,
                             const g2_jac* __restrict__ rsig, const g1_jac* __restrict__ rpk, g2_jac* red, g1_aff* sP,
                             g2_aff* sQ, uint32_t* ncand) {
  const int lane_ = threadIdx.x;
  if (lane_ == 0) *ncand = 0u;
  __syncthreads();
  g2_jac acc2; jac_set_inf(acc2);
  g1_jac acc1; jac_set_inf(acc1);
  uint32_t nc = 0;
  for (uint64_t k = a + lane_; k < b; k += 64) {
    const uint32_t s = perm[k];
    if (flags[s] & FLAG_CANDIDATE) { jac_add(acc2, acc2, rsig[s]); jac_add(acc1, acc1, rpk[s]); ++nc; }
  }
  if (nc) atomicAdd(ncand, nc);
  red[lane_] = acc2;
  __syncthreads();
  for (int w = 32; w > 0; w >>= 1) {
    if (lane_ < w) { g2_jac o = red[lane_ + w]; jac_add(acc2, acc2, o); red[lane_] = acc2; }
    __syncthreads();
  }
  if (lane_ == 0) { g2_aff q; jac_to_aff(q, acc2); *sQ = q; }
  __syncthreads();
  g1_jac* red1 = (g1_jac*)red;
  red1[lane_] = acc1;
  __syncthreads();
  for (int w = 32; w > 0; w >>= 1) {
    if (lane_ < w) { g1_jac o = red1[lane_ + w]; jac_add(acc1, acc1, o); red1[lane_] = acc1; }
    __syncthreads();
  }
  if (lane_ == 0) { g1_aff p; jac_to_aff(p, acc1); *sP = p; }
  __syncthreads();
}
// (the group sums and the two-pair loop do not fit 256 registers: one wave per SIMD, whatever the
// TU asks -- a waves_per_eu(1) attribute here would lift the shared out-of-line callees to 512 for
// every kernel of the TU)
__global__ void SSB_LB(LV_THREADS) k_fb_level(int l, int L, int lb, int n_roots, const uint32_t* __restrict__ ok,
                                              const uint32_t* __restrict__ start, const uint32_t* __restrict__ cnt,
                                              const uint32_t* __restrict__ perm, const uint32_t* __restrict__ gst,
                                              const uint32_t* __restrict__ flags, const g2_jac* __restrict__ rsig,
                                              const g1_jac* __restrict__ rpk, const g2_aff* __restrict__ H,
                                              const uint8_t* __restrict__ gv_prev, uint8_t* __restrict__ gv_cur,
                                              uint8_t* __restrict__ verdict, const uint32_t* __restrict__ nfail,
                                              const uint32_t* __restrict__ xok) {
  using namespace ssb::lane;
  if (*ok || (xok && *xok)) return;  // uniform: the batch passed / the committee stage decided it
  if (*nfail <= FB_SINGLE_MAX) return;   // (level 0 ran in k_fb_root; k_fb_single decides the few shares of failing roots)
  __shared__ lslot lds[LP_NCODE_CONST + BS_SLOTS];
  __shared__ g2_jac red[64];
  __shared__ g1_aff sP;
  __shared__ g2_aff sQ;
  __shared__ uint32_t flg, ncand;
  const int lane_ = threadIdx.x;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST, 0, 0, 0, (lu32*)&flg, lane_};
  lp_init_consts(g);
  const int F1 = BS_S0, B = F1 + 24, BP = B + 12, TMP = BP + 4;
  const uint32_t lg = (uint32_t)(lb * (L - 1 - l));
  const uint64_t Gs = 1ull << lg;
  const uint32_t* gl = gst + (size_t)l * (n_roots + 1);
  const uint32_t ngroups = gl[n_roots];
  for (uint32_t gid = blockIdx.x; gid < ngroups; gid += gridDim.x) {
    // root of the group: the last r with gl[r] <= gid
    int lo = 0, hi = n_roots;                  // invariant: gl[lo] <= gid < gl[hi]
    while (hi - lo > 1) { const int m = (lo + hi) >> 1; if (gl[m] <= gid) lo = m; else hi = m; }
    const int r = lo;
    const uint32_t j = gid - gl[r];
    const uint64_t seg_b = start[r], seg_e = seg_b + cnt[r];
    const uint64_t a = seg_b + (uint64_t)j * Gs, b = a + Gs < seg_e ? a + Gs : seg_e;
    if (l > 0) {
      const uint32_t* gp = gst + (size_t)(l - 1) * (n_roots + 1);
      const uint8_t pv = gv_prev[gp[r] + (j >> lb)];
      if (pv) { if (lane_ == 0) gv_cur[gid] = 1; continue; }   // parent passed: verdicts written
      // parent range [seg_b + (j/B) B Gs, + B Gs) equals [a, b): inherit the failure untested
      const uint64_t pa = seg_b + (uint64_t)(j >> lb) * (Gs << lb);
      const uint64_t pb = pa + (Gs << lb) < seg_e ? pa + (Gs << lb) : seg_e;
      if (pa == a && pb == b) {
        if (lane_ == 0) gv_cur[gid] = 0;
        if (lg == 0)
          for (uint64_t k = a + lane_; k < b; k += 64) { const uint32_t s = perm[k]; if (flags[s] & FLAG_CANDIDATE) verdict[s] = 0; }
        continue;
      }
    }
    level_group_sums(a, b, perm, flags, rsig, rpk, red, &sP, &sQ, &ncand);
    const bool pass = ncand ? pair_check(g, sP, sQ, H[r], F1, B, BP, TMP) : true;
    if (lane_ == 0) gv_cur[gid] = pass ? 1 : 0;
    if (pass || lg == 0)
      for (uint64_t k = a + lane_; k < b; k += 64) {
        const uint32_t s = perm[k];
        if (flags[s] & FLAG_CANDIDATE) verdict[s] = pass ? 1 : 0;
      }
    __syncthreads();
  }
}

}  // namespace k

namespace launch {

// log2 of the tree's branching factor: 16-ary (round 1 measured 16 against 4: one invalid share per
// C2 batch costs 3 tested levels instead of 5)
int fallback_log2_branch() { return 4; }
int fallback_levels(size_t n) {
  const int lb = fallback_log2_branch();
  int L = 1;
  uint64_t gs = 1;
  while (gs < n) { gs <<= lb; ++L; }
  return L;
}

void fallback_bisect(hipStream_t st, int n, int n_roots, const rlc_key& key, const uint32_t* ok, uint32_t* flags,
                     const uint32_t* share_root, const g2_aff* H, const g2_aff* sig, const g1_aff* pk, const fp12* froot,
                     const fb_ws& fw, uint8_t* verdict, bool fast_verdicts, const fb_jobs& jobs) {
  using namespace ssb::k;
  if (n <= 0 || n_roots <= 0) return;
  auto nb = [](size_t x, unsigned b) { return (unsigned)((x + b - 1) / b); };
  const int L = fallback_levels((size_t)n);
  const int lb = fallback_log2_branch();
  // the committee stage needs the jobs, the batch check's Miller product and the stage's workspace
  const bool committee = jobs.n_jobs > 0 && fw.slist && fw.nS && fw.xtk && fw.xok && fw.fex && fw.ftot && fw.kcnt &&
                         fw.kstart;
  const fb_jobs cj = committee ? jobs : fb_jobs{0, nullptr, nullptr, nullptr};
  const uint32_t* xok = committee ? fw.xok : nullptr;
  const fb_prep_args prep{n_roots, L, lb, share_root, fw.cnt, fw.start, fw.cursor, fw.gst, fw.perm, fw.rtk, fw.nfail,
                          committee ? jobs.ids : nullptr, committee ? fw.kcnt : nullptr, committee ? fw.kstart : nullptr,
                          committee ? fw.klist : nullptr, committee ? fw.xtk + 1 : nullptr};
  hipLaunchKernelGGL(k_fb_rlc, dim3(nb((size_t)n, 64) + nb((size_t)cj.n_jobs, 64) + 1), dim3(64), 0, st, n, key, ok, flags,
                     fw.k64, fast_verdicts ? verdict : (uint8_t*)nullptr, prep, cj, sig, fw.slist, fw.nS);
  if (committee)
    hipLaunchKernelGGL(k_fb_excl, dim3((unsigned)ex_pairs(n_roots) + EX_SINGLE_BLOCKS), dim3(64), 0, st, n_roots, ok,
                       (const uint32_t*)fw.nS, (const uint32_t*)fw.slist, (const uint32_t*)fw.start, (const uint32_t*)fw.cnt,
                       (const uint32_t*)fw.perm, flags, share_root, (const uint64_t*)fw.k64, sig, pk, H,
                       fw.ftot, fw.fex, fw.X, fw.xtk, fw.xok, verdict, (const uint32_t*)fw.kcnt, (const uint32_t*)fw.kstart,
                       fw.cursor, fw.rsig, fw.rpk, fw.negg1_pow, fw.rtk, (const uint32_t*)fw.klist);
  hipLaunchKernelGGL(k_fb_root, dim3(4 * (unsigned)n_roots), dim3(64), 0, st, L, n_roots, ok, (const uint32_t*)fw.start,
                     (const uint32_t*)fw.cnt, (const uint32_t*)fw.perm, (const uint32_t*)fw.gst, (const uint32_t*)flags,
                     (const uint64_t*)fw.k64, sig, froot, fw.X, fw.rtk, fw.gv0, fw.nfail, verdict, n, xok,
                     committee ? fw.nS : (uint32_t*)nullptr, cj, pk);
  if (L == 1) return;
  {
    const unsigned grid = std::min((unsigned)n, FB_GRID_MAX);
    hipLaunchKernelGGL(k_fb_single, dim3(grid), dim3(64), 0, st, n_roots, ok, (const uint32_t*)fw.nfail,
                       (const uint32_t*)fw.start, (const uint32_t*)fw.cnt, (const uint32_t*)fw.perm, (const uint32_t*)fw.gst,
                       (const uint8_t*)fw.gv0, (const uint32_t*)flags, share_root, H, sig, pk, verdict, xok, n,
                       (const uint64_t*)fw.k64, fw.rsig, fw.rpk);
  }
  for (int l = 1; l < L; ++l) {
    const uint64_t gs = 1ull << (lb * (L - 1 - l));
    const uint64_t bound = (uint64_t)n_roots + ((uint64_t)n + gs - 1) / gs;
    const unsigned grid = (unsigned)std::min(bound, (uint64_t)FB_GRID_MAX);
    uint8_t* cur = (l & 1) ? fw.gv1 : fw.gv0;
    const uint8_t* prev = (l & 1) ? fw.gv0 : fw.gv1;
    hipLaunchKernelGGL(k_fb_level, dim3(grid), dim3(LV_THREADS), 0, st, l, L, lb, n_roots, ok, (const uint32_t*)fw.start,
                       (const uint32_t*)fw.cnt, (const uint32_t*)fw.perm, (const uint32_t*)fw.gst, (const uint32_t*)flags,
                       (const g2_jac*)fw.rsig, (const g1_jac*)fw.rpk, H, prev, cur, verdict,
                       (const uint32_t*)fw.nfail, xok);
  }
}

}  // namespace launch
}  // namespace ssb

SSB_TRACE_READER(bisect)
