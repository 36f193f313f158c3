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
// Work at 1% invalid shares (C2: 64 roots x 256): ~3.5k group checks (4-ary: ~2.1k, in 5 levels)
// instead of 16,384 per-share checks; at one invalid share, 96.  Every kernel here is a no-op (uniform early exit) when the batch passed.
#include "ssb_kernels.h"
#include "ssb_lane_ops.h"

namespace ssb {
namespace k {

// One workgroup (the last block of k_fb_rlc's grid): counting sort of the shares by root (cnt,
// start, perm) and the group starts of every level (gst[l][r], n_roots + 1 words per level).
// Phases separated by workgroup barriers (global atomics and stores of one workgroup are ordered
// by them).  (It used to be a launch of its own, k_fb_prep: one more no-op launch on every passing
// batch's tail.)
struct fb_prep_args { int n_roots, L, lb; const uint32_t* share_root; uint32_t* cnt; uint32_t* start; uint32_t* cursor;
                      uint32_t* gst; uint32_t* perm; };
SSB_INL void fb_prep_block(int n, const fb_prep_args& a) {
  const int t = threadIdx.x, NT = blockDim.x, n_roots = a.n_roots, L = a.L, lb = a.lb;
  const uint32_t* __restrict__ share_root = a.share_root;
  uint32_t* __restrict__ cnt = a.cnt;
  uint32_t* __restrict__ start = a.start;
  uint32_t* __restrict__ cursor = a.cursor;
  uint32_t* __restrict__ gst = a.gst;
  uint32_t* __restrict__ perm = a.perm;
  for (int r = t; r < n_roots; r += NT) cnt[r] = 0u;
  __syncthreads();
  for (int s = t; s < n; s += NT)
    if (share_root[s] < (uint32_t)n_roots) atomicAdd(&cnt[share_root[s]], 1u);
  __syncthreads();
  if (t == 0) {
    uint32_t acc = 0;
    for (int r = 0; r < n_roots; ++r) { start[r] = acc; cursor[r] = acc; acc += cnt[r]; }
  } else if (t <= L) {
    const int l = t - 1;
    const uint32_t lg = (uint32_t)(lb * (L - 1 - l));   // Gs_l = 2^lg
    uint32_t* g = gst + (size_t)l * (n_roots + 1);
    uint32_t acc = 0;
    for (int r = 0; r < n_roots; ++r) {
      g[r] = acc;
      acc += (uint32_t)(((uint64_t)cnt[r] + (1ull << lg) - 1) >> lg);
    }
    g[n_roots] = acc;
  }
  __syncthreads();
  for (int s = t; s < n; s += NT)
    if (share_root[s] < (uint32_t)n_roots) perm[atomicAdd(&cursor[share_root[s]], 1u)] = (uint32_t)s;
}
// threads [0, n): rsig[s] = k_s sig_s;  [n, 2n): rpk[s] = k_s pk_s  (candidates only).  With
// `verdict` it also writes, grid-wide, the verdicts the batch check decides: every share of a
// passing batch, the non-candidates of a failing one (the candidates' follow from the group tests)
// (the grid's last block runs the counting sort by root, fb_prep_block)
__global__ void SSB_LB(64) k_fb_rlc(int n, rlc_key key, const uint32_t* __restrict__ ok,
                                   const uint32_t* __restrict__ flags, const g2_aff* __restrict__ sig_aff,
                                   const g1_aff* __restrict__ pk_aff, g2_jac* __restrict__ rsig,
                                   g1_jac* __restrict__ rpk, uint8_t* __restrict__ verdict, fb_prep_args prep) {
  const uint32_t pass = *ok;
  if (blockIdx.x == gridDim.x - 1) {   // uniform per block
    if (!pass) fb_prep_block(n, prep);
    return;
  }
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (verdict && g < n) {
    const bool cand = (flags[g] & FLAG_CANDIDATE) != 0;
    if (pass || !cand) verdict[g] = cand ? 1 : 0;
  }
  if (pass) return;
  // binary double-and-add (no window table): the private segment stays small -- every tail queue
  // reserves scratch for the largest kernel it has run, and this one is launched on every batch
  if (g < n) {
    if (flags[g] & FLAG_CANDIDATE) {
      const uint64_t k = rlc_scalar_odd(key, (uint64_t)g);
      const uint32_t kw[2] = {(uint32_t)k, (uint32_t)(k >> 32)};
      g2_jac r; jac_mul_aff(r, sig_aff[g], kw, 2); rsig[g] = r;
    }
  } else if (g < 2 * n) {
    const int s = g - n;
    if (flags[s] & FLAG_CANDIDATE) {
      const uint64_t k = rlc_scalar_odd(key, (uint64_t)s);
      const uint32_t kw[2] = {(uint32_t)k, (uint32_t)(k >> 32)};
      g1_jac r; jac_mul_aff(r, pk_aff[s], kw, 2); rpk[s] = r;
    }
  }
}

constexpr int bs_max(int a, int b) { return a > b ? a : b; }
constexpr int BS_S0 = bs_max(bs_max(bs_max(lane::MILLER_ITER_SCRATCH, lane::MILLER_ADDSTEP_SCRATCH),
                                    bs_max(lane::MILLER_ITER2_SCRATCH, lane::MILLER_ADDSTEP2_SCRATCH)),
                             lane::FP12_MUL_SCRATCH);
// F: f | T1 | T2 (24), B: the pairs (12), BP: 4 work slots, TMP: the final exponentiation's 84
constexpr int BS_SLOTS = BS_S0 + 24 + 12 + 4 + 84;

// One level of the group tree.  Workgroups (one wave) stride over the level's groups (control
// flow uniform per group): sums of the group's k_i pk_i and k_i sig_i (lane-strided, LDS tree),
// affine, then ONE two-pair lane-program Miller loop (f12_miller2: e(S_pk, H(r)) and e(-g1, S_sig)
// share the squarings of f; 1.33 single loops of latency instead of 2), final exponentiation.  (A
// two-wave variant running the two loops on two waves halved the resident workgroups and measured
// slower.)
// gv_prev / gv_cur: per-group results of the previous / this level (1 pass, 0 fail).
constexpr int LV_THREADS = 64;
__global__ void SSB_LB(LV_THREADS) k_fb_level(int l, int L, int lb, int n_roots, const uint32_t* __restrict__ ok,
                                              const uint32_t* __restrict__ start, const uint32_t* __restrict__ cnt,
                                              const uint32_t* __restrict__ perm, const uint32_t* __restrict__ gst,
                                              const uint32_t* __restrict__ flags, const g2_jac* __restrict__ rsig,
                                              const g1_jac* __restrict__ rpk, const g2_aff* __restrict__ H,
                                              const uint8_t* __restrict__ gv_prev, uint8_t* __restrict__ gv_cur,
                                              uint8_t* __restrict__ verdict) {
  using namespace ssb::lane;
  if (*ok) return;  // uniform: the batch passed
  __shared__ fp lds[LP_NCODE_CONST + BS_SLOTS];
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
    // sums over the group's candidates
    if (lane_ == 0) ncand = 0u;
    __syncthreads();
    g2_jac acc2; jac_set_inf(acc2);
    g1_jac acc1; jac_set_inf(acc1);
    uint32_t nc = 0;
    for (uint64_t k = a + lane_; k < b; k += 64) {
      const uint32_t s = perm[k];
      if (flags[s] & FLAG_CANDIDATE) { jac_add(acc2, acc2, rsig[s]); jac_add(acc1, acc1, rpk[s]); ++nc; }
    }
    if (nc) atomicAdd(&ncand, nc);
    red[lane_] = acc2;
    __syncthreads();
    for (int w = 32; w > 0; w >>= 1) {
      if (lane_ < w) { g2_jac o = red[lane_ + w]; jac_add(acc2, acc2, o); red[lane_] = acc2; }
      __syncthreads();
    }
    if (lane_ == 0) { g2_aff q; jac_to_aff(q, acc2); sQ = q; }
    __syncthreads();
    g1_jac* red1 = (g1_jac*)red;
    red1[lane_] = acc1;
    __syncthreads();
    for (int w = 32; w > 0; w >>= 1) {
      if (lane_ < w) { g1_jac o = red1[lane_ + w]; jac_add(acc1, acc1, o); red1[lane_] = acc1; }
      __syncthreads();
    }
    if (lane_ == 0) { g1_aff p; jac_to_aff(p, acc1); sP = p; }
    __syncthreads();
    bool pass = true;
    if (ncand) {
      const g1_aff P = sP;
      const g2_aff Q = sQ;
      const g1_aff ng = g1_neg_generator();
      const g2_aff h = H[r];
      if (!P.inf && !Q.inf) {                  // e(S_pk, H(r)) e(-g1, S_sig), one two-pair loop
        if (lane_ < 4) { g.s[B + lane_] = ((const fp*)&h)[lane_]; g.s[B + 6 + lane_] = ((const fp*)&Q)[lane_]; }
        if (lane_ == 4) { g.s[B + 4] = P.x; g.s[B + 10] = ng.x; }
        if (lane_ == 5) { g.s[B + 5] = P.y; g.s[B + 11] = ng.y; }
        __syncthreads();
        f12_miller2(g, F1, B, BP);
      } else if (!P.inf || !Q.inf) {           // one pair at infinity: e(O, .) = e(., O) = 1
        const g2_aff q = P.inf ? Q : h;
        if (lane_ < 4) g.s[B + lane_] = ((const fp*)&q)[lane_];
        if (lane_ == 4) g.s[B + 4] = P.inf ? ng.x : P.x;
        if (lane_ == 5) g.s[B + 5] = P.inf ? ng.y : P.y;
        __syncthreads();
        f12_miller(g, F1, B);
      } else {
        const fp12 one = fp12_one();
        if (lane_ < 12) g.s[F1 + lane_] = ((const fp*)&one)[lane_];
        __syncthreads();
      }
      f12_final_exp(g, F1, TMP);
      __syncthreads();
      fp12 e;
      ld12(e, g.s + F1);
      pass = fp12_is_one(e);
    }
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

void fallback_bisect(hipStream_t st, int n, int n_roots, const rlc_key& key, const uint32_t* ok, const uint32_t* flags,
                     const uint32_t* share_root, const g2_aff* H, const g2_aff* sig, const g1_aff* pk, uint32_t* cnt,
                     uint32_t* start, uint32_t* cursor, uint32_t* perm, uint32_t* gst, g2_jac* rsig, g1_jac* rpk,
                     uint8_t* gv0, uint8_t* gv1, uint8_t* verdict, bool fast_verdicts) {
  using namespace ssb::k;
  if (n <= 0 || n_roots <= 0) return;
  auto nb = [](size_t x, unsigned b) { return (unsigned)((x + b - 1) / b); };
  const int L = fallback_levels((size_t)n);
  const int lb = fallback_log2_branch();
  const fb_prep_args prep{n_roots, L, lb, share_root, cnt, start, cursor, gst, perm};
  hipLaunchKernelGGL(k_fb_rlc, dim3(nb(2 * (size_t)n, 64) + 1), dim3(64), 0, st, n, key, ok, flags, sig, pk, rsig, rpk,
                     fast_verdicts ? verdict : (uint8_t*)nullptr, prep);
  for (int l = 0; l < L; ++l) {
    const uint64_t gs = 1ull << (lb * (L - 1 - l));
    const uint64_t bound = (uint64_t)n_roots + ((uint64_t)n + gs - 1) / gs;
    const unsigned grid = (unsigned)(bound < 2048 ? bound : 2048);
    uint8_t* cur = (l & 1) ? gv1 : gv0;
    const uint8_t* prev = (l & 1) ? gv0 : gv1;
    hipLaunchKernelGGL(k_fb_level, dim3(grid), dim3(LV_THREADS), 0, st, l, L, lb, n_roots, ok, (const uint32_t*)start,
                       (const uint32_t*)cnt, (const uint32_t*)perm, (const uint32_t*)gst, flags, (const g2_jac*)rsig,
                       (const g1_jac*)rpk, H, prev, cur, verdict);
  }
}

}  // namespace launch
}  // namespace ssb
