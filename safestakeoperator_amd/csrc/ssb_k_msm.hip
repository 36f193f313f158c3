// ssb_k_msm.hip -- the random-linear-combination sums of the batch verify as bucket MSMs
// (the reference verifies share by share, src/crypto/generic_threshold.rs:156).
//
// The batch check  prod_r e(sum_{i in r} k_i pk_i, H_r) == e(g1, sum_i k_i sig_i)  needs, over the
// candidate shares, one G1 sum per signing root and one G2 sum, with the 64-bit RLC scalars
// k_i = rlc_scalar_odd(key, i) (secret per-call key, ssb_units.h).  Both are computed as Pippenger bucket MSMs:
//   - W = ceil(64 / c) windows of c bits; entry (i, w) lands in bucket (group, w, digit), digit 0
//     dropped.  k_msm_sort<false> (count) / k_scan_* / k_msm_sort<true> (scatter) counting-sort the entries by bucket key
//     (order inside a bucket is irrelevant: the group law is exact).
//   - k_msm_bucket: a team of J lanes per bucket adds its points (mixed additions, strided), then
//     tree-reduces the team through LDS.  Entries of shares that are not candidates (failed the
//     subgroup check) are skipped here, so the sort can run before the check finishes.
//   - k_msm_window: one workgroup per (group, window) forms sum_d d*B_d: each lane runs the
//     running-sum trick over its m consecutive buckets, a Kogge-Stone suffix scan over the lanes
//     supplies the lane offsets (sum_t t*S_t = sum_{t>=1} suffix_t), and a tree adds the lanes.
//   - G1 (per root): k_msm_horner combines the windows, sum_w 2^(c w) W_w, one lane per root.
//   - G2 (one group): no doubling chain -- window w becomes its own multi-pairing pair
//     e([2^(c w)](-g1), W_w) with the constant [2^(c w)](-g1) precomputed on the host.
// Every addition is the complete Jacobian formula of ssb_curve.h (infinity, doubling and opposite
// inputs handled), so the sums are exact for any inputs.
#include "ssb_kernels.h"
#include "ssb_blocks.h"
#include "ssb_lane_ops.h"

namespace ssb {
namespace k {

// cnt[key] += 1 per (share, window) entry (SCATTER: ent[cursor[key]++] = share)
template <bool SCATTER>
__global__ void SSB_LB(256) k_msm_sort(int n, rlc_key key, const uint32_t* __restrict__ sflags,
                                                  const uint32_t* __restrict__ pflags,
                                                  const uint32_t* __restrict__ share_root, msm_cfg c2, msm_cfg c1,
                                                  uint32_t* __restrict__ cnt, uint32_t* __restrict__ ent) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !share_decodable(sflags[i], pflags[i])) return;
  msm_sort_lane<SCATTER>(i, key, share_root, c2, c1, cnt, ent);
}
// ---- exclusive scan of the bucket counts: 1024 per block, block totals, offsets ----
constexpr int SCAN_T = 256, SCAN_PER = 4, SCAN_BLOCK = SCAN_T * SCAN_PER;
SSB_INL uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t& total) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int off = 1; off < SCAN_T; off <<= 1) {
    const uint32_t o = t >= off ? sh[t - off] : 0u;
    __syncthreads();
    sh[t] += o;
    __syncthreads();
  }
  total = sh[SCAN_T - 1];
  const uint32_t incl = sh[t];
  __syncthreads();
  return incl - v;
}
__global__ void SSB_LB(SCAN_T) k_scan_blocks(uint32_t K, const uint32_t* __restrict__ cnt,
                                                        uint32_t* __restrict__ start, uint32_t* __restrict__ bsum) {
  __shared__ uint32_t sh[SCAN_T];
  const uint32_t base = blockIdx.x * SCAN_BLOCK + threadIdx.x * SCAN_PER;
  uint32_t v[SCAN_PER], s = 0;
  for (int q = 0; q < SCAN_PER; ++q) { v[q] = base + q < K ? cnt[base + q] : 0u; s += v[q]; }
  uint32_t total;
  uint32_t run = block_excl_scan(s, sh, total);
  for (int q = 0; q < SCAN_PER; ++q) { if (base + q < K) start[base + q] = run; run += v[q]; }
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}
__global__ void SSB_LB(SCAN_T) k_scan_top(uint32_t nb, uint32_t* __restrict__ bsum) {
  __shared__ uint32_t sh[SCAN_T];
  const uint32_t base = threadIdx.x * SCAN_PER;
  uint32_t v[SCAN_PER], s = 0;
  for (int q = 0; q < SCAN_PER; ++q) { v[q] = base + q < nb ? bsum[base + q] : 0u; s += v[q]; }
  uint32_t total;
  uint32_t run = block_excl_scan(s, sh, total);
  for (int q = 0; q < SCAN_PER; ++q) { if (base + q < nb) bsum[base + q] = run; run += v[q]; }
}
__global__ void SSB_LB(256) k_scan_add(uint32_t K, uint32_t* __restrict__ start,
                                                  const uint32_t* __restrict__ bsum, uint32_t* __restrict__ cur) {
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= K) return;
  const uint32_t s = start[x] + bsum[x / SCAN_BLOCK];
  start[x] = s;
  cur[x] = s;
}

// ---- bucket order: within each MSM's key range, buckets by entry count, largest first, so the
// 64/J buckets that share a wave have (nearly) the same count and the lanes' loops stay converged
// (Poisson-sized buckets in key order cost ~2x in divergence).  512 bins = 2 MSMs x counts 0..255
// (larger counts share bin 255; only the convergence depends on the order, never the result).
constexpr int ORDER_BINS = 512;
__global__ void SSB_LB(256) k_order_hist(uint32_t K, uint32_t K2, const uint32_t* __restrict__ cnt,
                                                    uint32_t* __restrict__ bins) {
  const uint32_t key = blockIdx.x * blockDim.x + threadIdx.x;
  if (key >= K) return;
  const uint32_t c = cnt[key] < 255u ? cnt[key] : 255u;
  atomicAdd(&bins[(key >= K2 ? 256u : 0u) + 255u - c], 1u);
}
__global__ void SSB_LB(256) k_order_scatter(uint32_t K, uint32_t K2, const uint32_t* __restrict__ cnt,
                                                       uint32_t* __restrict__ bins, uint32_t* __restrict__ order) {
  const uint32_t key = blockIdx.x * blockDim.x + threadIdx.x;
  if (key >= K) return;
  const uint32_t c = cnt[key] < 255u ? cnt[key] : 255u;
  order[atomicAdd(&bins[(key >= K2 ? 256u : 0u) + 255u - c], 1u)] = key;
}

// ---- bucket sums (msm_bucket_block, ssb_blocks.h) ----
template <class F>
__global__ void SSB_LB2(64) k_msm_bucket(uint32_t nb, uint32_t base, int lj, const uint32_t* __restrict__ order,
                                                   const uint32_t* __restrict__ start,
                                                   const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ ent,
                                                   const uint32_t* __restrict__ flags, const aff<F>* __restrict__ pts,
                                                   jac<F>* __restrict__ bsum) {
  __shared__ jac<F> sh[64];
  msm_bucket_block<F>(blockIdx.x, sh, nb, base, lj, order, start, cnt, ent, flags, pts, bsum);
}

// ---- window sums (msm_window_block, ssb_blocks.h) ----
template <class F>
__global__ void SSB_LB(64) k_msm_window(int c, const jac<F>* __restrict__ bsum, jac<F>* __restrict__ out_jac,
                                                   aff<F>* __restrict__ out_q, g1_aff* __restrict__ out_p,
                                                   const g1_aff* __restrict__ negg1_pow, const uint32_t* __restrict__ redo,
                                                   const jac<F>* __restrict__ lane_sum) {
  __shared__ jac<F> sh[64];
  msm_window_block<F>(blockIdx.x, sh, c, bsum, out_jac, out_q, out_p, negg1_pow, redo, lane_sum);
}

// ---- narrow-window sums (msm_window_seq_block, ssb_blocks.h) ----
template <class F>
__global__ void SSB_LB(64) k_msm_window_seq(uint32_t ngw, int c, const jac<F>* __restrict__ bsum,
                                                       jac<F>* __restrict__ out_jac) {
  msm_window_seq_block<F>(blockIdx.x, ngw, c, bsum, out_jac);
}

// ---- the G2 and G1 sides in one launch (one-stream slots: the two MSMs overlap on the device
// instead of running back to back on the slot's stream; blocks [0, nblk2) are G2's) ----
struct msm_bucket_args {
  uint32_t nb, base; int lj; const uint32_t* order; const uint32_t* start; const uint32_t* cnt; const uint32_t* ent;
};
// the G1 side's merged MSM (msm_cfg::merged): the cached keys' precomputed bases and the shares' cache indices
struct g1_pre_args { const g1_aff* pow; const uint32_t* pidx; };
// hash_to_G2 stages riding along (nblk of their own; 0 = none): the SWU map beside the subgroup
// checks, the cofactor clearing beside the bucket sums, the affine output beside the window sums
struct h2c_fuse { int n; const fp2* u; g2_aff* q; g2_jac* hj; uint32_t* exc; int exact_all; g2_aff* out; };
#ifndef SSB_B2_WAVES   // experiment knob: waves per SIMD of the fused bucket launch
#define SSB_B2_WAVES 2
#endif
#ifndef SSB_SG_WAVES   // experiment knob: waves per SIMD of the subgroup-check launch
#define SSB_SG_WAVES 2
#endif
__global__ void __attribute__((amdgpu_flat_work_group_size(1, 64), amdgpu_waves_per_eu(SSB_B2_WAVES))) k_msm_bucket2(uint32_t nblk2, msm_bucket_args a2, msm_bucket_args a1,
                                         const uint32_t* __restrict__ flags, const g2_aff* __restrict__ sig,
                                         const g1_aff* __restrict__ pk, g2_jac* __restrict__ b2, g1_jac* __restrict__ b1,
                                         g1_pre_args pre) {
  __shared__ g2_jac sh[64];
  if (blockIdx.x < nblk2)
    msm_bucket_block<fp2>(blockIdx.x, sh, a2.nb, a2.base, a2.lj, a2.order, a2.start, a2.cnt, a2.ent, flags, sig, b2);
  else
    msm_bucket_block<fp>(blockIdx.x - nblk2, (g1_jac*)sh, a1.nb, a1.base, a1.lj, a1.order, a1.start, a1.cnt, a1.ent, flags,
                         pk, b1, pre.pow, pre.pidx);
}
// (the cofactor clearing's lane programs need 32 KB of LDS per block: they ride with the window
// sums, a launch of few blocks, not with the bucket sums, whose many blocks the LDS would thin out)
constexpr size_t WINDOW2_LDS = 64 * sizeof(g2_jac) > H2C_CLEAR_LDS ? 64 * sizeof(g2_jac) : H2C_CLEAR_LDS;
// With tickets (the fused one-stream path), the last G1-window block to finish also runs the G1
// Horner of every root, and the last clearing block the affine output of every root: both ride in
// this launch behind the G2 window sums instead of following in a launch of their own.
SSB_INL void msm_horner_lane(int g, int c, int W, const g1_jac* __restrict__ wsum, g1_aff* __restrict__ out) {
  const g1_jac* ws = wsum + (size_t)g * W;
  g1_jac acc = ws[W - 1];
  for (int w = W - 2; w >= 0; --w) {
#pragma unroll 1
    for (int q = 0; q < c; ++q) jac_dbl_inl(acc, acc);
    g1_jac o = ws[w];
    jac_add(acc, acc, o);
  }
  g1_aff a;
  jac_to_aff(a, acc);
  out[g] = a;
}
struct window2_tail { uint32_t* tickets; int ngroups1, W1; g1_aff* root_sum; int merged; };
// the merged G1 MSM's per-root reduce, one lane per root: root_sum[r] = sum_{d=1}^{15} d B_{r,d} by
// running sums (28 additions) -- no per-window sums and no Horner (60 doublings + 15 additions per
// root on one lane, the window launch's longest chain at 1.8 ms before the precomputed bases)
SSB_INL void msm_root_lane(int r, const g1_jac* __restrict__ b1, g1_aff* __restrict__ out) {
  const g1_jac* bk = b1 + ((size_t)r << 4);
  g1_jac S = bk[15], U = S;
  for (int d = 14; d >= 1; --d) {
    g1_jac o = bk[d];
    jac_add(S, S, o);
    jac_add(U, U, S);
  }
  g1_aff a;
  jac_to_aff(a, U);
  out[r] = a;
}
SSB_INL bool last_block(uint32_t* ticket, uint32_t nblocks, uint32_t* flag_lds) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    *flag_lds = atomicAdd(ticket, 1u) == nblocks - 1 ? 1u : 0u;
  }
  __syncthreads();
  const bool last = *flag_lds != 0;
  if (last) __threadfence();
  return last;
}
__global__ void SSB_LB(64) k_msm_window2(uint32_t nblk2, int c2, const g2_jac* __restrict__ b2, g2_aff* __restrict__ pair_q,
                                         g1_aff* __restrict__ pair_p, const g1_aff* __restrict__ negg1_pow,
                                         uint32_t nblk1, uint32_t ngw1, int c1, const g1_jac* __restrict__ b1,
                                         g1_jac* __restrict__ w1, h2c_fuse h, window2_tail tl) {
  __shared__ __attribute__((aligned(16))) char lds[WINDOW2_LDS];
  __shared__ uint32_t last;
  SSB_TRACE_T0();
  uint32_t bid = blockIdx.x;
  if (bid < nblk2) {
    msm_window_block<fp2>(bid, (g2_jac*)lds, c2, b2, (g2_jac*)nullptr, pair_q, pair_p, negg1_pow, (const uint32_t*)nullptr,
                          (const g2_jac*)nullptr);
    SSB_TRACE(TR_W2_G2);
    return;
  }
  bid -= nblk2;
  if (bid < nblk1) {
    if (tl.merged) {   // the merged G1 MSM: one reduce per root, straight to root_sum
      const int r = (int)bid * 64 + threadIdx.x;
      if (r < tl.ngroups1) msm_root_lane(r, b1, tl.root_sum);
      SSB_TRACE(TR_W2_G1);
      return;
    }
    if (!tl.tickets) { msm_window_seq_block<fp>(bid, ngw1, c1, b1, w1); return; }
    if (bid * 64 + threadIdx.x < ngw1) msm_window_seq_block<fp>(bid, ngw1, c1, b1, w1);
    SSB_TRACE(TR_W2_G1);
    if (last_block(&tl.tickets[1], nblk1, &last)) {
      for (int g = threadIdx.x; g < tl.ngroups1; g += 64) msm_horner_lane(g, c1, tl.W1, w1, tl.root_sum);
      if (threadIdx.x == 0) tl.tickets[1] = 0u;   // clean for the slot's next batch
      SSB_TRACE(TR_W2_HORNER);
    }
    return;
  }
  bid -= nblk1;
  h2c_clear_block(bid, (lane::lslot*)lds, h.n, h.q, h.hj, h.exc);
  SSB_TRACE(TR_W2_CLEAR);
  if (tl.tickets && last_block(&tl.tickets[2], (uint32_t)(h.n + 7) / 8, &last)) {
    for (uint32_t b = 0; b * 64 < (uint32_t)h.n; ++b) h2c_affine_block(b, h.n, h.q, h.hj, h.exc, h.exact_all, h.out);
    if (threadIdx.x == 0) tl.tickets[2] = 0u;
    SSB_TRACE(TR_W2_AFFINE);
  }
}

// ---- latency configuration (one batch in flight: ssb_set_pipeline_depth(1), one-stream slots) ----
// With a single batch on the device nothing competes for the CUs the window launch leaves idle, so
// the G2 window sums run as 8-lane programs (lp_g2_add: 6 product rounds per addition on a group of
// 8 lanes, against 43 dependent Fp products on one lane), 32 groups per window in one 256-lane
// block, the G1 side's per-root reduce likewise (4-lane groups, lp_g1_add), and the cofactor
// clearing rides in the bucket launch instead of the window launch.  Under
// load (depth > 1) the same forms measured slower -- four-wave, LDS-heavy blocks waiting for a CU
// with room -- so the pipelined path keeps the single-lane window block.
constexpr int WL_NT = 256;
constexpr int WL_G = lane::G2_ADD_G, WL_NG = WL_NT / WL_G, WL_NC = 6;
constexpr int WL_S = lane::G2_ADD_SCRATCH > lane::G2_DBL_SCRATCH ? lane::G2_ADD_SCRATCH : lane::G2_DBL_SCRATCH;
constexpr int WL_U = WL_S + WL_NC, WL_O = WL_U + WL_NC, WL_X = WL_O + WL_NC, WL_Y = WL_X + WL_NC, WL_T = WL_Y + WL_NC,
              WL_GS = WL_T + WL_NC;
constexpr size_t WL_SLOTS_LDS = (lane::LP_NCODE_CONST + WL_NG * WL_GS) * sizeof(lane::lslot);
static_assert(WL_SLOTS_LDS >= 64 * sizeof(g2_jac), "the exact redo's tree LDS aliases the lane slots");
// the merged G1 side's per-root reduce in the same launch: one group of 4 lanes per root (lp_g1_add)
constexpr int RL_G = lane::G1_ADD_G, RL_NG = WL_NT / RL_G, RL_NC = 3;
constexpr int RL_S = lane::G1_ADD_SCRATCH, RL_U = RL_S + RL_NC, RL_O = RL_U + RL_NC, RL_Y = RL_O + RL_NC, RL_GS = RL_Y + RL_NC;
static_assert((lane::LP_NCODE_CONST + RL_NG * RL_GS) * sizeof(lane::lslot) <= WL_SLOTS_LDS, "root reduce slots");
struct wl_flags { uint32_t flg[RL_NG > WL_NG ? RL_NG : WL_NG], has[WL_NG], exc_any; };
// One G2 window sum_d d B_d on WL_NG groups: group t owns the m = 2^c / WL_NG consecutive buckets
// [t m, (t + 1) m):  S_t = sum_e B_{tm+e}, U_t = sum_e e B_{tm+e} (running sums), a suffix scan of S
// over the groups, U_t += [m] suffix_t (t >= 1), a tree of U over the groups.  Operands at infinity
// (empty buckets and their sums) are tracked per group; an exceptional addition (equal or opposite
// points) makes the caller redo the window with the complete single-lane formulas.  Output:
// the affine pair (W_w, [2^(c w)](-g1)) of the multi-pairing, as msm_window_block writes it; returns
// true (uniformly, nothing written) when the window must be redone exactly.
SSB_INL bool msm_window_lane_block(uint32_t bid, lane::lslot* lds, wl_flags& F, int c, const g2_jac* __restrict__ bsum,
                                   g2_aff* __restrict__ out_q, g1_aff* __restrict__ out_p, const g1_aff* __restrict__ negg1_pow) {
  using namespace ssb::lane;
  const int t = threadIdx.x / WL_G, role = threadIdx.x % WL_G;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST + t * WL_GS, 0, 0, 0, (lu32*)&F.flg[t], role};
  if (threadIdx.x == 0) F.exc_any = 0u;
  lp_init_consts(g);
  // Window 0 holds odd digits only (the RLC scalars are odd): its even buckets are all empty, and the
  // running sums over them would add a point to itself.  It runs over the odd buckets B'_j = B_{2j+1}
  // instead -- sum_d d B_d = 2 sum_j j B'_j + sum_j B'_j -- the plain sum being the scan's suffix_0.
  const bool odd = bid == 0;
  const int m = (1 << c) / (odd ? 2 * WL_NG : WL_NG);
  const g2_jac* bk = bsum + ((size_t)bid << c) + (odd ? 1 : 0);
  const int st = odd ? 2 : 1;   // bucket stride
  lfp* base = (lfp*)lds + LP_NCODE_CONST;
  auto load = [&](int slot, const g2_jac& p) { if (role < WL_NC) lp_put(g.s + slot + role, lv_in(((const fp*)&p)[role])); };
  auto copy = [&](int dst, int src) { if (role < WL_NC) g.s[dst + role] = g.s[src + role]; };
  // Every program call is made by every group (the programs synchronise the block); a group whose
  // operand is infinity -- an empty bucket (window 0's even digits: the RLC scalars are odd), or a
  // sum of them -- keeps or takes the other operand instead of the program's result, so the lane
  // checks only fire on equal or opposite points (then the caller redoes the window exactly).
  uint32_t exc = 0;
  // acc <- acc + o (o at slot `os`, at infinity when oinf), through WL_Y
  auto acc_add = [&](int acc, bool& ainf, int os, bool oinf, bool use) {
    uint32_t e2 = 0;
    g2_add(g, acc, os, WL_Y, e2);
    if (use && !oinf) {
      if (ainf) copy(acc, os);
      else { exc |= e2; copy(acc, WL_Y); }
      ainf = false;
    }
    __syncthreads();
  };
  bool sinf = jac_is_inf(bk[st * (t * m + m - 1)]), uinf = sinf;
  load(WL_S, bk[st * (t * m + m - 1)]);
  load(WL_U, bk[st * (t * m + m - 1)]);
  for (int e = m - 2; e >= 0; --e) {
    // (group 0's bucket e = 0 is digit 0: never filled, of weight 0 in U_0, and S_0 feeds no suffix;
    // in the odd form it is B_1, of weight 0 in the j-sum and part of the plain sum)
    const bool binf = (!odd && t == 0 && e == 0) || jac_is_inf(bk[st * (t * m + e)]);
    load(WL_O, bk[st * (t * m + e)]);
    __syncthreads();
    acc_add(WL_S, sinf, WL_O, binf, true);
    if (e >= 1) acc_add(WL_U, uinf, WL_S, sinf, true);
  }
  // suffix scan: S_t <- sum_{t' >= t} S_t'
  for (int off = 1; off < WL_NG; off <<= 1) {
    copy(WL_X, WL_S);
    if (role == 0) F.has[t] = sinf ? 0u : 1u;
    __syncthreads();
    const bool act = t + off < WL_NG;
    const int src = act ? t + off : t;
    if (role < WL_NC) base[t * WL_GS + WL_O + role] = base[src * WL_GS + WL_X + role];
    const bool oinf = !F.has[src];
    __syncthreads();
    acc_add(WL_S, sinf, WL_O, oinf, act);
  }
  const bool tinf = sinf;   // (group 0: the plain sum of the odd form)
  copy(WL_T, WL_S);
  // U_t += [m] S_t for t >= 1 (group 0's suffix carries weight 0)
  for (int q = m; q > 1; q >>= 1) g2_dbl(g, WL_S, WL_S);
  acc_add(WL_U, uinf, WL_S, sinf, t >= 1);
  // tree over the groups
  for (int h = WL_NG / 2; h >= 1; h >>= 1) {
    copy(WL_X, WL_U);
    if (role == 0) F.has[t] = uinf ? 0u : 1u;
    __syncthreads();
    const bool act = t < h;
    const int src = act ? t + h : t;
    if (role < WL_NC) base[t * WL_GS + WL_O + role] = base[src * WL_GS + WL_X + role];
    const bool oinf = !F.has[src];
    __syncthreads();
    acc_add(WL_U, uinf, WL_O, oinf, act);
  }
  if (odd) {   // group 0: 2 U' + sum_j B'_j
    g2_dbl(g, WL_U, WL_U);
    bool ui = uinf;
    acc_add(WL_U, ui, WL_T, tinf, t == 0);
    uinf = ui;
  }
  if (exc && role == 0) atomicOr(&F.exc_any, 1u);
  __syncthreads();
  if (F.exc_any) return true;   // uniform: the caller redoes the window exactly
  if (threadIdx.x == 0) {
    g2_jac r;
    if (uinf) jac_set_inf(r);
    else for (int i = 0; i < WL_NC; ++i) ((fp*)&r)[i] = lv_out(lp_get(g.s + WL_U + i));
    g2_aff a;
    jac_to_aff(a, r);
    out_q[bid] = a;
    out_p[bid] = negg1_pow[c * bid];
  }
  return false;
}

// root_sum[r] = sum_{d=1}^{15} d B_{r,d} (msm_root_lane's running sums) on a group of RL_G lanes per
// root, RL_NG roots per block; operands at infinity tracked per group, a root whose additions met
// equal or opposite points is redone on one lane (msm_root_lane, no barriers).
SSB_INL void msm_root_lane_block(uint32_t bid, lane::lslot* lds, wl_flags& F, int ngroups, const g1_jac* __restrict__ b1,
                                 g1_aff* __restrict__ out) {
  using namespace ssb::lane;
  const int t = threadIdx.x / RL_G, role = threadIdx.x % RL_G;
  const int r = (int)bid * RL_NG + t;
  const bool act = r < ngroups;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST + t * RL_GS, 0, 0, 0, (lu32*)&F.flg[t], role};
  lp_init_consts(g);
  const g1_jac* bk = b1 + ((size_t)(act ? r : 0) << 4);
  auto load = [&](int slot, const g1_jac& p) { if (role < RL_NC) lp_put(g.s + slot + role, lv_in(((const fp*)&p)[role])); };
  auto copy = [&](int dst, int src) { if (role < RL_NC) g.s[dst + role] = g.s[src + role]; };
  uint32_t exc = 0;
  auto acc_add = [&](int acc, bool& ainf, int os, bool oinf) {
    uint32_t e2 = 0;
    g1_add(g, acc, os, RL_Y, e2);
    if (!oinf) {
      if (ainf) copy(acc, os);
      else { exc |= e2; copy(acc, RL_Y); }
      ainf = false;
    }
    __syncthreads();
  };
  bool sinf = jac_is_inf(bk[15]), uinf = sinf;
  load(RL_S, bk[15]);
  load(RL_U, bk[15]);
  for (int d = 14; d >= 1; --d) {
    const bool binf = jac_is_inf(bk[d]);
    load(RL_O, bk[d]);
    __syncthreads();
    acc_add(RL_S, sinf, RL_O, binf);
    acc_add(RL_U, uinf, RL_S, sinf);
  }
  if (!act || role != 0) return;
  if (exc) { msm_root_lane(r, b1, out); return; }
  g1_jac j;
  if (uinf) jac_set_inf(j);
  else for (int i = 0; i < RL_NC; ++i) ((fp*)&j)[i] = lv_out(lp_get(g.s + RL_U + i));
  g1_aff a;
  jac_to_aff(a, j);
  out[r] = a;
}
__global__ void __launch_bounds__(WL_NT) k_msm_window2_lat(uint32_t nblk2, int c2, const g2_jac* __restrict__ b2,
                                                         g2_aff* __restrict__ pair_q, g1_aff* __restrict__ pair_p,
                                                         const g1_aff* __restrict__ negg1_pow, const g1_jac* __restrict__ b1,
                                                         window2_tail tl) {
  __shared__ lane::lslot lds[WL_SLOTS_LDS / sizeof(lane::lslot)];
  __shared__ wl_flags F;
  SSB_TRACE_T0();
  if (blockIdx.x < nblk2) {
    const bool redo = msm_window_lane_block(blockIdx.x, lds, F, c2, b2, pair_q, pair_p, negg1_pow);
    SSB_TRACE(TR_W2_G2);
    if (redo) {   // (the slots are dead: the exact form's tree LDS aliases them)
      __syncthreads();
      msm_window_block<fp2>(blockIdx.x, (g2_jac*)lds, c2, b2, (g2_jac*)nullptr, pair_q, pair_p, negg1_pow,
                            (const uint32_t*)nullptr, (const g2_jac*)nullptr);
      SSB_TRACE(TR_W2_HORNER);
    }
    return;
  }
  msm_root_lane_block(blockIdx.x - nblk2, lds, F, tl.ngroups1, b1, tl.root_sum);   // the merged G1 side
  SSB_TRACE(TR_W2_G1);
}
// The bucket sums with the cofactor clearing riding along (latency configuration): blocks
// [nblk2 + nblk1, + (n + 7) / 8) clear eight roots each; the last of them writes every root's affine
// H(root).  No waves-per-EU bound: the bucket bodies may take a whole SIMD's registers here (the
// launch's ~750 waves fit the 1,024 SIMDs of an idle chip) and the lane programs keep the register
// budget the window launch gives them.
__global__ void __attribute__((amdgpu_flat_work_group_size(1, 64))) k_msm_bucket2_clr(
    uint32_t nblk2, uint32_t nblk1, msm_bucket_args a2, msm_bucket_args a1, const uint32_t* __restrict__ flags,
    const g2_aff* __restrict__ sig, const g1_aff* __restrict__ pk, g2_jac* __restrict__ b2, g1_jac* __restrict__ b1,
    g1_pre_args pre, h2c_fuse h, uint32_t* __restrict__ tickets) {
  constexpr size_t LDS = H2C_CLEAR_LDS > 64 * sizeof(g2_jac) ? H2C_CLEAR_LDS : 64 * sizeof(g2_jac);
  __shared__ __attribute__((aligned(16))) char lds[LDS];
  __shared__ uint32_t last;
  SSB_TRACE_T0();
  if (blockIdx.x < nblk2) {
    msm_bucket_block<fp2>(blockIdx.x, (g2_jac*)lds, a2.nb, a2.base, a2.lj, a2.order, a2.start, a2.cnt, a2.ent, flags, sig, b2);
    return;
  }
  if (blockIdx.x < nblk2 + nblk1) {
    msm_bucket_block<fp>(blockIdx.x - nblk2, (g1_jac*)lds, a1.nb, a1.base, a1.lj, a1.order, a1.start, a1.cnt, a1.ent, flags,
                         pk, b1, pre.pow, pre.pidx);
    return;
  }
  h2c_clear_block(blockIdx.x - nblk2 - nblk1, (lane::lslot*)lds, h.n, h.q, h.hj, h.exc);
  SSB_TRACE(TR_W2_CLEAR);
  if (last_block(&tickets[2], (uint32_t)(h.n + 7) / 8, &last)) {
    for (uint32_t b = 0; b * 64 < (uint32_t)h.n; ++b) h2c_affine_block(b, h.n, h.q, h.hj, h.exc, h.exact_all, h.out);
    if (threadIdx.x == 0) tickets[2] = 0u;
    SSB_TRACE(TR_W2_AFFINE);
  }
}

// ---- per-group Horner over the windows (G1 roots): out[g] = sum_w 2^(c w) W_{g,w}, affine ----
__global__ void SSB_LB(64) k_msm_horner(int ngroups, int c, int W, const g1_jac* __restrict__ wsum,
                                                   g1_aff* __restrict__ out, const uint32_t* __restrict__ redo) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngroups || (redo && !redo[g])) return;
  msm_horner_lane(g, c, W, wsum, out);
}

// the G1 Horner (blocks [0, nbh)) with the hash's affine output riding along
__global__ void SSB_LB(64) k_msm_horner2(uint32_t nbh, int ngroups, int c, int W, const g1_jac* __restrict__ wsum,
                                        g1_aff* __restrict__ out, h2c_fuse h) {
  if (blockIdx.x >= nbh) { h2c_affine_block(blockIdx.x - nbh, h.n, h.q, h.hj, h.exc, h.exact_all, h.out); return; }
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < ngroups) msm_horner_lane(g, c, W, wsum, out);
}

// per-share G1 RLC product (the G1 side when the roots' groups are small: 64 doublings per share
// beat a per-root bucket MSM whose window reduce / Horner overheads dominate at ~256 shares/root)
__global__ void SSB_LB(64) k_rlc_pk(int n, rlc_key key, const uint32_t* __restrict__ sflags,
                                               const uint32_t* __restrict__ pflags, const g1_aff* __restrict__ pk_aff,
                                               g1_jac* __restrict__ rpk) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  g1_jac r;
  if (share_decodable(sflags[s], pflags[s])) unit_rlc_pk(r, pk_aff[s], rlc_scalar_odd(key, (uint64_t)s));
  else jac_set_inf(r);
  rpk[s] = r;
}

// subgroup check of every decodable signature (psi(P) == [x]P, sig_groupcheck)
__global__ void SSB_LB2(64) k_subgroup(int n, const uint32_t* __restrict__ sflags,
                                                 const g2_aff* __restrict__ sig_aff, uint32_t* __restrict__ gflags) {
  __shared__ uint32_t keep[r28::KEEP_WORDS * 64];
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const uint32_t sf = sflags[s];
  gflags[s] = ((sf & DEC_OK) && !(sf & DEC_INF)) ? unit_subgroup(sig_aff[s], (r28::keep_t*)keep + threadIdx.x) : 0u;
}

// exact single-lane redo of the shares whose lane-group subgroup check met an exceptional addition
__global__ void SSB_LB2(64) k_subgroup_fix(int n, const uint32_t* __restrict__ sflags, const g2_aff* __restrict__ sig_aff,
                                          const uint32_t* __restrict__ exc, uint32_t* __restrict__ gflags) {
  __shared__ uint32_t keep[r28::KEEP_WORDS * 64];
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n || !exc[s]) return;
  const uint32_t sf = sflags[s];
  gflags[s] = ((sf & DEC_OK) && !(sf & DEC_INF)) ? unit_subgroup(sig_aff[s], (r28::keep_t*)keep + threadIdx.x) : 0u;
}

// subgroup checks (blocks [0, nbs)) with the hash's SWU map riding along (the next nbm blocks)
// and, for the fused sort (sc.ent != nullptr), the counting sort's scatter (the remaining blocks);
// a subgroup lane also writes the share's combined flags (k_flags) when sc.flags is given
struct sort_scatter { int n; rlc_key key; const uint32_t* share_root; msm_cfg c2, c1; uint32_t* cur; uint32_t* ent;
                      const uint32_t* pflags; uint32_t n_roots; uint32_t* flags; };
// the riding roles out of line: inlined, their register demand set the whole kernel's allocation and
// the subgroup lanes spilled (32 scratch stores in the kernel body against 5 in k_subgroup)
SSB_ROLE void sg_map_role(uint32_t b, h2c_cand* cs, const h2c_fuse& h) { h2c_map_block(b, cs, h.n, h.u, h.q); }
SSB_ROLE void sg_scatter_role(int i, const sort_scatter& sc) {
  msm_sort_lane<true>(i, sc.key, sc.share_root, sc.c2, sc.c1, sc.cur, sc.ent);
}
__global__ void __attribute__((amdgpu_flat_work_group_size(1, 64), amdgpu_waves_per_eu(SSB_SG_WAVES))) k_subgroup_map(int n, uint32_t nbs, const uint32_t* __restrict__ sflags,
                                           const g2_aff* __restrict__ sig_aff, uint32_t* __restrict__ gflags, h2c_fuse h,
                                           uint32_t nbm, sort_scatter sc) {
  // LDS: the map role's candidates, or the subgroup lanes' affine points (r28::KEEP_WORDS words each)
  constexpr size_t SG_LDS = H2C_MAP_LDS > r28::KEEP_WORDS * 64 * 4 ? H2C_MAP_LDS : r28::KEEP_WORDS * 64 * 4;
  __shared__ __attribute__((aligned(16))) char lds[SG_LDS];
  if (blockIdx.x >= nbs) {
    const uint32_t b = blockIdx.x - nbs;
    if (b < nbm) { sg_map_role(b, (h2c_cand*)lds, h); return; }
    const int i = (b - nbm) * 64 + threadIdx.x;
    if (i < sc.n) sg_scatter_role(i, sc);
    return;
  }
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const uint32_t sf = sflags[s];
  const uint32_t gf = ((sf & DEC_OK) && !(sf & DEC_INF)) ? unit_subgroup(sig_aff[s], (r28::keep_t*)lds + threadIdx.x) : 0u;
  gflags[s] = gf;
  if (sc.flags) {
    uint32_t f = combine_flags(sf, sc.pflags[s], gf);
    if (sc.share_root[s] >= sc.n_roots) f &= ~FLAG_CANDIDATE;
    sc.flags[s] = f;
  }
}

}  // namespace k

namespace launch {

using namespace ssb::k;

void msm_sort(hipStream_t st, int n, const rlc_key& key, const uint32_t* sflags, const uint32_t* pflags,
              const uint32_t* share_root, const msm_cfg& c2, const msm_cfg& c1, uint32_t K, uint32_t* cnt,
              uint32_t* start, uint32_t* cur, uint32_t* bsum, uint32_t* ent, uint32_t* order) {
  hipMemsetAsync(cnt, 0, (size_t)K * 4, st);
  const unsigned g = (unsigned)((n + 255) / 256), nb = (K + SCAN_BLOCK - 1) / SCAN_BLOCK;
  if (n) hipLaunchKernelGGL(k_msm_sort<false>, dim3(g), dim3(256), 0, st, n, key, sflags, pflags, share_root, c2, c1, cnt, ent);
  hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(SCAN_T), 0, st, K, cnt, start, bsum);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_T), 0, st, nb, bsum);
  hipLaunchKernelGGL(k_scan_add, dim3((K + 255) / 256), dim3(256), 0, st, K, start, bsum, cur);
  if (n) hipLaunchKernelGGL(k_msm_sort<true>, dim3(g), dim3(256), 0, st, n, key, sflags, pflags, share_root, c2, c1, cur, ent);
  // bucket order by count (bsum reused for the 512 bins)
  hipMemsetAsync(bsum, 0, ORDER_BINS * 4, st);
  hipLaunchKernelGGL(k_order_hist, dim3((K + 255) / 256), dim3(256), 0, st, K, c1.base, cnt, bsum);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_T), 0, st, (uint32_t)ORDER_BINS, bsum);
  hipLaunchKernelGGL(k_order_scatter, dim3((K + 255) / 256), dim3(256), 0, st, K, c1.base, cnt, bsum, order);
}

void msm_g2(hipStream_t st, const msm_cfg& c, int lj, const uint32_t* order, const uint32_t* start, const uint32_t* cnt, const uint32_t* ent,
            const uint32_t* flags, const g2_aff* sig, g2_jac* bsum, g2_aff* pair_q, g1_aff* pair_p,
            const g1_aff* negg1_pow) {
  const uint32_t nb = c.ngroups * c.W << c.c;
  hipLaunchKernelGGL(k_msm_bucket<fp2>, dim3((nb + (64u >> lj) - 1) / (64u >> lj)), dim3(64), 0, st, nb, c.base, lj, order, start,
                     cnt, ent, flags, sig, bsum);
  hipLaunchKernelGGL(k_msm_window<fp2>, dim3(c.ngroups * c.W), dim3(64), 0, st, (int)c.c, (const g2_jac*)bsum,
                     (g2_jac*)nullptr, pair_q, pair_p, negg1_pow, (const uint32_t*)nullptr, (const g2_jac*)nullptr);
}

void msm_g1(hipStream_t st, const msm_cfg& c, int lj, const uint32_t* order, const uint32_t* start, const uint32_t* cnt, const uint32_t* ent,
            const uint32_t* flags, const g1_aff* pk, g1_jac* bsum, g1_jac* wsum, g1_aff* root_sum) {
  const uint32_t nb = c.ngroups * c.W << c.c;
  const uint32_t nw = c.ngroups * c.W;
  hipLaunchKernelGGL(k_msm_bucket<fp>, dim3((nb + (64u >> lj) - 1) / (64u >> lj)), dim3(64), 0, st, nb, c.base, lj, order, start,
                     cnt, ent, flags, pk, bsum);
  if (c.c <= 4) {
    hipLaunchKernelGGL(k_msm_window_seq<fp>, dim3((nw + 63) / 64), dim3(64), 0, st, nw, (int)c.c, (const g1_jac*)bsum, wsum);
  } else {
    hipLaunchKernelGGL(k_msm_window<fp>, dim3(nw), dim3(64), 0, st, (int)c.c, (const g1_jac*)bsum, wsum,
                       (g1_aff*)nullptr, (g1_aff*)nullptr, (const g1_aff*)nullptr, (const uint32_t*)nullptr, (const g1_jac*)nullptr);
  }
  hipLaunchKernelGGL(k_msm_horner, dim3((c.ngroups + 63) / 64), dim3(64), 0, st, (int)c.ngroups, (int)c.c, (int)c.W,
                     (const g1_jac*)wsum, root_sum, (const uint32_t*)nullptr);
}

bool msm_fused_ok(const msm_cfg& c1) { return c1.c <= 4; }

h2c_fuse fuse_of(const h2c_ws* hw, int n_roots, g2_aff* out) {
  h2c_fuse h{0, nullptr, nullptr, nullptr, nullptr, 0, nullptr};
  if (hw && n_roots > 0) h = h2c_fuse{n_roots, hw->u, hw->q, hw->hj, hw->exc, h2c_exact_all(), out};
  return h;
}

void msm_both(hipStream_t st, const msm_cfg& c2, int lj2, const msm_cfg& c1, int lj1, const uint32_t* order,
              const uint32_t* start, const uint32_t* cnt, const uint32_t* ent, const uint32_t* flags, const g2_aff* sig,
              const g1_aff* pk, g2_jac* b2, g1_jac* b1, g2_aff* pair_q, g1_aff* pair_p, const g1_aff* negg1_pow,
              g1_jac* wsum1, g1_aff* root_sum, const h2c_ws* hw, int n_roots, g2_aff* H, uint32_t* tickets,
              const g1_aff* pk_pow, const uint32_t* pk_index, bool lat) {
  const h2c_fuse h = fuse_of(hw, n_roots, H);
  const uint32_t nb2 = msm_nbuckets(c2), nb1 = msm_nbuckets(c1);
  const g1_pre_args pre{c1.merged ? pk_pow : nullptr, c1.merged ? pk_index : nullptr};
  const uint32_t nblk2 = (nb2 + (64u >> lj2) - 1) / (64u >> lj2), nblk1 = (nb1 + (64u >> lj1) - 1) / (64u >> lj1);
  const uint32_t nbc = h.n ? (uint32_t)(h.n + 7) / 8 : 0u, nba = h.n ? (uint32_t)(h.n + 63) / 64 : 0u;
  const msm_bucket_args a2{nb2, c2.base, lj2, order, start, cnt, ent}, a1{nb1, c1.base, lj1, order, start, cnt, ent};
  // latency configuration (one batch in flight): the clearing beside the bucket sums, the G2 window
  // sums as lane programs (>= 2 buckets per lane group, window 0's odd ones included), the merged G1
  // side's per-root reduce beside them
  if (lat && tickets && h.n && c1.merged && c2.ngroups == 1 && (1u << c2.c) >= 4u * (uint32_t)WL_NG) {
    hipLaunchKernelGGL(k_msm_bucket2_clr, dim3(nblk2 + nblk1 + nbc), dim3(64), 0, st, nblk2, nblk1, a2, a1, flags, sig, pk, b2,
                       b1, pre, h, tickets);
    const window2_tail tl{tickets, (int)c1.ngroups, (int)c1.W, root_sum, 1};
    const uint32_t nw2 = c2.W, nbr = (c1.ngroups + RL_NG - 1) / RL_NG;
    hipLaunchKernelGGL(k_msm_window2_lat, dim3(nw2 + nbr), dim3(WL_NT), 0, st, nw2, (int)c2.c, (const g2_jac*)b2, pair_q, pair_p,
                       negg1_pow, (const g1_jac*)b1, tl);
    return;
  }
  hipLaunchKernelGGL(k_msm_bucket2, dim3(nblk2 + nblk1), dim3(64), 0, st, nblk2, a2, a1, flags, sig, pk, b2, b1, pre);
  const uint32_t nw2 = c2.ngroups * c2.W, nw1 = c1.ngroups * c1.W;
  const uint32_t nbw1 = c1.merged ? (c1.ngroups + 63) / 64 : (nw1 + 63) / 64;
  const window2_tail tl{tickets, (int)c1.ngroups, (int)c1.W, root_sum, (int)c1.merged};
  hipLaunchKernelGGL(k_msm_window2, dim3(nw2 + nbw1 + nbc), dim3(64), 0, st, nw2, (int)c2.c, (const g2_jac*)b2,
                     pair_q, pair_p, negg1_pow, nbw1, nw1, (int)c1.c, (const g1_jac*)b1, wsum1, h, tl);
  if (tickets) return;   // the Horner and the affine H ran in the window launch's last blocks
  // (a merged G1 side has no Horner and always runs with tickets -- run_verify checks)
  const uint32_t nbh = (c1.ngroups + 63) / 64;
  hipLaunchKernelGGL(k_msm_horner2, dim3(nbh + nba), dim3(64), 0, st, nbh, (int)c1.ngroups, (int)c1.c, (int)c1.W,
                     (const g1_jac*)wsum1, root_sum, h);
}

void subgroup_map(hipStream_t st, int n, const uint32_t* sflags, const g2_aff* sig, uint32_t* gflags, const h2c_ws* hw,
                  int n_roots, const fused_sort* fs) {
  const h2c_fuse h = fuse_of(hw, n_roots, nullptr);
  const uint32_t nbs = (uint32_t)(n + 63) / 64, nbm = h.n ? (uint32_t)(4 * h.n + 63) / 64 : 0u;
  sort_scatter sc{0, rlc_key{}, nullptr, msm_cfg{}, msm_cfg{}, nullptr, nullptr, nullptr, 0u, nullptr};
  uint32_t nsc = 0;
  if (fs) {
    sc = sort_scatter{n, fs->key, fs->share_root, fs->c2, fs->c1, fs->cur, fs->ent, fs->pflags, fs->n_roots, fs->flags};
    nsc = (uint32_t)(n + 63) / 64;
  }
  if (nbs + nbm + nsc)
    hipLaunchKernelGGL(k_subgroup_map, dim3(nbs + nbm + nsc), dim3(64), 0, st, n, nbs, sflags, sig, gflags, h, nbm, sc);
}

void subgroup(hipStream_t st, int n, const uint32_t* sflags, const g2_aff* sig, uint32_t* gflags, uint32_t* exc) {
  if (!n) return;
  const char* sg = getenv("SSB_SUBGROUP");
  const bool lane_path = sg && sg[0] == 'l';  // "lane"
  if (lane_path) {
    lane_subgroup(st, n, sflags, sig, gflags, exc);
    hipLaunchKernelGGL(k_subgroup_fix, dim3((n + 63) / 64), dim3(64), 0, st, n, sflags, sig, (const uint32_t*)exc, gflags);
  } else {
    hipLaunchKernelGGL(k_subgroup, dim3((n + 63) / 64), dim3(64), 0, st, n, sflags, sig, gflags);
  }
}

}  // namespace launch
}  // namespace ssb

SSB_TRACE_READER(msm)
