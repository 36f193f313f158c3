// ssb_kernels.h -- host-side launchers of the kernels that live in their own translation units
// (compiled in parallel, linked into libssbls.so).  Internal to the library: not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include "ssb_units.h"
#include "../../include/ssbls.h"

// The roles of a fused launch (its block ranges running different stages) stay inlined: out of line
// (SSB_VARIANT_DEFS=-DSSB_ROLES_OUTLINE, an experiment build) each role has its own register
// allocation and the subgroup lanes' loop spills drop, but the roles' argument structs go through
// scratch at every call and the measured HBM writes grew (round 4 PMC, profiles/r04_pmc_*.json:
// k_subgroup_map 155 -> 212 MB, k_decode_count 552 -> 635 MB per roofline launch).
#ifdef SSB_ROLES_OUTLINE
#define SSB_ROLE SSB_FN
#else
#define SSB_ROLE SSB_INL
#endif

// Experiment builds only (SSB_VARIANT_DEFS=-DSSB_TRACE_TAIL, bench_tools/trace_tail.py): the tail
// kernels record per-block start / end wall-clock stamps (100 MHz) in a device buffer of their
// translation unit (read back by ssb_debug_trace_<tu>), so the critical path inside a fused launch
// can be read without perturbing it; the product library compiles these to nothing.
#ifdef SSB_TRACE_TAIL
enum { TR_W2_G2 = 1, TR_W2_G1, TR_W2_HORNER, TR_W2_CLEAR, TR_W2_AFFINE, TR_MF_MILLER, TR_MF_GROUP, TR_MF_PRODUCT, TR_MF_FINAL,
       TR_EX_ITEM, TR_EX_GCOMB, TR_EX_GCHECK, TR_EX_SINGLE, TR_EX_PAIR, TR_EX_FINAL, TR_EX_ROOTPAIR, TR_EX_QSUM };
static __device__ unsigned long long ssb_trace_buf[4 * 2048];
static __device__ unsigned int ssb_trace_n;
#define SSB_TRACE_T0() const unsigned long long trace_t0_ = wall_clock64()
#define SSB_TRACE(tag)                                                                      \
  do {                                                                                      \
    if (threadIdx.x == 0) {                                                                 \
      const unsigned i_ = atomicAdd(&ssb_trace_n, 1u) & 2047u;                              \
      ssb_trace_buf[4 * i_] = (tag); ssb_trace_buf[4 * i_ + 1] = blockIdx.x;                \
      ssb_trace_buf[4 * i_ + 2] = trace_t0_; ssb_trace_buf[4 * i_ + 3] = wall_clock64();    \
    }                                                                                       \
  } while (0)
#define SSB_TRACE_READER(tu)                                                                \
  extern "C" int ssb_debug_trace_##tu(unsigned long long* out) {                            \
    unsigned int n = 0, z = 0;                                                              \
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(ssb_trace_n), 4) != hipSuccess) return -1;       \
    if (n > 2048) n = 2048;                                                                 \
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ssb_trace_buf), 32 * (size_t)n) != hipSuccess) return -1; \
    hipMemcpyToSymbol(HIP_SYMBOL(ssb_trace_n), &z, 4);                                      \
    return (int)n;                                                                          \
  }
#else
#define SSB_TRACE_T0() ((void)0)
#define SSB_TRACE(tag) ((void)0)
#define SSB_TRACE_READER(tu)
#endif

namespace ssb {

// DST passed by value to the hashing kernels
struct dst_arg { uint8_t b[SSB_MAX_DST + 1]; int len; };

// The a-1 scan + combine of a batch's jobs, run speculatively from the candidate flags (the
// one-stream path runs it beside the Miller loops; the exact pass on the verdicts follows only if
// the batch check failed)
struct spec_jobs {
  int n_jobs; uint32_t n_shares; const uint32_t* off; const uint32_t* tt; const uint64_t* ids; const uint32_t* flags;
  uint32_t* sel; int32_t* status; uint64_t* err; const g2_aff* sig_aff; uint32_t* fast; uint8_t* out96; fr* lam;
  uint32_t ratio;  // 1: jobs whose lambda_i are ratios of small integers are marked for k_combine_ratio (fast 2)
  int32_t* wst;    // the wire-record path: per-share record status, undecodable shares absent (select_job)
};

// the ratio combine's arguments riding in k_combine_terms_gls (phase T, blocks past nbt) and
// k_combine_sum (phase K): the jobs' ids, the per-job table regions, the per-job T
struct ratio_args { const uint64_t* ids; uint8_t* tabs; g2_jac* rT; uint64_t* rk; uint32_t nbt;
                    const g2_aff* sig; uint32_t exact; };
// k_combine_sum's extra blocks, per 64-job wave: one per fast-3 job a wave can hold (ratio jobs in a
// wave with fewer than RATIO_MIN_JOBS of them -- ssb_blocks.h -- run on lane groups, one workgroup each)
constexpr unsigned RATIO_LANE_PER_WAVE = 15;

// share -> (job, root) of an aggregate batch (share_lookup, ssb_blocks.h)
struct job_map {
  int n_jobs; uint32_t n_shares; const uint32_t* off; const uint32_t* tt; const uint32_t* job_root;
  uint32_t* share_job; uint32_t* share_root;
};

// One bucket MSM of the RLC sums (ssb_k_msm.hip): c-bit windows, W = ceil(64 / c) of them,
// `ngroups` independent sums; bucket key = base + ((group * W + window) << c) + digit.
// merged (the G1 side with the public-key cache's precomputed bases [2^(c w)] pk, c = 4, W = 16):
// every window of a group shares ONE set of buckets, key = base + (group << c) + digit, and the
// entry carries its window (entry = share << 4 | window): the digit d of window w adds
// [2^(c w)] pk_i to bucket d, so sum_d d B_d is the whole sum -- no per-window sums, no Horner.
struct msm_cfg { uint32_t c, W, base, ngroups, merged; };
SSB_INL uint32_t msm_nbuckets(const msm_cfg& c) { return (c.merged ? c.ngroups : c.ngroups * c.W) << c.c; }
constexpr uint32_t PKPOW_W = 16;   // precomputed bases per cached public key ([2^(4 w)] pk, w < 16)

namespace k {
constexpr int SUM_THREADS = 128;   // k_sum_* block size
constexpr int SEG_THREADS = 64;    // k_sum_seg block size
__global__ void k_root_hist(int n, int n_roots, const uint32_t* __restrict__ share_root, uint32_t* __restrict__ cnt);
__global__ void k_root_scan(int n_roots, const uint32_t* __restrict__ cnt, uint32_t* __restrict__ start,
                            uint32_t* __restrict__ cursor);
__global__ void k_root_scatter(int n, int n_roots, const uint32_t* __restrict__ share_root, uint32_t* __restrict__ cursor,
                               uint32_t* __restrict__ perm);
// rpk[s] = rlc_scalar_odd(key, s) * pk[s] for every decodable share (infinity otherwise)
__global__ void k_rlc_pk(int n, rlc_key key, const uint32_t* __restrict__ sflags, const uint32_t* __restrict__ pflags,
                         const g1_aff* __restrict__ pk_aff, g1_jac* __restrict__ rpk);
__global__ void k_sum_seg(int n_roots, const uint32_t* __restrict__ start, const uint32_t* __restrict__ cnt,
                          const uint32_t* __restrict__ perm, const uint32_t* __restrict__ flags,
                          const g1_jac* __restrict__ rpk, const g2_jac* __restrict__ rsig, g1_aff* __restrict__ s1,
                          g2_aff* __restrict__ s2);

__global__ void k_share_map(int n_jobs, uint32_t n_shares, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                            const uint32_t* __restrict__ job_root, uint32_t* __restrict__ share_job,
                            uint32_t* __restrict__ share_root);
__global__ void k_decode(int n, const uint8_t* __restrict__ sig96,
                                               const uint8_t* __restrict__ pk48, int group_check,
                                               g2_aff* __restrict__ sig_aff, g1_aff* __restrict__ pk_aff,
                                               uint32_t* __restrict__ flags);
__global__ void k_decode2(int n, const uint8_t* __restrict__ sig96, const uint8_t* __restrict__ pk48,
                                                g2_aff* __restrict__ sig_aff, g1_aff* __restrict__ pk_aff,
                                                uint32_t* __restrict__ sflags, uint32_t* __restrict__ pflags);
__global__ void k_decode_sig(int n, const uint8_t* __restrict__ sig96, g2_aff* __restrict__ sig_aff,
                             uint32_t* __restrict__ sflags);
__global__ void k_pk_gather(int n, const uint32_t* __restrict__ pk_index, uint32_t n_cache,
                            const g1_aff* __restrict__ cache_aff, const uint32_t* __restrict__ cache_flags,
                            g1_aff* __restrict__ pk_aff, uint32_t* __restrict__ pflags);
__global__ void k_pk_pow(int n, const g1_aff* __restrict__ pk_aff, const uint32_t* __restrict__ pflags,
                         g1_aff* __restrict__ pow);
__global__ void k_decode_pk(int n, const uint8_t* __restrict__ pk48, g1_aff* __restrict__ pk_aff,
                            uint32_t* __restrict__ pflags);
__global__ void k_flags(int n, const uint32_t* __restrict__ sflags, const uint32_t* __restrict__ pflags,
                        const uint32_t* __restrict__ gflags, const uint32_t* __restrict__ share_root, uint32_t n_roots,
                        uint32_t* __restrict__ flags);

__global__ void k_fallback_lane(int n, const uint32_t* __restrict__ ok, const uint32_t* __restrict__ flags,
                                const uint32_t* __restrict__ share_root, const g2_aff* __restrict__ H,
                                const g2_aff* __restrict__ sig_aff, const g1_aff* __restrict__ pk_aff,
                                uint8_t* __restrict__ verdict);
// (blocks [npairs, ..): the speculative a-1 scan + combine of sj's jobs, 64 per block)
__global__ void k_miller_pairs(int npairs, const g1_aff* __restrict__ P, const g2_aff* __restrict__ Q,
                               fp12* __restrict__ f, spec_jobs sj);
__global__ void k_fp12_prod8(int n, const fp12* __restrict__ in, fp12* __restrict__ out);
// Miller loops + product tree + final exponentiation in one launch (fused one-stream path):
// tk: 1 + ceil(npairs / 8) completion tickets (zero on entry, zero again on exit); f: npairs +
// ceil(npairs / 8) + 1 values (the last: the product before the final exponentiation)
__global__ void k_miller_final(int npairs, const g1_aff* __restrict__ P, const g2_aff* __restrict__ Q,
                               fp12* __restrict__ f, spec_jobs sj, uint32_t* __restrict__ tk, uint32_t* __restrict__ ok);
__global__ void k_final_lane(int n, const fp12* __restrict__ in, uint32_t* __restrict__ ok, int nv,
                             const uint32_t* __restrict__ flags, uint8_t* __restrict__ verdict);
__global__ void k_sign(int n, const uint8_t* __restrict__ sk32le, const uint32_t* __restrict__ root_idx,
                                             const g2_aff* __restrict__ H, uint8_t* __restrict__ out96);
__global__ void k_sk_to_pk(int n, const uint8_t* __restrict__ sk32le, uint8_t* __restrict__ out48);
__global__ void k_serialize_g2(int n, const g2_aff* __restrict__ pts, uint8_t* __restrict__ out192);
__global__ void k_pk_validate(int n, const uint8_t* __restrict__ pk48, uint8_t* __restrict__ valid,
                              uint8_t* __restrict__ out48);
__global__ void k_select(int n_jobs, uint32_t n_shares, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                         const uint64_t* __restrict__ ids, const uint8_t* __restrict__ verdict,
                         const uint32_t* __restrict__ flags, const uint32_t* __restrict__ skip_if_ok,
                         uint32_t* __restrict__ sel, int32_t* __restrict__ status, uint64_t* __restrict__ err);
__global__ void k_select_all(int n_jobs, const uint32_t* __restrict__ off, const uint32_t* __restrict__ flags,
                             uint32_t* __restrict__ sel, uint32_t* __restrict__ tt, int32_t* __restrict__ status,
                             uint64_t* __restrict__ err);
__global__ void k_lagrange(int n_jobs, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                           const uint64_t* __restrict__ ids, const uint32_t* __restrict__ sel,
                           const int32_t* __restrict__ status, const uint32_t* __restrict__ skip_if_ok,
                           const uint32_t* __restrict__ fast, fr* __restrict__ lam);
__global__ void k_combine_terms(int n, uint32_t n_jobs, const uint32_t* __restrict__ share_job,
                                                      const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                                                      const int32_t* __restrict__ status, const uint32_t* __restrict__ sel,
                                                      const fr* __restrict__ lam, const g2_aff* __restrict__ sig_aff,
                                                      const uint32_t* __restrict__ skip_if_ok, const uint32_t* __restrict__ fast,
                                                      g2_jac* __restrict__ term);
__global__ void k_combine_terms_gls(int n, uint32_t n_jobs, const uint32_t* __restrict__ share_job, const uint32_t* __restrict__ off,
                                    const uint32_t* __restrict__ tt, const int32_t* __restrict__ status,
                                    const uint32_t* __restrict__ sel, const fr* __restrict__ lam,
                                    const g2_aff* __restrict__ sig_aff, const uint32_t* __restrict__ skip_if_ok,
                                    const uint32_t* __restrict__ fast, g2_jac* __restrict__ term, ratio_args ra);
__global__ void k_combine_sum(int n_jobs, const uint32_t* __restrict__ off,
                                                    const uint32_t* __restrict__ tt, const int32_t* __restrict__ status,
                                                    const g2_jac* __restrict__ term, const uint32_t* __restrict__ skip_if_ok,
                                                    const uint32_t* __restrict__ fast, uint8_t* __restrict__ out96, int stride,
                                                    const uint32_t* __restrict__ sel, ratio_args ra);
__global__ void k_select_combine(int n_jobs, uint32_t n_shares, const uint32_t* __restrict__ off,
                                 const uint32_t* __restrict__ tt, const uint64_t* __restrict__ ids,
                                 const uint8_t* __restrict__ verdict, const uint32_t* __restrict__ flags,
                                 const uint32_t* __restrict__ skip_if_ok, uint32_t* __restrict__ sel,
                                 int32_t* __restrict__ status, uint64_t* __restrict__ err,
                                 const g2_aff* __restrict__ sig_aff, uint32_t* __restrict__ fast,
                                 uint8_t* __restrict__ out96, fr* __restrict__ lam, uint32_t ratio,
                                 int32_t* __restrict__ wst);
__global__ void k_combine_fast(int n_jobs, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                               const int32_t* __restrict__ status, const uint32_t* __restrict__ sel,
                               const uint64_t* __restrict__ ids, const g2_aff* __restrict__ sig_aff,
                               const uint32_t* __restrict__ skip_if_ok, uint32_t* __restrict__ fast,
                               uint8_t* __restrict__ out96);
__global__ void k_copy_u8(int n, const uint8_t* __restrict__ a, uint8_t* __restrict__ b);
__global__ void k_hold(const uint32_t* flag, uint32_t max_polls);

}  // namespace k

namespace launch {

// Lane-group kernels (ssb_k_lane.hip), one group of lanes per share.
//   gflags[s] = DEC_IN_GROUP if sig[s] passes psi(P) == [x]P (only for decodable, non-infinity
//   signatures: sflags[s] has DEC_OK and not DEC_INF);  exc[s] |= 1 when an addition was
//   exceptional (the share is then recomputed by the exact single-lane fallback).
void lane_subgroup(hipStream_t st, int n, const uint32_t* sflags, const g2_aff* sig, uint32_t* gflags, uint32_t* exc);
// staged hash_to_G2 of n roots into out (ssb_k_hash.hip); ws: hash_ws_bytes(n) device bytes
size_t hash_ws_bytes(size_t n);
// the staged hash's workspace (u, the SWU points q, the cleared Jacobian points hj, exc flags)
struct h2c_ws { fp2* u; g2_aff* q; g2_jac* hj; uint32_t* exc; };
h2c_ws carve_h2c(void* ws, size_t n);
int h2c_exact_all();
void h2c_u(hipStream_t st, int n, const uint8_t* roots, const dst_arg& dst, const h2c_ws& w, const uint8_t* lens = nullptr);
// (lens: per-message lengths <= 32, or nullptr for 32-byte roots)
void hash_to_g2(hipStream_t st, int n, const uint8_t* roots, const dst_arg& dst, g2_aff* out, void* ws,
                const uint8_t* lens = nullptr);
// RLC sums as bucket MSMs (ssb_k_msm.hip).  msm_sort: counting sort of the (share, window)
// entries of both MSMs by bucket key (K keys; cnt/start/cur: K words, bsum: 1024 words, ent: one
// word per entry).  msm_g2: window sums of sum_i k_i sig_i as multi-pairing pairs
// (pair_q[w] = W_w affine, pair_p[w] = [2^(c w)](-g1)).  msm_g1: root_sum[r] = sum_{i in r} k_i pk_i.
void msm_sort(hipStream_t st, int n, const rlc_key& key, const uint32_t* sflags, const uint32_t* pflags,
              const uint32_t* share_root, const msm_cfg& c2, const msm_cfg& c1, uint32_t K, uint32_t* cnt,
              uint32_t* start, uint32_t* cur, uint32_t* bsum, uint32_t* ent, uint32_t* order);
void msm_g2(hipStream_t st, const msm_cfg& c, int lj, const uint32_t* order, const uint32_t* start, const uint32_t* cnt, const uint32_t* ent,
            const uint32_t* flags, const g2_aff* sig, g2_jac* bsum, g2_aff* pair_q, g1_aff* pair_p,
            const g1_aff* negg1_pow);
void msm_g1(hipStream_t st, const msm_cfg& c, int lj, const uint32_t* order, const uint32_t* start, const uint32_t* cnt, const uint32_t* ent,
            const uint32_t* flags, const g1_aff* pk, g1_jac* bsum, g1_jac* wsum, g1_aff* root_sum);
// gflags[s] = DEC_IN_GROUP when signature s (decodable, not infinity) passes psi(P) == [x]P
// subgroup checks: single-lane (default) or SSB_SUBGROUP=lane (8-lane groups + exact redo of exceptional shares)
// msm_g2 + msm_g1 as three launches on one stream (bucket sums of both sides, window sums of both
// sides, the G1 Horner): the two MSMs overlap on the device.  Only with G1 windows of <= 16
// buckets (msm_fused_ok).  With hw (the staged hash's
// workspace, after h2c_u and subgroup_map's SWU map), the cofactor clearing rides along the
// bucket sums and the affine output H[0..n_roots) along the window sums.
bool msm_fused_ok(const msm_cfg& c1);
void msm_both(hipStream_t st, const msm_cfg& c2, int lj2, const msm_cfg& c1, int lj1, const uint32_t* order,
              const uint32_t* start, const uint32_t* cnt, const uint32_t* ent, const uint32_t* flags, const g2_aff* sig,
              const g1_aff* pk, g2_jac* b2, g1_jac* b1, g2_aff* pair_q, g1_aff* pair_p, const g1_aff* negg1_pow,
              g1_jac* wsum1, g1_aff* root_sum, const h2c_ws* hw = nullptr, int n_roots = 0, g2_aff* H = nullptr,
              uint32_t* tickets = nullptr, const g1_aff* pk_pow = nullptr, const uint32_t* pk_index = nullptr,
              bool lat = false);
// (lat: one batch in flight -- the latency forms of the bucket and window launches, ssb_k_msm.hip)
// (c1.merged: the G1 side reads the cached keys' precomputed bases pk_pow[pk_index[share] * PKPOW_W + window])
// (with tickets: the G1 Horner and the affine H(root) run in the window launch's last G1-window /
// last clearing block instead of a launch of their own)
// The counting sort of the MSM entries in two launches that ride along the batch's kernels
// (one-stream slots, K <= FUSED_SORT_KMAX keys): the count pass beside the decode
// (decode_count, whose last count block also runs the scans and the bucket order), the scatter beside
// the subgroup checks (subgroup_map).  Every share with an in-range root gets entries (the decode
// flags are not known yet); the bucket sums skip the non-candidates, as they do for the others.
constexpr uint32_t FUSED_SORT_KMAX = 65536;
struct fused_sort {
  rlc_key key; const uint32_t* share_root; msm_cfg c2, c1; uint32_t K;
  uint32_t* cnt; uint32_t* start; uint32_t* cur; uint32_t* ent; uint32_t* order;
  const uint32_t* pflags; uint32_t n_roots; uint32_t* flags;
  uint32_t* tickets;   // ntk words, zeroed by prep_fused: [0] count blocks done, [1] G1 windows, [2] clears,
                       // [4 ..) k_miller_final's groups
  uint32_t ntk;
  // jobs given (aggregate path): decode_count computes share -> (job, root) itself, writing
  // jm.share_job / jm.share_root (== share_root above) -- no k_share_map launch in front of the batch
  job_map jm;
};
// the subgroup checks with (hw != nullptr) the hash's SWU map of n_roots roots and (fs != nullptr)
// the sort's scatter in the same launch; with fs the lanes also write the combined share flags
void subgroup_map(hipStream_t st, int n, const uint32_t* sflags, const g2_aff* sig, uint32_t* gflags, const h2c_ws* hw,
                  int n_roots, const fused_sort* fs = nullptr);
// zero the sort's counts + the hash's first stage (expand_message_xmd) of n_roots roots
void prep_fused(hipStream_t st, const fused_sort& fs, int n_roots, const uint8_t* roots, const dst_arg& dst, const h2c_ws& hw);
// decode (signatures; public keys decoded or gathered from the cache) + the sort's count pass; the
// last count block to finish scans the counts (start, cursor) and orders the buckets
// (with dst and hw: the hash's first stage of n_roots roots rides along -- the slot's counts and
// tickets were left clean by its previous batch, so no prep launch runs in front)
void decode_count(hipStream_t st, int n, const uint8_t* sig96, const uint8_t* pk48, const uint32_t* pk_index,
                  uint32_t n_cache, const g1_aff* cache_aff, const uint32_t* cache_flags, g2_aff* sig_aff, g1_aff* pk_aff,
                  uint32_t* sflags, uint32_t* pflags, const fused_sort& fs, int n_roots = 0, const uint8_t* roots = nullptr,
                  const dst_arg* dst = nullptr, const h2c_ws* hw = nullptr);
// (the exclusive scan of the counts and the bucket order run in decode_count's last count block)
void subgroup(hipStream_t st, int n, const uint32_t* sflags, const g2_aff* sig, uint32_t* gflags, uint32_t* exc);
// Exact verdicts of a failed batch by group testing on a 16-ary tree of root-aligned share groups
// (ssb_k_bisect.hip); no-op when *ok.  froot: the batch check's Miller values, f[r] = e(PK_r, H(r))
// before the final exponentiation for r < n_roots.  Workspace (fb_ws): cnt/start/cursor/rtk n_roots
// words, perm n words, k64 n scalars, X 4 n_roots points, gst fallback_levels(n) * (n_roots + 1)
// words, rsig/rpk n points, gv0/gv1 n + n_roots bytes, nfail one word.
struct fb_ws {
  uint32_t *cnt, *start, *cursor, *perm, *gst, *rtk, *nfail;
  uint64_t* k64;
  g2_jac* X;
  g2_jac* rsig;
  g1_jac* rpk;
  uint8_t *gv0, *gv1;
  // the committee stage (aggregate batches on the fused path; all null otherwise): slist n words,
  // fex ex_pairs(n_roots) values, ftot = the batch check's Miller product before the final exponentiation
  // (k_miller_final), nS / xtk: two words of the slot's ticket block (zero on entry, zeroed again
  // by their consumers), xok one word
  uint32_t *slist, *nS, *xtk, *xok;
  fp12* fex;
  const fp12* ftot;
  uint32_t *kcnt, *kstart;   // per (root, id bucket) key: fb_keys(n_roots) words each (cursor too)
  const g1_aff* negg1_pow;   // [2^s](-g1), s < 64 (the exclusion check pairs quarter q of X with [2^16q] g1)
  uint32_t* klist;   // the non-empty keys in key order, their count at [fb_keys(n_roots)] (group-test items)
};
// the exclusion check's Fp12 values: one per quarter of every root's E_r, then one per quarter of
// every part of X (the suspect list cut into up to EX_X_PARTS slices; k_fb_excl's pair blocks, in
// that order)
constexpr int EX_X_PARTS = 16;
constexpr int ex_pairs(int n_roots) { return 4 * n_roots + 4 * EX_X_PARTS; }
// the jobs of an aggregate batch (share_off, t, ids), for the committee stage of the fallback
struct fb_jobs { int n_jobs; const uint32_t* off; const uint32_t* tt; const uint64_t* ids; };
int fallback_log2_branch();
int fallback_levels(size_t n);
// operator-id buckets per root of the failed-batch sort (fb_prep_block): 16 while the keys stay few
SSB_INL int fb_nbuckets(int n_roots) { return n_roots <= 1024 ? 16 : 1; }
inline size_t fb_keys(size_t n_roots) { return n_roots * (size_t)fb_nbuckets((int)n_roots); }
void fallback_bisect(hipStream_t st, int n, int n_roots, const rlc_key& key, const uint32_t* ok, uint32_t* flags,
                     const uint32_t* share_root, const g2_aff* H, const g2_aff* sig, const g1_aff* pk, const fp12* froot,
                     const fb_ws& fw, uint8_t* verdict, bool fast_verdicts, const fb_jobs& jobs);
// first use of a new queue: acquire its scratch for the largest slot kernel while the other queues
// are idle (ssb_k_combine.hip); synchronous, 0 on success
int prime_queue(hipStream_t st);
// wire-format records bincode(bls::Signature) -> 96-byte compressed signatures (ssb_k_wire.hip)
constexpr size_t WIRE_SIG_BYTES = 202;
// check_point: status 4 for bytes that do not decompress (ssb_decode_wire_sigs); 0: format and hex
// only (the aggregate's wire path, whose decode stage decompresses anyway -- select_job marks 4)
void wire_sig(hipStream_t st, int n, const uint8_t* wire, size_t stride, uint8_t* out96, int32_t* status,
              int check_point = 1);
// DKG share verification (ssb_k_dkg.hip): verdict[i] = ([s_i]h == sum_k [x_i^k] C_{i,k})
void feldman_share(hipStream_t st, int n, int t, const uint8_t* comm48, const uint64_t* x, const uint8_t* s32le,
                   const g1_aff* h, const uint32_t* hflags, uint8_t* verdict);
// DLEQ verification (ssb_k_dkg.hip): pts48 = n x (x1, y1, x2, y2) compressed, c32 / r32 LE scalars
void dleq_verify(hipStream_t st, int n, const uint8_t* pts48, const uint8_t* c32, const uint8_t* r32, uint8_t* verdict);

}  // namespace launch
}  // namespace ssb
