// ssb_k_lane.hip -- the per-share verification stage as lane-group kernels (gfx950).
//
// One 64-lane workgroup holds 64/G groups; each group of G lanes works on ONE share, running the
// generated lane programs (ssb_lane_progs.h) out of LDS.  Inactive groups (tail of the grid,
// undecodable shares) run the same schedule on a harmless point and discard the result, so every
// lane of the wave executes every instruction and every barrier.
//   k_lane_subgroup  psi(P) == [x]P                       (sig_groupcheck of blst verify)
//   k_lane_rlc_g2    r_i * sig_i, 64-bit odd RLC scalar   (lighthouse RAND_BITS = 64, a-7)
//   k_lane_rlc_g1    r_i * pk_i
//   k_lane_fixup     exact single-lane recomputation of the rare shares whose group stage met an
//                    exceptional addition (points of small order)
#include "ssb_kernels.h"
#include "ssb_lane_ops.h"

using namespace ssb;
using namespace ssb::lane;

namespace {

constexpr int G2G = G2_ADD_G, G2NG = 64 / G2G;
constexpr int G2S0 = G2_ADD_SCRATCH > G2_MADD_SCRATCH ? G2_ADD_SCRATCH : G2_MADD_SCRATCH;
constexpr int G1G = G1_ADD_G, G1NG = 64 / G1G;
constexpr int G1S0 = G1_ADD_SCRATCH > G1_MADD_SCRATCH ? G1_ADD_SCRATCH : G1_MADD_SCRATCH;

SSB_INL g2_aff dummy_g2() {  // any curve point: the results of inactive groups are discarded
  g2_aff p;
  p.x = fp2_zero(); p.y = fp2_one(); p.inf = 0;
  return p;
}

// subgroup check: user slots P(4) acc(6) tmp(10)
constexpr int SG_GS = G2S0 + 20;
__global__ void SSB_LB(64) k_lane_subgroup(int n, const uint32_t* __restrict__ sflags,
                                                      const g2_aff* __restrict__ sig, uint32_t* __restrict__ gflags,
                                                      uint32_t* __restrict__ exc_out) {
  __shared__ fp lds[LP_NCODE_CONST + G2NG * SG_GS];
  __shared__ uint32_t flg[G2NG];
  const int gi = threadIdx.x / G2G, role = threadIdx.x % G2G;
  const int s = blockIdx.x * G2NG + gi;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST + gi * SG_GS, 0, 0, 0, (lu32*)&flg[gi], role};
  lp_init_consts(g);
  const bool act = s < n && (sflags[s] & DEC_OK) && !(sflags[s] & DEC_INF);
  const int P = G2S0, ACC = P + 4, TMP = ACC + 6;
  {
    const g2_aff q = act ? sig[s] : dummy_g2();
    if (role < 4) g.s[P + role] = ((const fp*)&q)[role];
  }
  __syncthreads();
  uint32_t exc = 0;
  const bool in = g2_subgroup_check(g, P, ACC, TMP, exc);
  if (role == 0 && s < n) {
    gflags[s] = (act && in) ? DEC_IN_GROUP : 0u;
    exc_out[s] = act ? exc : 0u;
  }
}

// RLC on G2: user slots P(4) table(48) acc(6) tmp(6)
constexpr int R2_GS = G2S0 + 64;
__global__ void SSB_LB(64) k_lane_rlc_g2(int n, uint64_t seed, const uint32_t* __restrict__ sflags,
                                                    const g2_aff* __restrict__ sig, g2_jac* __restrict__ rsig,
                                                    uint32_t* __restrict__ exc_out) {
  __shared__ fp lds[LP_NCODE_CONST + G2NG * R2_GS];
  __shared__ uint32_t flg[G2NG];
  const int gi = threadIdx.x / G2G, role = threadIdx.x % G2G;
  const int s = blockIdx.x * G2NG + gi;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST + gi * R2_GS, 0, 0, 0, (lu32*)&flg[gi], role};
  lp_init_consts(g);
  const bool act = s < n && (sflags[s] & DEC_OK) && !(sflags[s] & DEC_INF);
  const int P = G2S0, TAB = P + 4, ACC = TAB + 48, TMP = ACC + 6;
  {
    const g2_aff q = act ? sig[s] : dummy_g2();
    if (role < 4) g.s[P + role] = ((const fp*)&q)[role];
  }
  __syncthreads();
  uint32_t exc = 0;
  g2_mul_u64_odd(g, P, rlc_scalar_odd(seed, (uint64_t)(s < n ? s : 0)), TAB, ACC, TMP, exc);
  if (s < n) {
    if (act) {
      if (role < 6) ((fp*)&rsig[s])[role] = g.s[ACC + role];
    } else {
      g2_jac inf; jac_set_inf(inf);
      if (role < 6) ((fp*)&rsig[s])[role] = ((const fp*)&inf)[role];
    }
    if (role == 0) exc_out[s] = act ? exc : 0u;
  }
}

// RLC on G1: user slots P(2) table(24) acc(3) tmp(3)
constexpr int R1_GS = G1S0 + 32;
__global__ void SSB_LB(64) k_lane_rlc_g1(int n, uint64_t seed, const uint32_t* __restrict__ pflags,
                                                    const g1_aff* __restrict__ pk, g1_jac* __restrict__ rpk,
                                                    uint32_t* __restrict__ exc_out) {
  __shared__ fp lds[LP_NCODE_CONST + G1NG * R1_GS];
  __shared__ uint32_t flg[G1NG];
  const int gi = threadIdx.x / G1G, role = threadIdx.x % G1G;
  const int s = blockIdx.x * G1NG + gi;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST + gi * R1_GS, 0, 0, 0, (lu32*)&flg[gi], role};
  lp_init_consts(g);
  const bool act = s < n && (pflags[s] & DEC_OK) && !(pflags[s] & DEC_INF);
  const int P = G1S0, TAB = P + 2, ACC = TAB + 24, TMP = ACC + 3;
  {
    g1_aff q;
    if (act) q = pk[s]; else { q.x = fp_zero(); q.y = fp_one(); q.inf = 0; }
    if (role < 2) g.s[P + role] = ((const fp*)&q)[role];
  }
  __syncthreads();
  uint32_t exc = 0;
  g1_mul_u64_odd(g, P, rlc_scalar_odd(seed, (uint64_t)(s < n ? s : 0)), TAB, ACC, TMP, exc);
  if (s < n) {
    if (act) {
      if (role < 3) ((fp*)&rpk[s])[role] = g.s[ACC + role];
    } else {
      g1_jac inf; jac_set_inf(inf);
      if (role < 3) ((fp*)&rpk[s])[role] = ((const fp*)&inf)[role];
    }
    if (role == 0) exc_out[s] = act ? exc : 0u;
  }
}

__global__ void SSB_LB(64) k_lane_fixup(int n, uint64_t seed, const uint32_t* __restrict__ sflags,
                                                   const uint32_t* __restrict__ pflags, const g2_aff* __restrict__ sig,
                                                   const g1_aff* __restrict__ pk, const uint32_t* __restrict__ exc_g2,
                                                   const uint32_t* __restrict__ exc_rlc2, const uint32_t* __restrict__ exc_rlc1,
                                                   uint32_t* __restrict__ gflags, g2_jac* __restrict__ rsig,
                                                   g1_jac* __restrict__ rpk) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  if (exc_g2[s]) gflags[s] = unit_subgroup(sig[s]);
  if (exc_rlc2[s]) { g2_jac r; unit_rlc_sig(r, sig[s], rlc_scalar_odd(seed, (uint64_t)s)); rsig[s] = r; }
  if (exc_rlc1[s]) { g1_jac r; unit_rlc_pk(r, pk[s], rlc_scalar_odd(seed, (uint64_t)s)); rpk[s] = r; }
  (void)sflags; (void)pflags;
}

}  // namespace

namespace ssb {
namespace launch {

void lane_subgroup(hipStream_t st, int n, const uint32_t* sflags, const g2_aff* sig, uint32_t* gflags, uint32_t* exc) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_lane_subgroup, dim3((n + G2NG - 1) / G2NG), dim3(64), 0, st, n, sflags, sig, gflags, exc);
}
void lane_rlc_g2(hipStream_t st, int n, uint64_t seed, const uint32_t* sflags, const g2_aff* sig, g2_jac* rsig,
                 uint32_t* exc) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_lane_rlc_g2, dim3((n + G2NG - 1) / G2NG), dim3(64), 0, st, n, seed, sflags, sig, rsig, exc);
}
void lane_rlc_g1(hipStream_t st, int n, uint64_t seed, const uint32_t* pflags, const g1_aff* pk, g1_jac* rpk,
                 uint32_t* exc) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_lane_rlc_g1, dim3((n + G1NG - 1) / G1NG), dim3(64), 0, st, n, seed, pflags, pk, rpk, exc);
}
void lane_fixup(hipStream_t st, int n, uint64_t seed, const uint32_t* sflags, const uint32_t* pflags,
                const g2_aff* sig, const g1_aff* pk, const uint32_t* exc, uint32_t* gflags, g2_jac* rsig,
                g1_jac* rpk) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_lane_fixup, dim3((n + 63) / 64), dim3(64), 0, st, n, seed, sflags, pflags, sig, pk, exc,
                     exc + n, exc + 2 * n, gflags, rsig, rpk);
}

}  // namespace launch
}  // namespace ssb
