// ssb_k_lane.hip -- the per-share verification stage as lane-group kernels (gfx950).
//
// One 64-lane workgroup holds 64/G groups; each group of G lanes works on ONE share, running the
// generated lane programs (ssb_lane_progs.h) out of LDS.  Inactive groups (tail of the grid,
// undecodable shares) run the same schedule on a harmless point and discard the result, so every
// lane of the wave executes every instruction and every barrier.
//   k_lane_subgroup  psi(P) == [x]P  (sig_groupcheck of blst verify; SSB_SUBGROUP=lane); shares whose
//                    group stage met an exceptional addition are redone by k_subgroup_fix (single lane)
#include "ssb_kernels.h"
#include "ssb_lane_ops.h"

using namespace ssb;
using namespace ssb::lane;

namespace {

constexpr int G2G = G2_ADD_G, G2NG = 64 / G2G;
constexpr int G2S0 = G2_ADD_SCRATCH > G2_MADD_SCRATCH ? G2_ADD_SCRATCH : G2_MADD_SCRATCH;

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
  __shared__ lslot lds[LP_NCODE_CONST + G2NG * SG_GS];
  __shared__ uint32_t flg[G2NG];
  const int gi = threadIdx.x / G2G, role = threadIdx.x % G2G;
  const int s = blockIdx.x * G2NG + gi;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST + gi * SG_GS, 0, 0, 0, (lu32*)&flg[gi], role};
  lp_init_consts(g);
  const bool act = s < n && (sflags[s] & DEC_OK) && !(sflags[s] & DEC_INF);
  const int P = G2S0, ACC = P + 4, TMP = ACC + 6;
  {
    const g2_aff q = act ? sig[s] : dummy_g2();
    if (role < 4) lp_put(g.s + P + role, lv_in(((const fp*)&q)[role]));
  }
  __syncthreads();
  uint32_t exc = 0;
  const bool in = g2_subgroup_check(g, P, ACC, TMP, exc);
  if (role == 0 && s < n) {
    gflags[s] = (act && in) ? DEC_IN_GROUP : 0u;
    exc_out[s] = act ? exc : 0u;
  }
}

}  // namespace

namespace ssb {
namespace launch {

void lane_subgroup(hipStream_t st, int n, const uint32_t* sflags, const g2_aff* sig, uint32_t* gflags, uint32_t* exc) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_lane_subgroup, dim3((n + G2NG - 1) / G2NG), dim3(64), 0, st, n, sflags, sig, gflags, exc);
}
}  // namespace launch
}  // namespace ssb
