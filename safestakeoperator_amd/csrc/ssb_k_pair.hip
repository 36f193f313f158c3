// ssb_k_pair.hip -- kernels (gfx950): wave-cooperative Miller loops and the final exponentiation.
// Launched from ssbls.hip (declarations in ssb_kernels.h); one TU per kernel family so the
// library compiles in parallel.
#include "ssb_kernels.h"
#include "ssb_wave.h"

namespace ssb {
namespace k {

constexpr int WAVE_MILLER_SLOTS = wave::S_USER + 30;
__global__ void __launch_bounds__(64) k_miller_wave(int n_roots, const g1_aff* __restrict__ root_sum,
                                                    const g2_aff* __restrict__ H, const g2_aff* __restrict__ sig_sum,
                                                    fp12* __restrict__ f) {
  __shared__ fp slots[WAVE_MILLER_SLOTS];
  const int p = blockIdx.x, lane = threadIdx.x;
  g1_aff P; g2_aff Q;
  if (p < n_roots) { P = root_sum[p]; Q = H[p]; } else { P = g1_neg_generator(); Q = *sig_sum; }
  if (P.inf || Q.inf) {  // e(O, Q) = e(P, O) = 1  (uniform per workgroup)
    if (lane == 0) f[p] = fp12_one();
    return;
  }
  wave::ws w{slots};
  wave::init(w, lane, 64);
  const int B = wave::S_USER;
  if (lane == 0) {
    slots[B + 24] = Q.x.c0; slots[B + 25] = Q.x.c1; slots[B + 26] = Q.y.c0; slots[B + 27] = Q.y.c1;
    slots[B + 28] = P.x; slots[B + 29] = P.y;
  }
  __syncthreads();
  wave::miller(w, B, lane, 64);
  if (lane == 0) { fp12 r; wave::load12(r, w, B); f[p] = r; }
}
constexpr int WAVE_FINAL_SLOTS = wave::S_USER + 12 * 10;
__global__ void __launch_bounds__(64) k_final_wave(int npairs, const fp12* __restrict__ f, uint32_t* __restrict__ ok) {
  __shared__ fp slots[WAVE_FINAL_SLOTS];
  const int lane = threadIdx.x;
  wave::ws w{slots};
  wave::init(w, lane, 64);
  const int ACC = wave::S_USER, IN = ACC + 12, TMP = ACC + 24;
  if (lane == 0) wave::store12(w, ACC, f[0]);
  __syncthreads();
  for (int i = 1; i < npairs; ++i) {
    if (lane == 0) wave::store12(w, IN, f[i]);
    __syncthreads();
    wave::run(w, wave::FP12_MUL, ACC, IN, ACC, lane, 64);
  }
  wave::final_exp(w, ACC, TMP, lane, 64);
  if (lane == 0) { fp12 e; wave::load12(e, w, ACC); *ok = fp12_is_one(e) ? 1u : 0u; }
}

}  // namespace k
}  // namespace ssb
