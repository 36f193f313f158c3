// ssb_k_hash.hip -- kernels (gfx950): hash_to_G2 per root, batched signing, sk -> pk, serialisation.
// Launched from ssbls.hip (declarations in ssb_kernels.h); one TU per kernel family so the
// library compiles in parallel.
#include "ssb_kernels.h"
#include "ssb_wave.h"

namespace ssb {
namespace k {

__global__ void __launch_bounds__(64) k_hash_to_g2(int n, const uint8_t* __restrict__ roots, dst_arg dst,
                                                   g2_aff* __restrict__ out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t m[32];
  for (int k = 0; k < 32; ++k) m[k] = roots[32 * i + k];
  g2_aff h;
  hash_to_g2(h, m, dst.b, dst.len);
  out[i] = h;
}
__global__ void __launch_bounds__(64) k_sign(int n, const uint8_t* __restrict__ sk32le, const uint32_t* __restrict__ root_idx,
                                             const g2_aff* __restrict__ H, uint8_t* __restrict__ out96) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  for (int w = 0; w < 8; ++w) {
    const uint8_t* q = sk32le + 32 * (size_t)i + 4 * w;
    k[w] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
  }
  g2_jac r;
  jac_mul_w4(r, H[root_idx[i]], k, 8);
  g2_aff a; jac_to_aff(a, r);
  uint8_t o[96];
  g2_compress(o, a);
  for (int b = 0; b < 96; ++b) out96[96 * (size_t)i + b] = o[b];
}
__global__ void __launch_bounds__(64) k_sk_to_pk(int n, const uint8_t* __restrict__ sk32le, uint8_t* __restrict__ out48) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  for (int w = 0; w < 8; ++w) {
    const uint8_t* q = sk32le + 32 * (size_t)i + 4 * w;
    k[w] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
  }
  g1_aff g; g.x = fp_from_c(G1_GEN_X); g.y = fp_from_c(G1_GEN_Y); g.inf = 0;
  g1_jac r;
  jac_mul_w4(r, g, k, 8);
  g1_aff a; jac_to_aff(a, r);
  uint8_t o[48];
  g1_compress(o, a);
  for (int b = 0; b < 48; ++b) out48[48 * (size_t)i + b] = o[b];
}
__global__ void k_serialize_g2(int n, const g2_aff* __restrict__ pts, uint8_t* __restrict__ out192) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t o[192];
  g2_serialize(o, pts[i]);
  for (int k = 0; k < 192; ++k) out192[192 * (size_t)i + k] = o[k];
}

}  // namespace k
}  // namespace ssb
