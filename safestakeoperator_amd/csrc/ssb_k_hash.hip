// ssb_k_hash.hip -- kernels (gfx950): hash_to_G2 per root, batched signing, sk -> pk, serialisation.
// Launched from ssbls.hip (declarations in ssb_kernels.h); one TU per kernel family so the
// library compiles in parallel.
#include "ssb_kernels.h"
#include "ssb_blocks.h"

namespace ssb {
namespace k {

// ---- staged hash_to_G2 (the RFC 9380 hash_to_curve of ssb_h2c.h, split into stages) ----
// 1: expand_message_xmd + the two field elements, one lane per root (message i: 32 bytes, or
// lens[i] <= 32 bytes at roots + 32 i when lens is given)
__global__ void SSB_LB(64) k_h2c_u(int n, const uint8_t* __restrict__ roots, const uint8_t* __restrict__ lens, dst_arg dst,
                                   fp2* __restrict__ u) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t m[32];
  for (int k = 0; k < 32; ++k) m[k] = roots[32 * i + k];
  const int len = lens ? (lens[i] < 32 ? lens[i] : 32) : 32;
  fp2 u0, u1;
  h2c_field(u0, u1, m, dst.b, dst.len, len);
  u[2 * i] = u0;
  u[2 * i + 1] = u1;
}

// 2: simplified SWU (h2c_map_block, ssb_blocks.h), 16 roots per block
__global__ void SSB_LB(64) k_h2c_map(int n, const fp2* __restrict__ u, g2_aff* __restrict__ q) {
  __shared__ h2c_cand cs[64];
  h2c_map_block(blockIdx.x, cs, n, u, q);
}

// 3: q0 + q1 and the cofactor clearing (h2c_clear_block, ssb_blocks.h)
__global__ void SSB_LB(64) k_h2c_clear(int n, const g2_aff* __restrict__ q, g2_jac* __restrict__ hj,
                                                  uint32_t* __restrict__ exc_out) {
  __shared__ lane::lslot lds[H2C_CLEAR_LDS / sizeof(lane::lslot) + 1];
  h2c_clear_block(blockIdx.x, lds, n, q, hj, exc_out);
}

// 4: affine output (h2c_affine_block, ssb_blocks.h)
__global__ void SSB_LB(64) k_h2c_affine(int n, const g2_aff* __restrict__ q, g2_jac* __restrict__ hj,
                                                   const uint32_t* __restrict__ exc, int exact_all, g2_aff* __restrict__ out) {
  h2c_affine_block(blockIdx.x, n, q, hj, exc, exact_all, out);
}

__global__ void SSB_LB(64) k_sign(int n, const uint8_t* __restrict__ sk32le, const uint32_t* __restrict__ root_idx,
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
__global__ void SSB_LB(64) k_sk_to_pk(int n, const uint8_t* __restrict__ sk32le, uint8_t* __restrict__ out48) {
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
// bls::PublicKey::deserialize + serialize (lighthouse -> blst key_validate): decode, not infinity,
// in G1 ([r]P == O, registration-time work, the plain windowed multiplication); valid[i] = 1 and the
// recompression in out48, else valid[i] = 0 and zeros.  Pinned by the keys the reference's own
// sources deserialize (tests/golden/reference_kats.json).
__global__ void SSB_LB(64) k_pk_validate(int n, const uint8_t* __restrict__ pk48, uint8_t* __restrict__ valid,
                                         uint8_t* __restrict__ out48) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t b[48];
  for (int k = 0; k < 48; ++k) b[k] = pk48[48 * (size_t)i + k];
  g1_aff a;
  const uint32_t f = unit_decode_pk(a, b);
  bool ok = (f & DEC_OK) && !(f & DEC_INF);
  if (ok) {
    g1_jac z;
    jac_mul_w4(z, a, R_LIMBS, 8);
    ok = f_is_zero(z.z);
  }
  uint8_t o[48];
  if (ok) g1_compress(o, a);
  else for (int k = 0; k < 48; ++k) o[k] = 0;
  valid[i] = ok ? 1 : 0;
  for (int k = 0; k < 48; ++k) out48[48 * (size_t)i + k] = o[k];
}
__global__ void k_serialize_g2(int n, const g2_aff* __restrict__ pts, uint8_t* __restrict__ out192) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t o[192];
  g2_serialize(o, pts[i]);
  for (int k = 0; k < 192; ++k) out192[192 * (size_t)i + k] = o[k];
}

}  // namespace k

namespace launch {
size_t hash_ws_bytes(size_t n) { return n * (2 * sizeof(fp2) + 2 * sizeof(g2_aff) + sizeof(g2_jac) + 4) + 1024; }
h2c_ws carve_h2c(void* ws, size_t n) {
  char* p = (char*)ws;
  auto take = [&](size_t b) { char* r = p; p += (b + 255) & ~(size_t)255; return r; };
  h2c_ws w;
  w.u = (fp2*)take(2 * n * sizeof(fp2));
  w.q = (g2_aff*)take(2 * n * sizeof(g2_aff));
  w.hj = (g2_jac*)take(n * sizeof(g2_jac));
  w.exc = (uint32_t*)take(n * 4);
  return w;
}
int h2c_exact_all() {
  const char* ex = getenv("SSB_H2C_EXACT");
  return (ex && atoi(ex) != 0) ? 1 : 0;
}
void h2c_u(hipStream_t st, int n, const uint8_t* roots, const dst_arg& dst, const h2c_ws& w, const uint8_t* lens) {
  hipLaunchKernelGGL(k::k_h2c_u, dim3((n + 63) / 64), dim3(64), 0, st, n, roots, lens, dst, w.u);
}
void hash_to_g2(hipStream_t st, int n, const uint8_t* roots, const dst_arg& dst, g2_aff* out, void* ws, const uint8_t* lens) {
  if (n <= 0) return;
  const h2c_ws w = carve_h2c(ws, (size_t)n);
  h2c_u(st, n, roots, dst, w, lens);
  hipLaunchKernelGGL(k::k_h2c_map, dim3((4 * n + 63) / 64), dim3(64), 0, st, n, (const fp2*)w.u, w.q);
  hipLaunchKernelGGL(k::k_h2c_clear, dim3((n + 7) / 8), dim3(64), 0, st, n, (const g2_aff*)w.q, w.hj, w.exc);
  hipLaunchKernelGGL(k::k_h2c_affine, dim3((n + 63) / 64), dim3(64), 0, st, n, (const g2_aff*)w.q, w.hj,
                     (const uint32_t*)w.exc, h2c_exact_all(), out);
}
}  // namespace launch
}  // namespace ssb
