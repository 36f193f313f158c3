// ssb_k_hash.hip -- kernels (gfx950): hash_to_G2 per root, batched signing, sk -> pk, serialisation.
// Launched from ssbls.hip (declarations in ssb_kernels.h); one TU per kernel family so the
// library compiles in parallel.
#include "ssb_kernels.h"
#include "ssb_lane_ops.h"

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

// 2: simplified SWU, one lane per (root, u_j, candidate x1 / x2): both square roots run at once
// instead of one after the other; then the 3-isogeny.  Lanes 4i+2j+c, 16 roots per block.
__global__ void SSB_LB(64) k_h2c_map(int n, const fp2* __restrict__ u, g2_aff* __restrict__ q) {
  struct cand_t { fp2 x, y; uint32_t ok; };
  __shared__ cand_t cs[64];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = t >> 2, j = (t >> 1) & 1, c = t & 1;
  const bool act = i < n;
  fp2 uu = act ? u[2 * i + j] : fp2_one();
  fp2 x, y;
  const bool ok = sswu_candidate(x, y, uu, c);
  cs[threadIdx.x].x = x; cs[threadIdx.x].y = y; cs[threadIdx.x].ok = ok ? 1u : 0u;
  __syncthreads();
  if (act && c == 0) {
    const cand_t o = cs[threadIdx.x + 1];
    g2_aff r;
    sswu_finish(r, uu, ok ? x : o.x, ok ? y : o.y);
    q[2 * i + j] = r;
  }
}

// 3: q0 + q1 and the cofactor clearing as lane-group programs (8 lanes per root)
constexpr int H2C_S0 = lane::G2_ADD_SCRATCH > lane::G2_MADD_SCRATCH ? lane::G2_ADD_SCRATCH : lane::G2_MADD_SCRATCH;
constexpr int H2C_GS = H2C_S0 + 6 + 4 + 6 + 30;
__global__ void SSB_LB(64) k_h2c_clear(int n, const g2_aff* __restrict__ q, g2_jac* __restrict__ hj,
                                                  uint32_t* __restrict__ exc_out) {
  using namespace ssb::lane;
  __shared__ fp lds[LP_NCODE_CONST + 8 * H2C_GS];
  __shared__ uint32_t flg[8];
  const int gi = threadIdx.x / 8, role = threadIdx.x % 8;
  const int i = blockIdx.x * 8 + gi;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST + gi * H2C_GS, 0, 0, 0, (lu32*)&flg[gi], role};
  lp_init_consts(g);
  const bool act = i < n;
  const int P = H2C_S0, Q1 = P + 6, R = Q1 + 4, W = R + 6;
  {
    g2_aff a0, a1;
    if (act) { a0 = q[2 * i]; a1 = q[2 * i + 1]; } else { a0.x = fp2_zero(); a0.y = fp2_one(); a1 = a0; a1.x = fp2_one(); }
    if (role < 4) { g.s[P + role] = ((const fp*)&a0)[role]; g.s[Q1 + role] = ((const fp*)&a1)[role]; }
    if (role == 4) g.s[P + 4] = fp_one();
    if (role == 5) g.s[P + 5] = fp_zero();
  }
  __syncthreads();
  uint32_t exc = 0;
  g2_madd(g, P, Q1, P, exc);      // q0 + q1 (q0, q1 never infinity: iso3_map of the SWU points)
  g2_clear_cofactor(g, P, R, W, exc);
  if (act) {
    if (role < 6) ((fp*)&hj[i])[role] = g.s[R + role];
    if (role == 0) exc_out[i] = exc;
  }
}

// 4: affine output; a root whose lane-group stage met an exceptional addition (or every root,
// with exact_all: the test knob SSB_H2C_EXACT) is redone exactly, hj[i] serving as its temporary
__global__ void SSB_LB(64) k_h2c_affine(int n, const g2_aff* __restrict__ q, g2_jac* __restrict__ hj,
                                                   const uint32_t* __restrict__ exc, int exact_all, g2_aff* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
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
void hash_to_g2(hipStream_t st, int n, const uint8_t* roots, const dst_arg& dst, g2_aff* out, void* ws, const uint8_t* lens) {
  if (n <= 0) return;
  char* p = (char*)ws;
  auto take = [&](size_t b) { char* r = p; p += (b + 255) & ~(size_t)255; return r; };
  fp2* u = (fp2*)take(2 * n * sizeof(fp2));
  g2_aff* q = (g2_aff*)take(2 * n * sizeof(g2_aff));
  g2_jac* hj = (g2_jac*)take(n * sizeof(g2_jac));
  uint32_t* exc = (uint32_t*)take(n * 4);
  hipLaunchKernelGGL(k::k_h2c_u, dim3((n + 63) / 64), dim3(64), 0, st, n, roots, lens, dst, u);
  hipLaunchKernelGGL(k::k_h2c_map, dim3((4 * n + 63) / 64), dim3(64), 0, st, n, u, q);
  hipLaunchKernelGGL(k::k_h2c_clear, dim3((n + 7) / 8), dim3(64), 0, st, n, q, hj, exc);
  const char* ex = getenv("SSB_H2C_EXACT");
  const int exact_all = (ex && atoi(ex) != 0) ? 1 : 0;
  hipLaunchKernelGGL(k::k_h2c_affine, dim3((n + 63) / 64), dim3(64), 0, st, n, q, hj, exc, exact_all, out);
}
}  // namespace launch
}  // namespace ssb
