// ssb_k_dkg.hip -- kernels (gfx950): batched DKG / VSS share verification.
//
// DKG::share_verification (src/crypto/dkg.rs:433-450) checks, per received share,
//     blst_p1_mult(h, s) == CommittedPoly::eval(party)
// with eval = C_0 + sum_{i>=1} [x^i mod r] C_i (src/math/polynomial.rs:68-81).  Here one thread
// per check: [s]h by a 4-bit fixed window over the low 255 bits of s (blst_p1_mult's nbits = 255),
// and the evaluation by Horner in the group, acc = [x] acc + C_i for i = t-1 .. 0 -- the same
// group element, since every C_i used has order r and the integer x^i equals x^i mod r on it.
// Commitments arrive compressed (CommittedPoly::to_bytes, polynomial.rs:88-99 without the count
// prefix).  Decoding follows CommittedPoly::from_bytes (polynomial.rs:101-118): the return code of
// blst_p1_uncompress is ignored, so a commitment that does not decode leaves the all-zero affine
// point, which blst_p1_from_affine turns into the identity -- here too it counts as infinity.
// A commitment that decodes to a curve point OUTSIDE G1 fails the check: blst_p1_mult multiplies
// 255-bit scalars by GLV, which equals [k]P only on G1, so the reference's result for such a point
// is blst-implementation-defined (and unequal to [s]h unless crafted); the engine rejects it
// (documented deviation).  Registration-time work, rare: plain single-lane code.
// k_dleq_verify: the Chaum-Pedersen proofs of exchange_group_public_keys.
#include "ssb_kernels.h"

namespace ssb {
namespace k {

// [x]P for a Jacobian P and a 64-bit x (binary, from the top set bit)
SSB_FN void g1_mul_u64_jac(g1_jac& r, const g1_jac& p, uint64_t x) {
  g1_jac acc; jac_set_inf(acc);
  for (int i = 63; i >= 0; --i) {
    if (!jac_is_inf(acc)) jac_dbl(acc, acc);
    if ((x >> i) & 1ull) jac_add(acc, acc, p);
  }
  r = acc;
}

// [r]P == O: membership in the order-r subgroup G1 (r from ssb_consts.h)
SSB_FN bool g1_in_subgroup(const g1_aff& p) {
  g1_jac q;
  jac_mul_aff(q, p, R_LIMBS, 8);
  return jac_is_inf(q);
}

SSB_INL bool g1_jac_eq(const g1_jac& a, const g1_jac& b) {
  const bool ia = jac_is_inf(a), ib = jac_is_inf(b);
  if (ia || ib) return ia && ib;
  fp za2, zb2, za3, zb3, l, r;
  fp_sqr(za2, a.z); fp_sqr(zb2, b.z);
  fp_mul(l, a.x, zb2); fp_mul(r, b.x, za2);
  if (!fp_eq(l, r)) return false;
  fp_mul(za3, za2, a.z); fp_mul(zb3, zb2, b.z);
  fp_mul(l, a.y, zb3); fp_mul(r, b.y, za3);
  return fp_eq(l, r);
}

__global__ void SSB_LB(64) k_feldman_share(int n, int t, const uint8_t* __restrict__ comm48, const uint64_t* __restrict__ x,
                                          const uint8_t* __restrict__ s32le, const g1_aff* __restrict__ h,
                                          const uint32_t* __restrict__ hflags, uint8_t* __restrict__ verdict) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t hf = *hflags;
  if (!(hf & DEC_OK)) { verdict[i] = 0; return; }
  bool ok = true;
  g1_jac acc; jac_set_inf(acc);
  for (int c = t - 1; c >= 0 && ok; --c) {
    uint8_t b[48];
    const uint8_t* src = comm48 + ((size_t)i * t + c) * 48;
    for (int k2 = 0; k2 < 48; ++k2) b[k2] = src[k2];
    g1_aff C;
    const uint32_t st = g1_decompress(C, b);
    if (c != t - 1) g1_mul_u64_jac(acc, acc, x[i]);
    if (!(st & DEC_OK) || C.inf) continue;      // undecodable: the identity, as the reference
    if (!g1_in_subgroup(C)) { ok = false; break; }
    jac_add_aff(acc, acc, C);
  }
  if (!ok) { verdict[i] = 0; return; }
  uint32_t k[8];
  for (int w = 0; w < 8; ++w) {
    const uint8_t* q = s32le + 32 * (size_t)i + 4 * w;
    k[w] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
  }
  k[7] &= 0x7fffffffu;                          // 255 bits, as blst_p1_mult(.., 255)
  g1_jac y;
  if (hf & DEC_INF) jac_set_inf(y); else jac_mul_w4(y, *h, k, 8);
  verdict[i] = g1_jac_eq(y, acc) ? 1 : 0;
}

// ---- DLEQ proof verification: DKG::dleq_verify (src/crypto/dkg.rs:674-692) ----
SSB_INL void load_scalar255(uint32_t* k, const uint8_t* b32) {
  for (int w = 0; w < 8; ++w) {
    const uint8_t* q = b32 + 4 * w;
    k[w] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
  }
  k[7] &= 0x7fffffffu;                          // blst_p1_mult(.., 255)
}
// a 256-bit little-endian chunk reduced mod r (chunk < 2^256 < 3r: at most two subtractions)
SSB_INL void fr_reduce256(uint32_t* v) {
  for (int pass = 0; pass < 2; ++pass) {
    uint32_t t[8], br = 0;
    for (int i = 0; i < 8; ++i) t[i] = subb(v[i], R_LIMBS[i], br, br);
    if (!br) for (int i = 0; i < 8; ++i) v[i] = t[i];
  }
}
// hash_points_to_blst_scalar (src/utils/blst_utils.rs:273-278): the 288-byte concatenation read as a
// little-endian integer mod r (blst_scalar_from_le_bytes): Horner over 32-byte chunks from the top,
// acc = acc * 2^256 + chunk (acc * 2^256 mod r = MontMul(acc, 2^512 mod r))
SSB_INL void le_bytes_mod_r(uint32_t* acc, const uint8_t* b, int nchunks) {
  for (int i = 0; i < 8; ++i) acc[i] = 0;
  for (int k = nchunks - 1; k >= 0; --k) {
    uint32_t c[8];
    for (int w = 0; w < 8; ++w) {
      const uint8_t* q = b + 32 * k + 4 * w;
      c[w] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
    }
    fr_reduce256(c);
    uint32_t t[8];
    mp_mont_mul<8>(t, acc, R_R2, R_LIMBS, R_INV32);
    mp_add_mod<8>(acc, t, c, R_LIMBS);
  }
}

__global__ void SSB_LB(64) k_dleq_verify(int n, const uint8_t* __restrict__ pts48, const uint8_t* __restrict__ c32,
                                        const uint8_t* __restrict__ r32, uint8_t* __restrict__ verdict) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t buf[288];                             // x1 y1 x2 y2 t1 t2, compressed
  for (int k = 0; k < 192; ++k) buf[k] = pts48[192 * (size_t)i + k];
  g1_aff P[4];
  for (int q = 0; q < 4; ++q)
    if (!(g1_decompress(P[q], buf + 48 * q) & DEC_OK)) { verdict[i] = 0; return; }
  uint32_t rk[8], ck[8];
  load_scalar255(rk, r32 + 32 * (size_t)i);
  load_scalar255(ck, c32 + 32 * (size_t)i);
  for (int h = 0; h < 2; ++h) {                 // t_h = [r] x_h + [c] y_h
    g1_jac a, b;
    if (P[2 * h].inf) jac_set_inf(a); else jac_mul_w4(a, P[2 * h], rk, 8);
    if (P[2 * h + 1].inf) jac_set_inf(b); else jac_mul_w4(b, P[2 * h + 1], ck, 8);
    jac_add(a, a, b);
    g1_aff t; jac_to_aff(t, a);
    g1_compress(buf + 192 + 48 * h, t);
  }
  uint32_t e[8];
  le_bytes_mod_r(e, buf, 9);
  bool ok = true;                               // proof.c == c_ (the 32 scalar bytes)
  for (int w = 0; w < 8; ++w) {
    const uint8_t* q = c32 + 32 * (size_t)i + 4 * w;
    const uint32_t cw = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
    ok = ok && cw == e[w];
  }
  verdict[i] = ok ? 1 : 0;
}

}  // namespace k

namespace launch {
void dleq_verify(hipStream_t st, int n, const uint8_t* pts48, const uint8_t* c32, const uint8_t* r32, uint8_t* verdict) {
  if (n > 0)
    hipLaunchKernelGGL(k::k_dleq_verify, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, n, pts48, c32, r32, verdict);
}
void feldman_share(hipStream_t st, int n, int t, const uint8_t* comm48, const uint64_t* x, const uint8_t* s32le,
                   const g1_aff* h, const uint32_t* hflags, uint8_t* verdict) {
  if (n > 0)
    hipLaunchKernelGGL(k::k_feldman_share, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, n, t, comm48, x, s32le, h,
                       hflags, verdict);
}
}  // namespace launch
}  // namespace ssb
