// ssb_curve.h -- G1 (E: y^2 = x^3 + 4 over Fp) and G2 (E': y^2 = x^3 + 4(1+u) over Fp2) in
// Jacobian coordinates, ZCash (de)serialisation and the G2 subgroup check.
//
// Replaces, on the device: blst_p2_uncompress/blst_p1_uncompress (lighthouse Signature /
// PublicKey deserialize), blst_p2_from_affine / blst_p2_mult / blst_p2_serialize / add
// (src/crypto/impls/blst.rs:72-86), blst_p2_compress (Signature::serialize, :86) and the
// sig_groupcheck inside Signature::verify (src/crypto/generic_threshold.rs:156).
#pragma once
#include "ssb_field.h"

namespace ssb {

// ---- field-generic overloads so the curve code is written once for Fp and Fp2 ----
SSB_INL void f_add(fp& r, const fp& a, const fp& b) { fp_add(r, a, b); }
SSB_INL void f_sub(fp& r, const fp& a, const fp& b) { fp_sub(r, a, b); }
SSB_INL void f_dbl(fp& r, const fp& a) { fp_dbl(r, a); }
SSB_INL void f_neg(fp& r, const fp& a) { fp_neg(r, a); }
SSB_INL void f_mul(fp& r, const fp& a, const fp& b) { fp_mul(r, a, b); }
SSB_INL void f_sqr(fp& r, const fp& a) { fp_sqr(r, a); }
SSB_INL bool f_is_zero(const fp& a) { return fp_is_zero(a); }
SSB_INL bool f_eq(const fp& a, const fp& b) { return fp_eq(a, b); }
SSB_INL void f_inv(fp& r, const fp& a) { fp_inv(r, a); }
SSB_INL void f_set_one(fp& r) { r = fp_one(); }
SSB_INL void f_set_zero(fp& r) { r = fp_zero(); }
SSB_INL void f_add(fp2& r, const fp2& a, const fp2& b) { fp2_add(r, a, b); }
SSB_INL void f_sub(fp2& r, const fp2& a, const fp2& b) { fp2_sub(r, a, b); }
SSB_INL void f_dbl(fp2& r, const fp2& a) { fp2_dbl(r, a); }
SSB_INL void f_neg(fp2& r, const fp2& a) { fp2_neg(r, a); }
SSB_INL void f_mul(fp2& r, const fp2& a, const fp2& b) { fp2_mul(r, a, b); }
SSB_INL void f_sqr(fp2& r, const fp2& a) { fp2_sqr(r, a); }
SSB_INL bool f_is_zero(const fp2& a) { return fp2_is_zero(a); }
SSB_INL bool f_eq(const fp2& a, const fp2& b) { return fp2_eq(a, b); }
SSB_INL void f_inv(fp2& r, const fp2& a) { fp2_inv(r, a); }
SSB_INL void f_set_one(fp2& r) { r = fp2_one(); }
SSB_INL void f_set_zero(fp2& r) { r = fp2_zero(); }

template <class F> struct aff { F x, y; uint32_t inf; };
template <class F> struct jac { F x, y, z; };  // x = X/Z^2, y = Y/Z^3; Z == 0 <=> infinity

using g1_aff = aff<fp>;
using g2_aff = aff<fp2>;
using g1_jac = jac<fp>;
using g2_jac = jac<fp2>;

template <class F> SSB_INL void jac_set_inf(jac<F>& r) { f_set_one(r.x); f_set_one(r.y); f_set_zero(r.z); }
template <class F> SSB_INL bool jac_is_inf(const jac<F>& p) { return f_is_zero(p.z); }
template <class F> SSB_INL void jac_from_aff(jac<F>& r, const aff<F>& a) {
  if (a.inf) { jac_set_inf(r); return; }
  r.x = a.x; r.y = a.y; f_set_one(r.z);
}
template <class F> SSB_INL void jac_neg(jac<F>& r, const jac<F>& p) { r.x = p.x; f_neg(r.y, p.y); r.z = p.z; }

// dbl-2009-l (a = 0): 2M + 5S.  Infinity in -> infinity out (Z3 = 2YZ = 0).
// jac_dbl_inl is inlined into the doubling loops of the scalar multiplications: measured on
// MI355X (bench_tools/dbl_bench.hip) 2.48 G G2-doublings/s inlined against 1.65 G through a call,
// whose argument and callee-saved-register traffic goes through scratch.  jac_dbl is the
// out-of-line copy for the cold call sites.
template <class F> SSB_INL void jac_dbl_inl(jac<F>& r, const jac<F>& p) {
  F A, B, C, D, E, Fv, t;
  f_sqr(A, p.x);
  f_sqr(B, p.y);
  f_sqr(C, B);
  f_add(t, p.x, B); f_sqr(t, t); f_sub(t, t, A); f_sub(t, t, C); f_dbl(D, t);
  f_dbl(E, A); f_add(E, E, A);
  f_sqr(Fv, E);
  F x3, y3, z3;
  f_dbl(t, D); f_sub(x3, Fv, t);
  f_mul(z3, p.y, p.z); f_dbl(z3, z3);
  f_sub(t, D, x3); f_mul(y3, E, t);
  f_dbl(C, C); f_dbl(C, C); f_dbl(C, C);
  f_sub(y3, y3, C);
  r.x = x3; r.y = y3; r.z = z3;
}
template <class F> SSB_FN void jac_dbl(jac<F>& r, const jac<F>& p) { jac_dbl_inl(r, p); }

// madd-2007-bl: r = p + q, q affine.  Handles infinity and the doubling/opposite cases.
// (_inl: inlined into the MSM bucket loops; jac_add_aff: out-of-line copy)
template <class F> SSB_INL void jac_add_aff_inl(jac<F>& r, const jac<F>& p, const aff<F>& q) {
  if (q.inf) { r = p; return; }
  if (jac_is_inf(p)) { jac_from_aff(r, q); return; }
  F Z1Z1, U2, S2, H, HH, I, J, rr, V, t;
  f_sqr(Z1Z1, p.z);
  f_mul(U2, q.x, Z1Z1);
  f_mul(S2, q.y, p.z); f_mul(S2, S2, Z1Z1);
  f_sub(H, U2, p.x);
  f_sub(rr, S2, p.y);
  if (f_is_zero(H)) {
    if (f_is_zero(rr)) { jac<F> d; jac_from_aff(d, q); jac_dbl(r, d); }
    else jac_set_inf(r);
    return;
  }
  f_dbl(rr, rr);
  f_sqr(HH, H);
  f_dbl(I, HH); f_dbl(I, I);
  f_mul(J, H, I);
  f_mul(V, p.x, I);
  F x3, y3, z3;
  f_sqr(x3, rr); f_sub(x3, x3, J); f_dbl(t, V); f_sub(x3, x3, t);
  f_sub(t, V, x3); f_mul(y3, rr, t); f_mul(t, p.y, J); f_dbl(t, t); f_sub(y3, y3, t);
  f_add(z3, p.z, H); f_sqr(z3, z3); f_sub(z3, z3, Z1Z1); f_sub(z3, z3, HH);
  r.x = x3; r.y = y3; r.z = z3;
}
template <class F> SSB_FN void jac_add_aff(jac<F>& r, const jac<F>& p, const aff<F>& q) { jac_add_aff_inl(r, p, q); }
// a += *qp in place, the same formula and special cases as jac_add_aff_inl, written for the bucket
// loops at two waves per SIMD (256 registers): q's coordinates are loaded where they are consumed,
// temporaries die early (at most six Fp2 values live besides a product's operands), and the rare
// doubling branch is inlined -- a call there made the loop save its live registers around it.
// Static spill census of a G2 bucket loop (bench_tools/isa_scratch.py): 83 scratch stores and 71
// loads on the addition's path with jac_add_aff_inl, 27 / 27 with this form.
template <class F> SSB_INL void jac_madd_at(jac<F>& a, const aff<F>* __restrict__ qp) {
  if (qp->inf) return;
  if (jac_is_inf(a)) { jac_from_aff(a, *qp); return; }
  F Z1Z1, r, H;
  f_sqr(Z1Z1, a.z);
  { F S2; const F y2 = qp->y; f_mul(S2, y2, a.z); f_mul(S2, S2, Z1Z1); f_sub(r, S2, a.y); }   // S2 - Y1
  { F U2; const F x2 = qp->x; f_mul(U2, x2, Z1Z1); f_sub(H, U2, a.x); }                       // U2 - X1
  if (f_is_zero(H)) {
    if (f_is_zero(r)) { jac<F> d; jac_from_aff(d, *qp); jac_dbl_inl(a, d); } else jac_set_inf(a);
    return;
  }
  f_dbl(r, r);
  F I;
  {
    F HH, t;
    f_sqr(HH, H);
    f_add(t, a.z, H); f_sqr(t, t); f_sub(t, t, Z1Z1); f_sub(a.z, t, HH);   // Z3 = (Z1 + H)^2 - Z1Z1 - HH
    f_dbl(I, HH); f_dbl(I, I);
  }
  F V; f_mul(V, a.x, I);
  F J; f_mul(J, H, I);
  F t; f_mul(t, a.y, J);
  f_sqr(a.x, r); f_sub(a.x, a.x, J); f_dbl(J, V); f_sub(a.x, a.x, J);     // X3 = r^2 - J - 2V
  f_sub(V, V, a.x); f_mul(a.y, r, V); f_dbl(t, t); f_sub(a.y, a.y, t);    // Y3 = r (V - X3) - 2 Y1 J
}

// add-2007-bl: general Jacobian addition with the special cases.
template <class F> SSB_INL void jac_add_inl(jac<F>& r, const jac<F>& p, const jac<F>& q) {
  if (jac_is_inf(p)) { r = q; return; }
  if (jac_is_inf(q)) { r = p; return; }
  F Z1Z1, Z2Z2, U1, U2, S1, S2, H, I, J, rr, V, t;
  f_sqr(Z1Z1, p.z);
  f_sqr(Z2Z2, q.z);
  f_mul(U1, p.x, Z2Z2);
  f_mul(U2, q.x, Z1Z1);
  f_mul(S1, p.y, q.z); f_mul(S1, S1, Z2Z2);
  f_mul(S2, q.y, p.z); f_mul(S2, S2, Z1Z1);
  f_sub(H, U2, U1);
  f_sub(rr, S2, S1);
  if (f_is_zero(H)) {
    if (f_is_zero(rr)) jac_dbl_inl(r, p); else jac_set_inf(r);
    return;
  }
  f_dbl(rr, rr);
  f_dbl(I, H); f_sqr(I, I);
  f_mul(J, H, I);
  f_mul(V, U1, I);
  F x3, y3, z3;
  f_sqr(x3, rr); f_sub(x3, x3, J); f_dbl(t, V); f_sub(x3, x3, t);
  f_sub(t, V, x3); f_mul(y3, rr, t); f_mul(t, S1, J); f_dbl(t, t); f_sub(y3, y3, t);
  f_add(z3, p.z, q.z); f_sqr(z3, z3); f_sub(z3, z3, Z1Z1); f_sub(z3, z3, Z2Z2); f_mul(z3, z3, H);
  r.x = x3; r.y = y3; r.z = z3;
}
template <class F> SSB_FN void jac_add(jac<F>& r, const jac<F>& p, const jac<F>& q) { jac_add_inl(r, p, q); }

template <class F> SSB_FN void jac_to_aff(aff<F>& r, const jac<F>& p) {
  if (jac_is_inf(p)) { f_set_zero(r.x); f_set_zero(r.y); r.inf = 1; return; }
  F zi, zi2, zi3;
  f_inv(zi, p.z);
  f_sqr(zi2, zi);
  f_mul(zi3, zi2, zi);
  f_mul(r.x, p.x, zi2);
  f_mul(r.y, p.y, zi3);
  r.inf = 0;
}

// Jacobian point == affine point
template <class F> SSB_INL bool jac_eq_aff(const jac<F>& p, const aff<F>& q) {
  if (jac_is_inf(p) || q.inf) return jac_is_inf(p) && q.inf;
  F z2, z3, t;
  f_sqr(z2, p.z);
  f_mul(z3, z2, p.z);
  f_mul(t, q.x, z2);
  if (!f_eq(t, p.x)) return false;
  f_mul(t, q.y, z3);
  return f_eq(t, p.y);
}

// [k]P for a per-lane scalar given as `nwords` little-endian 32-bit words (binary, MSB first).
template <class F> SSB_FN void jac_mul_aff(jac<F>& r, const aff<F>& p, const uint32_t* k, int nwords) {
  jac<F> acc;
  jac_set_inf(acc);
  for (int i = 32 * nwords - 1; i >= 0; --i) {
    jac_dbl_inl(acc, acc);
    if ((k[i >> 5] >> (i & 31)) & 1u) jac_add_aff(acc, acc, p);
  }
  r = acc;
}

// [k]P with a 4-bit fixed window over a Jacobian table (per-lane scalar, divergence-friendly:
// every lane runs the same dbl/add schedule; only the table row differs).
template <class F> SSB_FN void jac_mul_w4(jac<F>& r, const aff<F>& p, const uint32_t* k, int nwords) {
  jac<F> tab[16];
  jac_set_inf(tab[0]);
  jac_from_aff(tab[1], p);
  for (int i = 2; i < 16; ++i) jac_add_aff(tab[i], tab[i - 1], p);
  jac<F> acc;
  jac_set_inf(acc);
  for (int w = 8 * nwords - 1; w >= 0; --w) {
    if (w != 8 * nwords - 1) {
#pragma unroll 1
      for (int q = 0; q < 4; ++q) jac_dbl_inl(acc, acc);
    }
    const uint32_t d = (k[w >> 3] >> ((w & 7) * 4)) & 15u;
    jac_add(acc, acc, tab[d]);
  }
  r = acc;
}

// [k]P for an affine P and an ODD scalar of `nwords` 32-bit LE words: regular signed window, w = 4
// (Joye-Tunstall recoding: 8*nwords odd digits in [-15, 15], every window adds a table entry).
// The table holds the 8 odd multiples P, 3P, .., 15P (half the 16-entry table of jac_mul_w4, so
// half the private memory per lane).  Exact for every input: jac_add handles all special cases.
template <class F> SSB_FN void jac_mul_sw4_odd(jac<F>& r, const aff<F>& p, const uint32_t* k_in, int nwords) {
  int8_t dig[64];
  uint32_t k[8];
  for (int i = 0; i < 8; ++i) k[i] = i < nwords ? k_in[i] : 0u;
  const int W = 8 * nwords;
  for (int j = 0; j < W - 1; ++j) {  // d = (k mod 32) - 16;  k = (k - d) / 16
    const int d = (int)(k[0] & 31u) - 16;
    dig[j] = (int8_t)d;
    uint32_t br = 0;                   // k -= d (d < 0: k += |d|), then k >>= 4
    if (d >= 0) {
      uint32_t s = (uint32_t)d;
      for (int i = 0; i < nwords; ++i) { k[i] = subb(k[i], s, br, br); s = 0; }
    } else {
      uint32_t s = (uint32_t)(-d), c = 0;
      for (int i = 0; i < nwords; ++i) { k[i] = addc(k[i], s, c, c); s = 0; }
    }
    for (int i = 0; i < nwords - 1; ++i) k[i] = (k[i] >> 4) | (k[i + 1] << 28);
    k[nwords - 1] >>= 4;
  }
  dig[W - 1] = (int8_t)k[0];
  jac<F> tab[8], p2;
  jac_from_aff(tab[0], p);
  jac_dbl(p2, tab[0]);
  jac_add_aff(tab[1], p2, p);
  for (int i = 2; i < 8; ++i) jac_add(tab[i], tab[i - 1], p2);
  jac<F> acc = tab[(dig[W - 1] - 1) >> 1];
  for (int j = W - 2; j >= 0; --j) {
#pragma unroll 1
    for (int q = 0; q < 4; ++q) jac_dbl_inl(acc, acc);
    const int d = dig[j];
    jac<F> t = tab[((d < 0 ? -d : d) - 1) >> 1];
    if (d < 0) jac_neg(t, t);
    jac_add(acc, acc, t);
  }
  r = acc;
}

// [|x|]P, x = -0xd201000000010000 (wave-uniform scalar: branch-free across lanes)
template <class F> SSB_FN void jac_mul_x_abs(jac<F>& r, const jac<F>& p) {
  jac<F> acc = p;
  for (int i = 62; i >= 0; --i) {
    jac_dbl_inl(acc, acc);
    if ((BLS_X_ABS >> i) & 1ull) jac_add(acc, acc, p);
  }
  r = acc;
}
template <class F> SSB_FN void jac_mul_x_abs_aff(jac<F>& r, const aff<F>& p) {
  jac<F> acc; jac_from_aff(acc, p);
  for (int i = 62; i >= 0; --i) {
    jac_dbl_inl(acc, acc);
    if ((BLS_X_ABS >> i) & 1ull) jac_add_aff(acc, acc, p);
  }
  r = acc;
}

// ---- G2 endomorphism psi = twist^-1 o Frobenius o twist: (conj(x) cx, conj(y) cy) ----
SSB_INL void g2_psi_aff(g2_aff& r, const g2_aff& p) {
  fp2 cx = fp2_from_c(PSI_CX), cy = fp2_from_c(PSI_CY), t;
  fp2_conj(t, p.x); fp2_mul(r.x, t, cx);
  fp2_conj(t, p.y); fp2_mul(r.y, t, cy);
  r.inf = p.inf;
}
SSB_INL void g2_psi_jac(g2_jac& r, const g2_jac& p) {
  fp2 cx = fp2_from_c(PSI_CX), cy = fp2_from_c(PSI_CY), t;
  fp2_conj(t, p.x); fp2_mul(r.x, t, cx);
  fp2_conj(t, p.y); fp2_mul(r.y, t, cy);
  fp2_conj(r.z, p.z);
}

// G2 membership (sig_groupcheck): psi(P) == [x]P  (Scott 2021; == [r]P == O on BLS12-381)
// Mixed addition for the membership test's [|x|]P chain, ordered so few temporaries are live (the
// occupancy-2 subgroup kernel spills 54 registers with it, 146 with jac_add_aff_inl).  Returns
// false on the exceptional case acc == +-P: then [k -+ 1]P = O for the chain's current prefix k,
// 1 <= k -+ 1 < r, so P cannot have order r -- the answer is "not in G2" without the doubling.
SSB_INL bool g2_add_aff_sg(g2_jac& r, const g2_jac& p, const g2_aff& q) {
  if (jac_is_inf(p)) { jac_from_aff(r, q); return true; }
  fp2 Z1Z1, H, rr, HH, z3, t;
  fp2_sqr(Z1Z1, p.z);
  fp2_mul(H, q.x, Z1Z1); fp2_sub(H, H, p.x);                        // U2 - X1
  fp2_mul(t, q.y, p.z); fp2_mul(t, t, Z1Z1); fp2_sub(rr, t, p.y);   // S2 - Y1
  if (fp2_is_zero(H)) return false;
  fp2_dbl(rr, rr);
  fp2_sqr(HH, H);
  fp2_add(z3, p.z, H); fp2_sqr(z3, z3); fp2_sub(z3, z3, Z1Z1); fp2_sub(z3, z3, HH);
  fp2 I, J, V;
  fp2_dbl(I, HH); fp2_dbl(I, I);
  fp2_mul(J, H, I);
  fp2_mul(V, p.x, I);
  fp2 x3, y3;
  fp2_sqr(x3, rr); fp2_sub(x3, x3, J); fp2_dbl(t, V); fp2_sub(x3, x3, t);
  fp2_sub(t, V, x3); fp2_mul(y3, rr, t); fp2_mul(t, p.y, J); fp2_dbl(t, t); fp2_sub(y3, y3, t);
  r.x = x3; r.y = y3; r.z = z3;
  return true;
}
// call-free membership test (the occupancy-2 subgroup kernel); same answers as g2_in_subgroup
SSB_INL bool g2_in_subgroup_inl(const g2_aff& p) {
  if (p.inf) return true;
  g2_jac acc; jac_from_aff(acc, p);
  for (int i = 62; i >= 0; --i) {
    jac_dbl_inl(acc, acc);
    if (((BLS_X_ABS >> i) & 1ull) && !g2_add_aff_sg(acc, acc, p)) return false;
  }
  jac_neg(acc, acc);  // x < 0
  g2_aff ps;
  g2_psi_aff(ps, p);
  return jac_eq_aff(acc, ps);
}
SSB_FN bool g2_in_subgroup(const g2_aff& p) {
  if (p.inf) return true;
  g2_jac xp;
  jac_mul_x_abs_aff(xp, p);
  jac_neg(xp, xp);  // x < 0
  g2_aff ps;
  g2_psi_aff(ps, p);
  return jac_eq_aff(xp, ps);
}

// ---- decoding status bits (also exported in include/ssbls.h) ----
enum : uint32_t {
  DEC_OK = 1u,          // bytes decoded to a curve point (blst *_uncompress == BLST_SUCCESS)
  DEC_INF = 2u,         // the point is the point at infinity
  DEC_IN_GROUP = 4u,    // passed the subgroup check (G2 signatures only)
};

// blst_p2_uncompress semantics.  Returns DEC_* bits (0 on BLST_BAD_ENCODING / NOT_ON_CURVE).
template <bool INL = true>
SSB_INL uint32_t g2_decompress_inl(g2_aff& r, const uint8_t* in) {
  const uint8_t b0 = in[0];
  r.inf = 0;
  if (!(b0 & 0x80)) return 0;
  if (b0 & 0x40) {
    bool zero = (b0 & 0x3f) == 0;
    for (int i = 1; i < 96; ++i) zero = zero && in[i] == 0;
    if (!zero) return 0;
    r.x = fp2_zero(); r.y = fp2_zero(); r.inf = 1;
    return DEC_OK | DEC_INF;
  }
  fp x1, x0;
  if (!fp_from_be48(x1, in, 0x1f)) return 0;
  if (!fp_from_be48(x0, in + 48, 0xff)) return 0;
  fp2 x;
  fp_to_mont(x.c0, x0);
  fp_to_mont(x.c1, x1);
  fp2 y2, t;
  fp2_sqr(t, x); fp2_mul(y2, t, x);
  fp2 b = fp2_from_c(FP2_B2);
  fp2_add(y2, y2, b);
  fp2 y;
  if (!fp2_sqrt_inl<INL>(y, y2)) return 0;
  const bool want = (b0 & 0x20) != 0;
  if (fp2_lex_largest(y) != want) fp2_neg(y, y);
  r.x = x; r.y = y;
  return DEC_OK;
}
SSB_FN uint32_t g2_decompress(g2_aff& r, const uint8_t* in) { return g2_decompress_inl<false>(r, in); }

SSB_INL uint32_t g1_decompress_inl(g1_aff& r, const uint8_t* in) {
  const uint8_t b0 = in[0];
  r.inf = 0;
  if (!(b0 & 0x80)) return 0;
  if (b0 & 0x40) {
    bool zero = (b0 & 0x3f) == 0;
    for (int i = 1; i < 48; ++i) zero = zero && in[i] == 0;
    if (!zero) return 0;
    r.x = fp_zero(); r.y = fp_zero(); r.inf = 1;
    return DEC_OK | DEC_INF;
  }
  fp xc;
  if (!fp_from_be48(xc, in, 0x1f)) return 0;
  fp x; fp_to_mont(x, xc);
  fp y2, t;
  fp_sqr(t, x); fp_mul(y2, t, x);
  fp b = fp_from_c(FP_B1);
  fp_add(y2, y2, b);
  fp y;
  if (!fp_sqrt_inl(y, y2)) return 0;
  const bool want = (b0 & 0x20) != 0;
  if (fp_lex_largest(y) != want) fp_neg(y, y);
  r.x = x; r.y = y;
  return DEC_OK;
}
SSB_FN uint32_t g1_decompress(g1_aff& r, const uint8_t* in) { return g1_decompress_inl(r, in); }

// blst_p2_compress (Signature::serialize): x.c1 | x.c0 big-endian, flags in byte 0
SSB_FN void g2_compress(uint8_t* out, const g2_aff& p) {
  if (p.inf) {
    out[0] = 0xc0;
    for (int i = 1; i < 96; ++i) out[i] = 0;
    return;
  }
  fp c;
  fp_from_mont(c, p.x.c1); fp_to_be48(out, c);
  fp_from_mont(c, p.x.c0); fp_to_be48(out + 48, c);
  out[0] |= 0x80;
  if (fp2_lex_largest(p.y)) out[0] |= 0x20;
}

SSB_FN void g1_compress(uint8_t* out, const g1_aff& p) {
  if (p.inf) {
    out[0] = 0xc0;
    for (int i = 1; i < 48; ++i) out[i] = 0;
    return;
  }
  fp c;
  fp_from_mont(c, p.x); fp_to_be48(out, c);
  out[0] |= 0x80;
  if (fp_lex_largest(p.y)) out[0] |= 0x20;
}

// blst_p2_serialize (uncompressed, 192 bytes)
SSB_FN void g2_serialize(uint8_t* out, const g2_aff& p) {
  if (p.inf) {
    out[0] = 0x40;
    for (int i = 1; i < 192; ++i) out[i] = 0;
    return;
  }
  fp c;
  fp_from_mont(c, p.x.c1); fp_to_be48(out, c);
  fp_from_mont(c, p.x.c0); fp_to_be48(out + 48, c);
  fp_from_mont(c, p.y.c1); fp_to_be48(out + 96, c);
  fp_from_mont(c, p.y.c0); fp_to_be48(out + 144, c);
}

}  // namespace ssb
