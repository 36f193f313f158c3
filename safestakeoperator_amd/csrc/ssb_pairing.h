// ssb_pairing.h -- optimal-ate Miller loop (Jacobian G2 steps with sparse 0/1/4 line values)
// and the final exponentiation (p^12-1)/r, for the pairing check inside blst's
// Signature::verify (src/crypto/generic_threshold.rs:156) and its random-linear-combination
// batch form (lighthouse verify_signature_sets semantics).
#pragma once
#include "ssb_curve.h"

namespace ssb {

// Tangent at T (Jacobian), T <- 2T.  Line (scaled by a factor in Fp2, killed by the final
// exponentiation):  l = (3X^3 - 2Y^2) + (-3X^2 Z^2 xP) v + (2 Y Z^3 yP) v w.
SSB_FN void miller_dbl_step(g2_jac& T, fp2& l0, fp2& l1, fp2& l4, const g1_aff& P) {
  fp2 A, B, C, D, E, F, ZZ, t;
  fp2_sqr(A, T.x);
  fp2_sqr(B, T.y);
  fp2_sqr(C, B);
  fp2_add(t, T.x, B); fp2_sqr(t, t); fp2_sub(t, t, A); fp2_sub(t, t, C); fp2_dbl(D, t);
  fp2_dbl(E, A); fp2_add(E, E, A);
  fp2_sqr(F, E);
  fp2_sqr(ZZ, T.z);
  // line from the old T
  fp2_mul(l0, E, T.x); fp2 b2; fp2_dbl(b2, B); fp2_sub(l0, l0, b2);
  fp2_mul(l1, E, ZZ); fp2_neg(l1, l1); fp2_mul_fp(l1, l1, P.x);
  fp2 x3, y3, z3;
  fp2_dbl(t, D); fp2_sub(x3, F, t);
  fp2_mul(z3, T.y, T.z); fp2_dbl(z3, z3);
  fp2_sub(t, D, x3); fp2_mul(y3, E, t);
  fp2_dbl(C, C); fp2_dbl(C, C); fp2_dbl(C, C);
  fp2_sub(y3, y3, C);
  fp2_mul(l4, z3, ZZ); fp2_mul_fp(l4, l4, P.y);
  T.x = x3; T.y = y3; T.z = z3;
}

// Chord through T (Jacobian) and Q (affine), T <- T + Q.
// l = (r xQ - yQ Z3) + (-r xP) v + (Z3 yP) v w,  r = 2(yQ Z^3 - Y), Z3 = 2 Z (xQ Z^2 - X).
SSB_FN void miller_add_step(g2_jac& T, fp2& l0, fp2& l1, fp2& l4, const g2_aff& Q, const g1_aff& P) {
  fp2 ZZ, U2, S2, H, HH, I, J, rr, V, t;
  fp2_sqr(ZZ, T.z);
  fp2_mul(U2, Q.x, ZZ);
  fp2_mul(S2, Q.y, T.z); fp2_mul(S2, S2, ZZ);
  fp2_sub(H, U2, T.x);
  fp2_sub(rr, S2, T.y); fp2_dbl(rr, rr);
  fp2_sqr(HH, H);
  fp2_dbl(I, HH); fp2_dbl(I, I);
  fp2_mul(J, H, I);
  fp2_mul(V, T.x, I);
  fp2 x3, y3, z3;
  fp2_sqr(x3, rr); fp2_sub(x3, x3, J); fp2_dbl(t, V); fp2_sub(x3, x3, t);
  fp2_sub(t, V, x3); fp2_mul(y3, rr, t); fp2_mul(t, T.y, J); fp2_dbl(t, t); fp2_sub(y3, y3, t);
  fp2_add(z3, T.z, H); fp2_sqr(z3, z3); fp2_sub(z3, z3, ZZ); fp2_sub(z3, z3, HH);
  fp2_mul(l0, rr, Q.x); fp2_mul(t, Q.y, z3); fp2_sub(l0, l0, t);
  fp2_neg(l1, rr); fp2_mul_fp(l1, l1, P.x);
  fp2_mul_fp(l4, z3, P.y);
  T.x = x3; T.y = y3; T.z = z3;
}

// f_{|x|,Q}(P), conjugated (x < 0).  Either point at infinity gives 1.
SSB_FN void miller_loop(fp12& f, const g1_aff& P, const g2_aff& Q) {
  f = fp12_one();
  if (P.inf || Q.inf) return;
  g2_jac T; jac_from_aff(T, Q);
  fp2 l0, l1, l4;
  bool first = true;
  for (int i = 62; i >= 0; --i) {
    if (!first) fp12_sqr(f, f);
    miller_dbl_step(T, l0, l1, l4, P);
    fp12_mul_014(f, f, l0, l1, l4);
    first = false;
    if ((BLS_X_ABS >> i) & 1ull) {
      miller_add_step(T, l0, l1, l4, Q, P);
      fp12_mul_014(f, f, l0, l1, l4);
    }
  }
  fp12_conj(f, f);
}

// f^((p^12-1)/r): easy part (p^6-1)(p^2+1), hard part by the x-adic chain
// (Hayashida-Hayasaka-Teruya form; computes the 3*(p^4-p^2+1)/r power, and since 3 does not
// divide r, the result is 1 exactly when the true pairing value is 1).
SSB_FN void final_exponentiation(fp12& r, const fp12& f) {
  fp12 t0, t1, t2, t3, t4, t5, t6;
  fp12_conj(t0, f);
  fp12_inv(t1, f);
  fp12_mul(t2, t0, t1);
  t1 = t2;
  fp12_frob(t2, t2, 2);
  fp12_mul(t2, t2, t1);
  fp12_cyc_sqr(t1, t2); fp12_conj(t1, t1);
  fp12_cyc_exp_x(t3, t2);
  fp12_cyc_sqr(t4, t3);
  fp12_mul(t5, t1, t3);
  fp12_cyc_exp_x(t1, t5);
  fp12_cyc_exp_x(t0, t1);
  fp12_cyc_exp_x(t6, t0);
  fp12_mul(t6, t6, t4);
  fp12_cyc_exp_x(t4, t6);
  fp12_conj(t5, t5);
  fp12_mul(t5, t5, t2);
  fp12_mul(t4, t4, t5);
  fp12_conj(t5, t2);
  fp12_mul(t1, t1, t2);
  fp12_frob(t1, t1, 3);
  fp12_mul(t6, t6, t5);
  fp12_frob(t6, t6, 1);
  fp12_mul(t3, t3, t0);
  fp12_frob(t3, t3, 2);
  fp12_mul(t3, t3, t1);
  fp12_mul(t3, t3, t6);
  fp12_mul(r, t3, t4);
}

}  // namespace ssb
