// ssb_f28.h -- the per-share G2 subgroup checks in the reduced radix of ssb_f28_field.h (round 6).
//
// Fp as 14 limbs of 28 bits, Montgomery form with R = 2^392 (p < 2^381: 11 bits of slack).  The
// product is product-scanning (FIPS) with ONE 64-bit accumulator per column and no carry handling
// inside a column: a limb product is < 2^58 (operand limbs < 2^29 / 2^30) and a column holds at
// most 42 of them (two products summed + the reduction), < 2^64 -- so every limb product is ONE
// v_mad_u64_u32, where the engine's 12 x 32-bit product (ssb_field.h) needs a v_mad_u64_u32 and a
// v_addc per limb product.  Measured on the ISA: 496 VALU instructions per product (392 of them
// MADs) against 671 (288 MADs) -- bench_tools/r28_bench.hip.
//
// Values are kept LAZILY reduced: a product's output is < 2p (it is (ab + mp)/R < ab/R + p, and
// the callers keep ab < R p, i.e. the operands' bounds in units of p multiply to < 2520); additions
// and subtractions leave values of a few p, with every limb normalized to < 2^28 (the top limb holds
// the rest); a subtraction a - b is a + K - b with a 'spread' multiple K of p whose limbs dominate
// b's (gen_f28.py); fold() brings a value below 2p (one 64-bit quotient estimate from the top
// limbs, one multiple of p subtracted), canon() below p.  The bound bookkeeping of each formula is
// written next to it (g2_subgroup_r28, ssb_curve.h).
//
// Exactness: every function computes the exact residue class (the tests compare the subgroup check
// with the engine's on subgroup points, non-subgroup curve points and infinity, host and GPU).
#pragma once
#include "ssb_curve.h"

namespace ssb {
namespace r28 {

// ---- Fp2 = Fp[u] / (u^2 + 1) ----
SSB_INL void add2(f2& r, const f2& a, const f2& b) { add(r.c0, a.c0, b.c0); add(r.c1, a.c1, b.c1); }
SSB_INL void sub2(f2& r, const f2& a, const f2& b, const uint32_t* K) { sub(r.c0, a.c0, b.c0, K); sub(r.c1, a.c1, b.c1, K); }
SSB_INL void dbl2(f2& r, const f2& a) { dbl(r.c0, a.c0); dbl(r.c1, a.c1); }
SSB_INL void fold2(f2& r, const f2& a) { fold(r.c0, a.c0); fold(r.c1, a.c1); }
SSB_INL void add_raw2(f2& r, const f2& a, const f2& b) { add_raw(r.c0, a.c0, b.c0); add_raw(r.c1, a.c1, b.c1); }
// r = a b: c0 = a0 b0 + a1 (K - b1), c1 = a0 b1 + a1 b0 -- two reductions (lazy), K above b1.
// Bounds (units of p): bA0 bB0 + bA1 k < 2520 and bA0 bB1 + bA1 bB0 < 2520; output < 2p each.
SSB_INL void mul2x(f2& r, const f2& a, const f2& b, const uint32_t* K) {
  SSB_CNT(fp_mul); SSB_CNT(fp_mul); SSB_CNT(fp_mul);   // (the engine's unit: an Fp2 product = 3)
  f nb1; neg_raw(nb1, b.c1, K);
  f c0, c1;
  mul2(c0, a.c0, b.c0, a.c1, nb1);
  mul2(c1, a.c0, b.c1, a.c1, b.c0);
  r.c0 = c0; r.c1 = c1;
}
// r = a^2: c0 = (a0 + a1)(a0 + K - a1), c1 = 2 a0 a1.  Bounds: 2 bA (bA + k) < 2520, K above a1;
// output c0 < 2p, c1 < 4p.
SSB_INL void sqr2(f2& r, const f2& a, const uint32_t* K) {
  f s, d, m;
  add_raw(s, a.c0, a.c1);
#pragma unroll
  for (int i = 0; i < 14; ++i) d.l[i] = a.c0.l[i] + K[i] - a.c1.l[i];   // < 2^30 per limb
  mul(m, a.c0, a.c1);
  mul(r.c0, s, d);
  dbl(r.c1, m);
}
SSB_INL void from_engine2(f2& r, const fp2& a) { from_engine(r.c0, a.c0); from_engine(r.c1, a.c1); }
SSB_INL bool is_zero2(const f2& a) { return is_zero(a.c0) && is_zero(a.c1); }

// ---- the G2 membership test psi(P) == [x]P in this representation (same answers as
// g2_in_subgroup_inl, ssb_curve.h, for every input) ----
// Bounds are in units of p, per component; the point's coordinates stay X < 12p, Y < 2p, Z < 4p.
// Doubling, a = 0 (dbl-2009-l): A = X^2, B = Y^2, C = B^2, D = 2((X+B)^2 - A - C), E = 3A,
// X3 = E^2 - 2D, Y3 = E(D - X3) - 8C, Z3 = 2YZ.
SSB_INL void g2_dbl(f2& X, f2& Y, f2& Z) {
  f2 A, B, C, t, D, E, F, w, X3, Y3, Z3;
  sqr2(A, X, K16P);              // 2 * 12 * (12 + 16) < 2520;  A < (2, 4)
  sqr2(B, Y, K4P);               // B < (2, 4)
  sqr2(C, B, K8P);               // C < (2, 4)
  add2(t, X, B);                 // < 16
  sqr2(t, t, K32P);              // 2 * 16 * (16 + 32) = 1536;  < (2, 4)
  dbl_sub_sub(D.c0, t.c0, A.c0, C.c0, KK16P);   // 2 (t^2 + 16p - A - C) < 40
  dbl_sub_sub(D.c1, t.c1, A.c1, C.c1, KK16P);
  fold2(D, D);                   // < 2
  mul_small(E.c0, A.c0, 3); mul_small(E.c1, A.c1, 3);   // < 12
  sqr2(F, E, K16P);              // 2 * 12 * 28 = 672;  < (2, 4)
  sub_dbl(X3.c0, F.c0, D.c0, KK8P); sub_dbl(X3.c1, F.c1, D.c1, KK8P);   // F + 8p - 2D < 12
  sub2(w, D, X3, K16P);          // < 18
  mul2x(Y3, E, w, K32P);         // 12 * 18 + 12 * 32 = 600;  < 2
  f2 c8; mul_small(c8.c0, C.c0, 8); mul_small(c8.c1, C.c1, 8);   // < 32
  sub2(Y3, Y3, c8, K64P);        // < 66
  fold2(Y3, Y3);                 // < 2
  f2 y2; add_raw2(y2, Y, Y);     // 2Y, limbs < 2^29 (a product operand)
  mul2x(Z3, y2, Z, K8P);         // 4 * 4 + 4 * 8 = 48;  Z3 = 2YZ < 2
  X = X3; Y = Y3; Z = Z3;
}
// Per-lane LDS the additions park the accumulator's X and Y in (word k of the lane at keep[k * S]):
// with X1, Y1, Z1, the affine point and the formula's temporaries all live the addition held more
// than the 256 registers of the kernel's two waves per SIMD, and spilled ~170 scratch accesses per
// addition (4.8 KB of HBM traffic per share at 8 x C2, gpurun_out/r06i).  The affine point itself is
// re-read from the input (global memory, engine form, L2-resident) at each use and converted by a
// shift (from_engine_shift), so it holds no registers through the 63 doublings either.
#if defined(__HIP_DEVICE_COMPILE__)
#define SSB_F28_LDS __attribute__((address_space(3)))
#else
#define SSB_F28_LDS
#endif
typedef SSB_F28_LDS uint32_t keep_t;
// (volatile: the compiler would otherwise forward the stored values to the loads and keep them in
// registers after all, its choice being the spilling one)
template <int S> SSB_INL void keep_st(keep_t* k, const f2& a) {
  volatile keep_t* v = k;
#pragma unroll
  for (int i = 0; i < 14; ++i) { v[i * S] = a.c0.l[i]; v[(14 + i) * S] = a.c1.l[i]; }
}
template <int S> SSB_INL void keep_ld(f2& a, const keep_t* k) {
  const volatile keep_t* v = k;
#pragma unroll
  for (int i = 0; i < 14; ++i) { a.c0.l[i] = v[i * S]; a.c1.l[i] = v[(14 + i) * S]; }
}
constexpr int KEEP_WORDS = 56;
// a coordinate of the input point, read at its use (the empty asm is a compiler barrier: the loads
// are not hoisted into registers that would live through the loop), < 2p
SSB_INL void ld_coord(f2& r, const fp2& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  __asm__ __volatile__("" ::: "memory");
#endif
  from_engine_shift(r.c0, a.c0);
  from_engine_shift(r.c1, a.c1);
}
// Mixed addition acc + P (madd-2007-bl, P's coordinates < 2p), Z3 = 2 Z1 H, X1 / Y1 parked in `keep`
// while the products run.  acc at infinity gives the point; acc == +-P (H == 0) returns false -- then
// [k -+ 1]P = O for the chain's prefix k, so P is not of order r.
template <int S> SSB_INL bool g2_madd(f2& X1, f2& Y1, f2& Z1, const g2_aff& p, keep_t* keep) {
  if (is_zero2(Z1)) {
    ld_coord(X1, p.x); ld_coord(Y1, p.y);
    Z1.c0 = cst(ONE28);
    for (int i = 0; i < 14; ++i) Z1.c1.l[i] = 0u;
    return true;
  }
  keep_st<S>(keep, X1);
  keep_st<S>(keep + 28 * S, Y1);
  f2 Z1Z1, U2, S2, H;
  sqr2(Z1Z1, Z1, K8P);           // < (2, 4)
  { f2 x2; ld_coord(x2, p.x); mul2x(U2, x2, Z1Z1, K8P); }                  // 2 * 4 + 2 * 8 = 24;  < 2
  { f2 y2, t; ld_coord(y2, p.y); mul2x(t, y2, Z1, K8P); mul2x(S2, t, Z1Z1, K8P); }   // < 2
  { f2 X; keep_ld<S>(X, keep); sub2(H, U2, X, K16P); }                     // X1 < 12: H < 18
  if (is_zero2(H)) return false;
  f2 Z3; mul2x(Z3, Z1, H, K32P);  // 4 * 18 + 4 * 32 = 200;  < 2
  dbl2(Z3, Z3);                  // < 4
  f2 rr; { f2 Y; keep_ld<S>(Y, keep + 28 * S); sub2(rr, S2, Y, K4P); }    // Y1 < 2: < 6
  dbl2(rr, rr);                  // < 12
  f2 I, J;
  { f2 HH; sqr2(HH, H, K32P); dbl2(I, HH); dbl2(I, I); }                   // 2 * 18 * 50 = 1800;  I < 16
  mul2x(J, H, I, K32P);          // 18 * 16 + 18 * 32 = 864;  < 2
  f2 V; { f2 X; keep_ld<S>(X, keep); mul2x(V, X, I, K32P); }               // 12 * 16 + 12 * 32 = 576;  < 2
  f2 X3; sqr2(X3, rr, K16P);     // 2 * 12 * 28 = 672;  < (2, 4)
  { f2 jv; dbl2(jv, V); add2(jv, jv, J); sub2(X3, X3, jv, K8P); }          // jv < 6: X3 < 12
  f2 Y3; { f2 w; sub2(w, V, X3, K16P); mul2x(Y3, rr, w, K32P); }           // w < 18; 12 * 18 + 12 * 32 = 600;  < 2
  { f2 Y, yj; keep_ld<S>(Y, keep + 28 * S); mul2x(yj, Y, J, K4P); dbl2(yj, yj); sub2(Y3, Y3, yj, K8P); }   // yj < 4: < 10
  fold2(Y3, Y3);                 // < 2
  X1 = X3; Y1 = Y3; Z1 = Z3;
  return true;
}
// psi(P) == [x]P, x = -|x|: [|x|]P by the wave-uniform double-and-add chain, then
// X == psi(P).x Z^2 and -Y == psi(P).y Z^3 (mod p).  keep: KEEP_WORDS words at stride S.
template <int S> SSB_INL bool g2_in_subgroup_keep(const g2_aff& p, keep_t* keep) {
  if (p.inf) return true;
  f2 X, Y, Z;
  ld_coord(X, p.x);              // < 2
  ld_coord(Y, p.y);
  Z.c0 = cst(ONE28);
  for (int i = 0; i < 14; ++i) Z.c1.l[i] = 0u;
  for (int i = 62; i >= 0; --i) {
    g2_dbl(X, Y, Z);
    if ((BLS_X_ABS >> i) & 1ull)
      if (!g2_madd<S>(X, Y, Z, p, keep)) return false;
  }
  if (is_zero2(Z)) return false;   // [x]P = O, psi(P) != O
  f2 cx, cy, px, py;
  cx.c0 = cst(PSI_CX28_0); cx.c1 = cst(PSI_CX28_1);
  cy.c0 = cst(PSI_CY28_0); cy.c1 = cst(PSI_CY28_1);
  {
    f2 x2, cj; ld_coord(x2, p.x);
    cj = x2; neg_raw(cj.c1, x2.c1, K4P); norm(cj.c1);   // conj(x2) < 4
    mul2x(px, cj, cx, K4P);      // < 2
  }
  {
    f2 y2, cj; ld_coord(y2, p.y);
    cj = y2; neg_raw(cj.c1, y2.c1, K4P); norm(cj.c1);
    mul2x(py, cj, cy, K4P);      // < 2
  }
  f2 Z2, Z3, lx, ly;
  sqr2(Z2, Z, K8P);              // < (2, 4)
  mul2x(Z3, Z2, Z, K8P);         // 4 * 4 + 4 * 8 = 48;  < 2
  mul2x(lx, px, Z2, K8P);        // < 2
  mul2x(ly, py, Z3, K4P);        // < 2
  if (!eq(X.c0, lx.c0) || !eq(X.c1, lx.c1)) return false;
  f2 s; add2(s, Y, ly);          // -Y == ly  <=>  Y + ly == 0
  return is_zero2(s);
}
#if !defined(__HIP_DEVICE_COMPILE__)
SSB_INL bool g2_in_subgroup(const g2_aff& p) { uint32_t k[KEEP_WORDS]; return g2_in_subgroup_keep<1>(p, k); }
#endif

}  // namespace r28
}  // namespace ssb
