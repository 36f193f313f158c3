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

// ---- complete G2 additions for the MSM sums (the bucket sums of k_msm_bucket2, ssb_blocks.h; pt2_add
// is host-tested for the window sums, which stay in the engine's form: inlined into their chains the
// reduced-radix additions spilled ~3 KB per lane at 256 architectural registers) ----
// A Jacobian point with an explicit infinity flag (a lazily reduced Z is not cheaply compared with 0);
// coordinates bounded as in the subgroup chain: X < 12p, Y < 2p, Z < 4p.  Every input, including
// equal and opposite points, gives the exact sum (the formulas' exceptional cases are branches).
struct pt2 { f2 x, y, z; bool inf; };
SSB_INL void pt2_set_inf(pt2& a) { a.inf = true; }
SSB_INL void pt2_from_aff(pt2& a, const g2_aff& p) {
  a.inf = p.inf != 0;
  ld_coord(a.x, p.x); ld_coord(a.y, p.y);
  a.z.c0 = cst(ONE28);
  for (int i = 0; i < 14; ++i) a.z.c1.l[i] = 0u;
}
// the engine's Jacobian point (12 x 32-bit, z == 0 at infinity) in and out
SSB_INL void pt2_from_engine(pt2& a, const g2_jac& p) {
  a.inf = jac_is_inf(p);
  from_engine_shift(a.x.c0, p.x.c0); from_engine_shift(a.x.c1, p.x.c1);
  from_engine_shift(a.y.c0, p.y.c0); from_engine_shift(a.y.c1, p.y.c1);
  from_engine_shift(a.z.c0, p.z.c0); from_engine_shift(a.z.c1, p.z.c1);
}
SSB_INL void pt2_to_engine(g2_jac& r, const pt2& a) {
  if (a.inf) { jac_set_inf(r); return; }
  f2 x = a.x, z = a.z;
  fold2(x, x); fold2(z, z);      // (X < 12p, Z < 4p: below 2p for the conversion)
  to_engine_shift(r.x.c0, x.c0); to_engine_shift(r.x.c1, x.c1);
  to_engine_shift(r.y.c0, a.y.c0); to_engine_shift(r.y.c1, a.y.c1);
  to_engine_shift(r.z.c0, z.c0); to_engine_shift(r.z.c1, z.c1);
}
SSB_INL void pt2_dbl(pt2& a) {
  if (!a.inf) g2_dbl(a.x, a.y, a.z);   // (Y = 0 has no G2 point: the doubling never meets infinity)
}
// a += P, P affine (engine form in global memory, read at its uses), X1 / Y1 parked in `keep` while
// the products run (as the subgroup chain's g2_madd); H == 0: 2P when the points are equal, else O
template <int S> SSB_INL void pt2_madd(pt2& a, const g2_aff& p, keep_t* keep) {
  if (p.inf) return;
  if (a.inf) { pt2_from_aff(a, p); return; }
  keep_st<S>(keep, a.x);
  keep_st<S>(keep + 28 * S, a.y);
  f2 Z1Z1, U2, S2, H;
  sqr2(Z1Z1, a.z, K8P);          // Z1 < 4: 2 * 4 * 12 = 96;  < (2, 4)
  { f2 x2; ld_coord(x2, p.x); mul2x(U2, x2, Z1Z1, K8P); }                  // 2 * 2 + 2 * 8 = 20;  < 2
  { f2 y2, t; ld_coord(y2, p.y); mul2x(t, y2, a.z, K8P); mul2x(S2, t, Z1Z1, K8P); }   // < 2
  { f2 X; keep_ld<S>(X, keep); sub2(H, U2, X, K16P); }                     // X1 < 12: H < 18
  f2 rr; { f2 Y; keep_ld<S>(Y, keep + 28 * S); sub2(rr, S2, Y, K4P); }    // Y1 < 2: < 6
  if (is_zero2(H)) {
    if (is_zero2(rr)) { pt2_from_aff(a, p); g2_dbl(a.x, a.y, a.z); }      // acc == P
    else a.inf = true;                                                     // acc == -P
    return;
  }
  f2 Z3; mul2x(Z3, a.z, H, K32P);  // 4 * 18 + 4 * 32 = 200;  < 2
  dbl2(Z3, Z3);                  // < 4
  dbl2(rr, rr);                  // < 12
  f2 I, J;
  { f2 HH; sqr2(HH, H, K32P); dbl2(I, HH); dbl2(I, I); }                   // 2 * 18 * 50 = 1800;  I < 16
  mul2x(J, H, I, K32P);          // 18 * 16 + 18 * 32 = 864;  < 2
  f2 V; { f2 X; keep_ld<S>(X, keep); mul2x(V, X, I, K32P); }               // 12 * 16 + 12 * 32 = 576;  < 2
  f2 X3; sqr2(X3, rr, K16P);     // 2 * 12 * 28 = 672;  < (2, 4)
  { f2 jv; dbl2(jv, V); add2(jv, jv, J); sub2(X3, X3, jv, K8P); }          // jv < 6: X3 < 12
  f2 Y3; { f2 w; sub2(w, V, X3, K16P); mul2x(Y3, rr, w, K32P); }           // w < 18; 12 * 18 + 12 * 32 = 600;  < 2
  { f2 Y, yj; keep_ld<S>(Y, keep + 28 * S); mul2x(yj, Y, J, K4P); dbl2(yj, yj); sub2(Y3, Y3, yj, K8P); }   // < 10
  fold2(Y3, Y3);                 // < 2
  a.x = X3; a.y = Y3; a.z = Z3;
}
// a += b (add-2007-bl), both Jacobian
SSB_INL void pt2_add(pt2& a, const pt2& b) {
  if (b.inf) return;
  if (a.inf) { a = b; return; }
  f2 Z1Z1, Z2Z2, U1, U2, S1, S2, H, rr;
  sqr2(Z1Z1, a.z, K8P);          // Z < 4: 2 * 4 * 12 = 96;  < (2, 4)
  sqr2(Z2Z2, b.z, K8P);
  mul2x(U1, a.x, Z2Z2, K8P);     // 12 * 2 + 12 * 8 = 120, 12 * 4 + 12 * 2 = 72;  < 2
  mul2x(U2, b.x, Z1Z1, K8P);
  { f2 t; mul2x(t, a.y, b.z, K8P); mul2x(S1, t, Z2Z2, K8P); }              // 2 * 4 + 2 * 8 = 24; 2 * 2 + 2 * 8 = 20;  < 2
  { f2 t; mul2x(t, b.y, a.z, K8P); mul2x(S2, t, Z1Z1, K8P); }
  sub2(H, U2, U1, K4P);          // < 6
  sub2(rr, S2, S1, K4P);         // < 6
  if (is_zero2(H)) {
    if (is_zero2(rr)) g2_dbl(a.x, a.y, a.z);   // a == b
    else a.inf = true;                         // a == -b
    return;
  }
  dbl2(rr, rr);                  // < 12
  f2 I; dbl2(I, H); sqr2(I, I, K16P);                                       // 2H < 12: 2 * 12 * 28 = 672;  < (2, 4)
  f2 J; mul2x(J, H, I, K8P);     // 6 * 2 + 6 * 8 = 60, 6 * 4 + 6 * 2 = 36;  < 2
  f2 V; mul2x(V, U1, I, K8P);    // < 2
  f2 X3; sqr2(X3, rr, K16P);     // 2 * 12 * 28 = 672;  < (2, 4)
  { f2 jv; dbl2(jv, V); add2(jv, jv, J); sub2(X3, X3, jv, K8P); }          // jv < 6: X3 < 12
  f2 Y3; { f2 w; sub2(w, V, X3, K16P); mul2x(Y3, rr, w, K32P); }           // w < 18: 600;  < 2
  { f2 sj; mul2x(sj, S1, J, K4P); dbl2(sj, sj); sub2(Y3, Y3, sj, K8P); }   // 2 * 2 + 2 * 4 = 12; sj < 4: Y3 < 10
  fold2(Y3, Y3);                 // < 2
  f2 Z3;
  { f2 zs; add2(zs, a.z, b.z); sqr2(zs, zs, K16P);                          // < 8: 2 * 8 * 24 = 384;  < (2, 4)
    sub2(zs, zs, Z1Z1, K8P); sub2(zs, zs, Z2Z2, K8P);                       // < 20
    mul2x(Z3, zs, H, K8P); }     // 20 * 6 + 20 * 8 = 280, 20 * 6 + 20 * 6 = 240;  < 2
  a.x = X3; a.y = Y3; a.z = Z3;
}


// ---- the same for G1 (E: y^2 = x^3 + 4 over Fp), for the merged G1 MSM's bucket sums ----
// coordinates X < 12p, Y < 2p, Z < 4p as for G2; every formula's bound next to it
struct pt1 { f x, y, z; bool inf; };
SSB_INL void pt1_from_aff(pt1& a, const g1_aff& p) {
  a.inf = p.inf != 0;
#if defined(__HIP_DEVICE_COMPILE__)
  __asm__ __volatile__("" ::: "memory");
#endif
  from_engine_shift(a.x, p.x); from_engine_shift(a.y, p.y);
  a.z = cst(ONE28);
}
SSB_INL void pt1_to_engine(g1_jac& r, const pt1& a) {
  if (a.inf) { jac_set_inf(r); return; }
  f x, z; fold(x, a.x); fold(z, a.z);
  to_engine_shift(r.x, x); to_engine_shift(r.y, a.y); to_engine_shift(r.z, z);
}
// dbl-2009-l over Fp (a = 0); (Y = 0 has no point of G1's order: never infinity)
SSB_INL void g1_dbl28(f& X, f& Y, f& Z) {
  f A, B, C, t, D, E, F, X3, Y3, Z3;
  sqr(A, X);                     // X < 12: 144;  < 2
  sqr(B, Y);                     // < 2
  sqr(C, B);                     // < 2
  add(t, X, B); sqr(t, t);       // < 14: 196;  < 2
  dbl_sub_sub(D, t, A, C, KK8P); // 2 (t + 8p - A - C) < 20
  fold(D, D);                    // < 2
  mul_small(E, A, 3);            // < 6
  sqr(F, E);                     // 36;  < 2
  sub_dbl(X3, F, D, KK8P);       // F + 8p - 2D < 10
  { f w; sub(w, D, X3, K16P); mul(Y3, E, w); }                             // w < 18: 6 * 18 = 108;  < 2
  { f c8; mul_small(c8, C, 8); sub(Y3, Y3, c8, K32P); fold(Y3, Y3); }     // c8 < 16: < 34, folded < 2
  { f y2; add_raw(y2, Y, Y); mul(Z3, y2, Z); }                             // 4 * 4 = 16;  < 2
  X = X3; Y = Y3; Z = Z3;
}
// a += P (madd-2007-bl), P affine (engine form in global memory); complete like pt2_madd
SSB_INL void pt1_madd(pt1& a, const g1_aff& p) {
  if (p.inf) return;
  if (a.inf) { pt1_from_aff(a, p); return; }
  f Z1Z1, U2, S2, H, rr;
  sqr(Z1Z1, a.z);                // Z1 < 4: 16;  < 2
  {
    f x2, y2;
#if defined(__HIP_DEVICE_COMPILE__)
    __asm__ __volatile__("" ::: "memory");
#endif
    from_engine_shift(x2, p.x); from_engine_shift(y2, p.y);               // < 2
    mul(U2, x2, Z1Z1);           // < 2
    f t; mul(t, y2, a.z); mul(S2, t, Z1Z1);                                // 8, 4;  < 2
  }
  sub(H, U2, a.x, K16P);         // X1 < 12: < 18
  sub(rr, S2, a.y, K4P);         // Y1 < 2: < 6
  if (is_zero(H)) {
    if (is_zero(rr)) { pt1_from_aff(a, p); g1_dbl28(a.x, a.y, a.z); }     // a == P
    else a.inf = true;                                                     // a == -P
    return;
  }
  f Z3; mul(Z3, a.z, H); dbl(Z3, Z3);                                      // 4 * 18 = 72;  < 2, doubled < 4
  dbl(rr, rr);                   // < 12
  f I, J, V;
  { f HH; sqr(HH, H); dbl(I, HH); dbl(I, I); }                             // 324;  I < 8
  mul(J, H, I);                  // 18 * 8 = 144;  < 2
  mul(V, a.x, I);                // 12 * 8 = 96;  < 2
  f X3; sqr(X3, rr);             // 144;  < 2
  { f jv; dbl(jv, V); add(jv, jv, J); sub(X3, X3, jv, K8P); }              // jv < 6: X3 < 10
  f Y3; { f w; sub(w, V, X3, K16P); mul(Y3, rr, w); }                      // w < 18: 12 * 18 = 216;  < 2
  { f yj; mul(yj, a.y, J); dbl(yj, yj); sub(Y3, Y3, yj, K8P); }            // 2 * 2;  yj < 4: < 10
  fold(Y3, Y3);                  // < 2
  a.x = X3; a.y = Y3; a.z = Z3;
}

}  // namespace r28
}  // namespace ssb
