// ssb_lane_ops.h -- group-level routines built from the lane-group programs: scalar
// multiplications, the G2 subgroup check, point sums.  Everything here is written for one group
// (G lanes on the device, a role loop on the host): slots are group-relative indices into g.s.
//
// Exceptional inputs: every addition program carries zero checks (an input at infinity, or
// H = 0: doubling / opposite points).  A routine ORs their result into `exc`; a share whose
// routine raised `exc` is recomputed by the exact single-lane code (the callers' fallback), so
// results are exact for every input, including adversarial points of small order.
#pragma once
#include "ssb_lane.h"

namespace ssb {
namespace lane {

// ---- program calls (inputs/outputs by group-relative slot) ----
template <class GR> SSB_INL void lg_reset_flag(const GR& g) {
  LP_FOR(1) { if (role == 0) *g.flag = 0u; }
  LP_SYNC();
}
template <class GR> SSB_INL void g2_dbl(GR& g, int a, int d) { g.a = a; g.d = d; lp_g2_dbl(g); }
template <class GR> SSB_INL void g2_add(GR& g, int a, int b, int d, uint32_t& exc) {
  g.a = a; g.b = b; g.d = d;
  lg_reset_flag(g);
  lp_g2_add(g);
  exc |= lp_fired(*g.flag, G2_ADD_CHECK_MASKS, G2_ADD_NCHECK) ? 1u : 0u;
}
template <class GR> SSB_INL void g2_madd(GR& g, int a, int b, int d, uint32_t& exc) {
  g.a = a; g.b = b; g.d = d;
  lg_reset_flag(g);
  lp_g2_madd(g);
  exc |= lp_fired(*g.flag, G2_MADD_CHECK_MASKS, G2_MADD_NCHECK) ? 1u : 0u;
}
template <class GR> SSB_INL void g1_dbl(GR& g, int a, int d) { g.a = a; g.d = d; lp_g1_dbl(g); }
template <class GR> SSB_INL void g1_add(GR& g, int a, int b, int d, uint32_t& exc) {
  g.a = a; g.b = b; g.d = d;
  lg_reset_flag(g);
  lp_g1_add(g);
  exc |= lp_fired(*g.flag, G1_ADD_CHECK_MASKS, G1_ADD_NCHECK) ? 1u : 0u;
}
template <class GR> SSB_INL void g1_madd(GR& g, int a, int b, int d, uint32_t& exc) {
  g.a = a; g.b = b; g.d = d;
  lg_reset_flag(g);
  lp_g1_madd(g);
  exc |= lp_fired(*g.flag, G1_MADD_CHECK_MASKS, G1_MADD_NCHECK) ? 1u : 0u;
}

// affine (n coords) at `src` -> Jacobian (n coords + Z = 1 in the last n/2) at `dst`
template <int G, class GR> SSB_INL void lg_aff_to_jac(GR& g, int src, int dst, int ncoord) {
  LP_FOR(G) {
    for (int i = role; i < ncoord + ncoord / 2; i += G) {
      if (i < ncoord) g.s[dst + i] = g.s[src + i];
      else lp_put(g.s + dst + i, (i == ncoord) ? lv_one() : lv_zero());
    }
  }
  LP_SYNC();
}

template <int G, class GR> SSB_INL void lg_copy(GR& g, int src, int dst, int n) {
  LP_FOR(G) { for (int i = role; i < n; i += G) g.s[dst + i] = g.s[src + i]; }
  LP_SYNC();
}

// ---- windowed multiplication: regular signed-window recoding (Joye-Tunstall), w = 4 ----
// k odd: k = sum d_i 16^i, d_i odd in [-15, 15], 16 digits, top digit positive, so every
// window adds a table entry (no data-dependent control flow across the groups of a wave).

// [k]P for an affine G2 point P at slot `p` (4 slots) and an ODD 64-bit scalar, w = 4 regular
// window.  Table of odd multiples at `tab` (8 x 6 slots), accumulator / result at `acc` (6),
// temporary B operand at `tmp` (6).
template <class GR> SSB_INL void g2_mul_u64_odd(GR& g, int p, uint64_t k, int tab, int acc, int tmp, uint32_t& exc) {
  constexpr int G = G2_ADD_G;
  // table: T1 = P, T2 = 2P (at tmp), T3 = T2 + P, T(2j+1) = T(2j-1) + T2
  lg_aff_to_jac<G>(g, p, tab, 4);
  g2_dbl(g, tab, tmp);
  g2_madd(g, tmp, p, tab + 6, exc);
  for (int j = 2; j < 8; ++j) g2_add(g, tab + 6 * (j - 1), tmp, tab + 6 * j, exc);
  // digits, most significant first
  int dig[16];
  {
    uint64_t kk = k;
    for (int j = 0; j < 15; ++j) { const int d = (int)(kk & 31u) - 16; dig[j] = d; kk = (kk - (uint64_t)(int64_t)d) >> 4; }
    dig[15] = (int)kk;
  }
  lg_copy<G>(g, tab + 6 * ((dig[15] - 1) >> 1), acc, 6);
  for (int w = 14; w >= 0; --w) {
    g2_dbl(g, acc, acc); g2_dbl(g, acc, acc); g2_dbl(g, acc, acc); g2_dbl(g, acc, acc);
    const int d = dig[w];
    const int e = tab + 6 * (((d < 0 ? -d : d) - 1) >> 1);
    LP_FOR(G) {
      if (role < 6) {
        lv v = lp_get(g.s + e + role);
        if (d < 0 && (role == 2 || role == 3)) lv_neg(v);
        lp_put(g.s + tmp + role, v);
      }
    }
    LP_SYNC();
    g2_add(g, acc, tmp, acc, exc);
  }
}

template <class GR> SSB_INL void g1_mul_u64_odd(GR& g, int p, uint64_t k, int tab, int acc, int tmp, uint32_t& exc) {
  constexpr int G = G1_ADD_G;
  lg_aff_to_jac<G>(g, p, tab, 2);
  g1_dbl(g, tab, tmp);
  g1_madd(g, tmp, p, tab + 3, exc);
  for (int j = 2; j < 8; ++j) g1_add(g, tab + 3 * (j - 1), tmp, tab + 3 * j, exc);
  int dig[16];
  {
    uint64_t kk = k;
    for (int j = 0; j < 15; ++j) { const int d = (int)(kk & 31u) - 16; dig[j] = d; kk = (kk - (uint64_t)(int64_t)d) >> 4; }
    dig[15] = (int)kk;
  }
  lg_copy<G>(g, tab + 3 * ((dig[15] - 1) >> 1), acc, 3);
  for (int w = 14; w >= 0; --w) {
    g1_dbl(g, acc, acc); g1_dbl(g, acc, acc); g1_dbl(g, acc, acc); g1_dbl(g, acc, acc);
    const int d = dig[w];
    const int e = tab + 3 * (((d < 0 ? -d : d) - 1) >> 1);
    LP_FOR(G) {
      if (role < 3) {
        lv v = lp_get(g.s + e + role);
        if (d < 0 && role == 1) lv_neg(v);
        lp_put(g.s + tmp + role, v);
      }
    }
    LP_SYNC();
    g1_add(g, acc, tmp, acc, exc);
  }
}

// G2 membership psi(P) == [x]P for an affine, non-infinity P at slot `p` (4 slots); uses
// `acc` (6) and `tmp` (6).  Returns the verdict; exc is raised when an addition was exceptional.
template <class GR> SSB_INL bool g2_subgroup_check(GR& g, int p, int acc, int tmp, uint32_t& exc) {
  constexpr int G = G2_ADD_G;
  lg_aff_to_jac<G>(g, p, acc, 4);
  for (int i = 62; i >= 0; --i) {
    g2_dbl(g, acc, acc);
    if ((BLS_X_ABS >> i) & 1ull) g2_madd(g, acc, p, acc, exc);
  }
  // -psi(P) (affine) at tmp, then (x' Z^2 - X, y' Z^3 - Y) at tmp + 4: zero iff [|x|]P == -psi(P)
  g.a = p; g.d = tmp; lp_g2_npsi_aff(g);
  g.a = acc; g.b = tmp; g.d = tmp + 4; lp_g2_eq_aff(g);
  // [|x|]P at infinity (2-torsion met by a doubling) is exceptional: exact fallback
  if (lv_is_zero(lp_get(g.s + acc + 4)) && lv_is_zero(lp_get(g.s + acc + 5))) exc |= 1u;
  bool eq = true;
  for (int i = 0; i < 4; ++i) eq = eq && lv_is_zero(lp_get(g.s + tmp + 4 + i));
  return eq;
}

// dst = -src for a G2 Jacobian point (6 slots; negate Y)
template <class GR> SSB_INL void g2_neg_copy(GR& g, int src, int dst) {
  constexpr int G = G2_ADD_G;
  LP_FOR(G) {
    if (role < 6) {
      lv v = lp_get(g.s + src + role);
      if (role == 2 || role == 3) lv_neg(v);
      lp_put(g.s + dst + role, v);
    }
  }
  LP_SYNC();
}
template <class GR> SSB_INL void g2_psi(GR& g, int a, int d) { g.a = a; g.d = d; lp_g2_psi(g); }

// acc = [|x|]P for a G2 Jacobian P at slot `p` (6 slots)
template <class GR> SSB_INL void g2_mul_x_abs(GR& g, int p, int acc, uint32_t& exc) {
  lg_copy<G2_ADD_G>(g, p, acc, 6);
  for (int i = 62; i >= 0; --i) {
    g2_dbl(g, acc, acc);
    if ((BLS_X_ABS >> i) & 1ull) g2_add(g, acc, p, acc, exc);
  }
}

// h_eff * P (RFC 9380 G.3, the same chain as ssb::clear_cofactor_g2) for a Jacobian P at `p`;
// result at `r`.  Work slots: 5 x 6 starting at `w`.
template <class GR> SSB_INL void g2_clear_cofactor(GR& g, int p, int r, int w, uint32_t& exc) {
  const int T1 = w, T2 = w + 6, T3 = w + 12, N = w + 18, X = w + 24;
  g2_mul_x_abs(g, p, X, exc);        // [|x|]P
  g2_neg_copy(g, X, T1);             // t1 = [x]P
  g2_psi(g, p, T2);                  // t2 = psi(P)
  g2_dbl(g, p, T3);                  // 2P
  g2_psi(g, T3, T3);
  g2_psi(g, T3, T3);                 // t3 = psi^2(2P)
  g2_neg_copy(g, T2, N);
  g2_add(g, T3, N, T3, exc);         // t3 = psi^2(2P) - psi(P)
  g2_add(g, T1, T2, T2, exc);        // t2 = [x]P + psi(P)
  g2_mul_x_abs(g, T2, N, exc);
  g2_neg_copy(g, N, T2);             // t2 = [x^2]P + [x]psi(P)
  g2_add(g, T3, T2, T3, exc);
  g2_add(g, T3, X, T3, exc);         // - t1 = [|x|]P
  g2_neg_copy(g, p, N);
  g2_add(g, T3, N, r, exc);          // - P
}

// ---- Fp12 programs (G = 64, one group per wave) ----
// an fp12 (engine form) out of / into 12 slots, in the fields' order (c0.c0.c0, c0.c0.c1, c0.c1.c0, ..)
SSB_INL void ld12(fp12& f, const lfp* s) {
  for (int k = 0; k < 12; ++k) ((fp*)&f)[k] = lv_out(lp_get(s + k));
}
SSB_INL void st12(lfp* s, const fp12& f) {
  for (int k = 0; k < 12; ++k) lp_put(s + k, lv_in(((const fp*)&f)[k]));
}
template <class GR> SSB_INL void f12_mul(GR& g, int a, int b, int d) { g.a = a; g.b = b; g.d = d; lp_fp12_mul(g); }
template <class GR> SSB_INL void f12_cyc_sqr(GR& g, int a, int d) { g.a = a; g.d = d; lp_fp12_cyc_sqr(g); }
template <class GR> SSB_INL void f12_cyc_sqr2(GR& g, int a, int d) { g.a = a; g.d = d; lp_fp12_cyc_sqr2(g); }
template <class GR> SSB_INL void f12_conj(GR& g, int a, int d) { g.a = a; g.d = d; lp_fp12_conj(g); }
template <class GR> SSB_INL void f12_frob(GR& g, int n, int a, int d) {
  g.a = a; g.d = d;
  if (n == 1) lp_fp12_frob1(g); else if (n == 2) lp_fp12_frob2(g); else lp_fp12_frob3(g);
}

// r = f^x (x = -0xd201000000010000), f cyclotomic; r != f.  The runs of squarings between the
// multiplications (1, 2, 3, 9, 32, 16) go two at a time through lp_fp12_cyc_sqr2 (three program
// stages instead of four: the first squaring's output stage is folded into the second's operands)
template <class GR> SSB_INL void f12_cyc_exp_x(GR& g, int r, int f) {
  lg_copy<64>(g, f, r, 12);
  int run = 0;
  for (int i = 62; i >= 0; --i) {
    ++run;
    const bool bit = ((BLS_X_ABS >> i) & 1ull) != 0;
    if (bit || i == 0) {
      for (; run >= 2; run -= 2) f12_cyc_sqr2(g, r, r);
      if (run) { f12_cyc_sqr(g, r, r); run = 0; }
      if (bit) f12_mul(g, r, f, r);
    }
  }
  f12_conj(g, r, r);
}

// slots d[0..11] = (a[0..5] as an Fp6)^-1 (the w-half zero), on one lane; out of line, so its
// Fp6 temporaries live in its own frame, not in every kernel that runs a final exponentiation
SSB_FN void fp6_inv_slots(const lfp* a, lfp* d) {
  // the slots hold an fp6's fields in order (c0.c0, c0.c1, c1.c0, ..): the six values in the engine's
  // form are laid out as an fp6 in the bytes of d's slots [0, 6) and inverted into those of [6, 11),
  // through flat pointers (no copies in a frame), then brought back into slots [0, 6)
  static_assert(6 * sizeof(lslot) >= sizeof(fp6) && 5 * sizeof(lslot) >= sizeof(fp6), "fp6 in the slots");
  fp6* x = (fp6*)(d);
  fp6* y = (fp6*)(d + 6);
  for (int k = 0; k < 6; ++k) { const fp v = lv_out(lp_get(a + k)); ((fp*)x)[k] = v; }
  fp6_inv(*y, *x);
  for (int k = 0; k < 6; ++k) { const fp v = ((const fp*)y)[k]; lp_put(d + k, lv_in(v)); }
  for (int k = 6; k < 12; ++k) lp_put(d + k, lv_zero());
}

// final exponentiation of the Fp12 value at `f` (in place); 7 x 12 work slots at `tmp`.
// Same chain as ssb::final_exponentiation.
template <class GR> SSB_INL void f12_final_exp(GR& g, int f, int tmp) {
  const int t0 = tmp, t1 = tmp + 12, t2 = tmp + 24, t3 = tmp + 36, t4 = tmp + 48, t5 = tmp + 60, t6 = tmp + 72;
  f12_conj(g, f, t0);
  // f^-1 = conj(f) / N with N = f conj(f) = c0^2 - v c1^2 in Fp6: the two Fp12 products run as
  // lane programs, only the Fp6 inversion of N stays on one lane (an Fp12 inversion there held
  // ~2 KB of private segment per lane, the largest on the batch streams).
  f12_mul(g, f, t0, t2);  // N: slots t2 .. t2+5 (the w-half is zero)
  LP_FOR(1) {
    if (role == 0) fp6_inv_slots(g.s + t2, g.s + t1);
  }
  LP_SYNC();
  f12_mul(g, t1, t0, t1);  // f^-1
  f12_mul(g, t0, t1, t2);
  lg_copy<64>(g, t2, t1, 12);
  f12_frob(g, 2, t2, t2);
  f12_mul(g, t2, t1, t2);
  f12_cyc_sqr(g, t2, t1);
  f12_conj(g, t1, t1);
  f12_cyc_exp_x(g, t3, t2);
  f12_cyc_sqr(g, t3, t4);
  f12_mul(g, t1, t3, t5);
  f12_cyc_exp_x(g, t1, t5);
  f12_cyc_exp_x(g, t0, t1);
  f12_cyc_exp_x(g, t6, t0);
  f12_mul(g, t6, t4, t6);
  f12_cyc_exp_x(g, t4, t6);
  f12_conj(g, t5, t5);
  f12_mul(g, t5, t2, t5);
  f12_mul(g, t4, t5, t4);
  f12_conj(g, t2, t5);
  f12_mul(g, t1, t2, t1);
  f12_frob(g, 3, t1, t1);
  f12_mul(g, t6, t5, t6);
  f12_frob(g, 1, t6, t6);
  f12_mul(g, t3, t0, t3);
  f12_frob(g, 2, t3, t3);
  f12_mul(g, t3, t1, t3);
  f12_mul(g, t3, t6, t3);
  f12_mul(g, t3, t4, f);
}

// Miller loop f_{|x|,Q}(P) (conjugated).  Slots: F = f (12) | T (6) at `F`; B = (xQ0, xQ1, yQ0,
// yQ1, xP, yP) at `b`.  Same schedule as ssb::miller_loop (the first squaring of f = 1 is a
// harmless no-op here).
template <class GR> SSB_INL void f12_miller(GR& g, int F, int b) {
  LP_FOR(64) {
    if (role < 18) {
      if (role >= 12 && role < 16) g.s[F + role] = g.s[b + role - 12];
      else lp_put(g.s + F + role, (role == 0 || role == 16) ? lv_one() : lv_zero());
    }
  }
  LP_SYNC();
  for (int i = 62; i >= 0; --i) {
    g.a = F; g.b = b + 4; g.d = F; lp_miller_iter(g);
    if ((BLS_X_ABS >> i) & 1ull) { g.a = F; g.b = b; g.d = F; lp_miller_addstep(g); }
  }
  f12_conj(g, F, F);
}

// Two Miller loops at once, f = f_{|x|,Q1}(P1) f_{|x|,Q2}(P2) (conjugated): the squaring of f is
// shared and both lines ride in the same product rounds (lp_miller_iter2: 8 program stages per
// iteration against 6 for one pair, so a two-pair check costs 1.33 single loops instead of 2).
// Slots: F = f (12) | T1 (6) | T2 (6) at `F`; b = (xQ1, yQ1 (4), xP1, yP1, xQ2, yQ2 (4), xP2, yP2)
// at `b`; bp = 4 work slots (P1, P2 copied there for the doubling steps).
template <class GR> SSB_INL void f12_miller2(GR& g, int F, int b, int bp) {
  LP_FOR(64) {
    if (role < 28) {
      lv v;
      if (role < 12) v = (role == 0) ? lv_one() : lv_zero();
      else if (role < 16) v = lp_get(g.s + b + role - 12);                       // T1 = (Q1, 1)
      else if (role < 18) v = (role == 16) ? lv_one() : lv_zero();
      else if (role < 22) v = lp_get(g.s + b + 6 + role - 18);                   // T2 = (Q2, 1)
      else if (role < 24) v = (role == 22) ? lv_one() : lv_zero();
      else v = lp_get(g.s + b + (role < 26 ? 4 + role - 24 : 10 + role - 26));   // (P1, P2)
      if (role < 24) lp_put(g.s + F + role, v);
      else lp_put(g.s + bp + role - 24, v);
    }
  }
  LP_SYNC();
  for (int i = 62; i >= 0; --i) {
    g.a = F; g.b = bp; g.d = F; lp_miller_iter2(g);
    if ((BLS_X_ABS >> i) & 1ull) { g.a = F; g.b = b; g.d = F; lp_miller_addstep2(g); }
  }
  f12_conj(g, F, F);
}

}  // namespace lane
}  // namespace ssb
