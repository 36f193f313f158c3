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
      fp v;
      if (i < ncoord) v = g.s[src + i];
      else v = (i == ncoord) ? fp_one() : fp_zero();
      g.s[dst + i] = v;
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
        fp v = g.s[e + role];
        if (d < 0 && (role == 2 || role == 3)) fp_neg(v, v);
        g.s[tmp + role] = v;
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
        fp v = g.s[e + role];
        if (d < 0 && role == 1) fp_neg(v, v);
        g.s[tmp + role] = v;
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
  if (fp_is_zero(g.s[acc + 4]) && fp_is_zero(g.s[acc + 5])) exc |= 1u;
  bool eq = true;
  for (int i = 0; i < 4; ++i) eq = eq && fp_is_zero(g.s[tmp + 4 + i]);
  return eq;
}

// dst = -src for a G2 Jacobian point (6 slots; negate Y)
template <class GR> SSB_INL void g2_neg_copy(GR& g, int src, int dst) {
  constexpr int G = G2_ADD_G;
  LP_FOR(G) {
    if (role < 6) {
      fp v = g.s[src + role];
      if (role == 2 || role == 3) fp_neg(v, v);
      g.s[dst + role] = v;
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

}  // namespace lane
}  // namespace ssb
