// ssb_f28_field.h -- reduced-radix Fp for the per-share kernels (round 6): the G2 subgroup checks
// (ssb_f28.h) and the fixed-exponent powers of the square roots (fp_pow_sw_inl, ssb_field.h).
// Included by ssb_field.h after the engine's fp type (for the conversions).
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
#include "ssb_f28_consts.h"

namespace ssb {
namespace r28 {

struct f { uint32_t l[14]; };
struct f2 { f c0, c1; };
constexpr uint32_t M28 = (1u << 28) - 1;

// re-slice a 12 x 32-bit integer (< 2^384) into 14 x 28-bit limbs
SSB_INL void from32(f& r, const uint32_t* w) {
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const int b = 28 * k, i = b >> 5, s = b & 31;
    uint32_t v = w[i < 12 ? i : 11] >> s;
    if (s > 4 && i + 1 < 12) v |= w[i + 1] << (32 - s);
    r.l[k] = i < 12 ? (v & M28) : 0u;
  }
}
// ... and back (a normalized value < 2^384)
SSB_INL void to32(uint32_t* w, const f& a) {
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int b = 32 * i, k = b / 28, s = b % 28;
    uint32_t v = a.l[k] >> s;
    if (k + 1 < 14) v |= a.l[k + 1] << (28 - s);
    if (s > 24 && k + 2 < 14) v |= a.l[k + 2] << (56 - s);
    w[i] = v;
  }
}

// r = a b / 2^392 mod p, r < 2p normalized.  Requires every limb product < 2^60 and a b < R p.
SSB_INL void mul(f& r, const f& a, const f& b) {
  SSB_CNT(fp_mul);
  uint32_t m[14];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; ++k) {
#pragma unroll
    for (int j = 0; j < 14; ++j)
      if (k - j >= 0 && k - j < 14) acc += (uint64_t)a.l[j] * b.l[k - j];
#pragma unroll
    for (int j = 0; j < 14; ++j)
      if (j < k && k - j < 14) acc += (uint64_t)m[j] * P28[k - j];
    if (k < 14) {
      m[k] = ((uint32_t)acc * P28_INV) & M28;
      acc += (uint64_t)m[k] * P28[0];   // the low 28 bits become zero
    } else {
      r.l[k - 14] = (uint32_t)acc & M28;
    }
    acc >>= 28;
  }
  r.l[13] = (uint32_t)acc;
}
// r = a^2 / 2^392 mod p, r < 2p normalized: the column's cross products a_i a_j (i < j) once, doubled,
// plus the square term -- 105 limb products instead of 196 before the reduction's 196 (the square-root
// powers of decompression are ~85% squarings).  Requires limbs < 2^30 and a^2 < R p.
SSB_INL void sqr(f& r, const f& a) {
  SSB_CNT(fp_mul);
  uint32_t m[14];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; ++k) {
    uint64_t x = 0;
#pragma unroll
    for (int j = 0; j < 14; ++j)
      if (k - j > j && k - j < 14) x += (uint64_t)a.l[j] * a.l[k - j];
    acc += x + x;   // (x < 7 * 2^56: with the square term and the reduction the column stays < 2^61)
    if ((k & 1) == 0 && k / 2 < 14) acc += (uint64_t)a.l[k / 2] * a.l[k / 2];
#pragma unroll
    for (int j = 0; j < 14; ++j)
      if (j < k && k - j < 14) acc += (uint64_t)m[j] * P28[k - j];
    if (k < 14) {
      m[k] = ((uint32_t)acc * P28_INV) & M28;
      acc += (uint64_t)m[k] * P28[0];
    } else {
      r.l[k - 14] = (uint32_t)acc & M28;
    }
    acc >>= 28;
  }
  r.l[13] = (uint32_t)acc;
}
// r = (a b + c d) / 2^392 mod p, r < 2p: both products summed into each column before the column's
// reduction (one reduction for two products).  Requires limb products < 2^58 and a b + c d < R p.
SSB_INL void mul2(f& r, const f& a, const f& b, const f& c, const f& d) {
  uint32_t m[14];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; ++k) {
#pragma unroll
    for (int j = 0; j < 14; ++j)
      if (k - j >= 0 && k - j < 14) acc += (uint64_t)a.l[j] * b.l[k - j];
#pragma unroll
    for (int j = 0; j < 14; ++j)
      if (k - j >= 0 && k - j < 14) acc += (uint64_t)c.l[j] * d.l[k - j];
#pragma unroll
    for (int j = 0; j < 14; ++j)
      if (j < k && k - j < 14) acc += (uint64_t)m[j] * P28[k - j];
    if (k < 14) {
      m[k] = ((uint32_t)acc * P28_INV) & M28;
      acc += (uint64_t)m[k] * P28[0];
    } else {
      r.l[k - 14] = (uint32_t)acc & M28;
    }
    acc >>= 28;
  }
  r.l[13] = (uint32_t)acc;
}

// carry normalization: limbs 0..12 < 2^28 (inputs: limbs < 2^31)
SSB_INL void norm(f& x) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const uint32_t v = x.l[i] + c;
    x.l[i] = v & M28;
    c = v >> 28;
  }
  x.l[13] += c;
}
// r = a + b (normalized)
SSB_INL void add(f& r, const f& a, const f& b) {
#pragma unroll
  for (int i = 0; i < 14; ++i) r.l[i] = a.l[i] + b.l[i];
  norm(r);
}
// r = a + b, limbs NOT normalized (< 2^29 for normalized inputs): a product operand only
SSB_INL void add_raw(f& r, const f& a, const f& b) {
#pragma unroll
  for (int i = 0; i < 14; ++i) r.l[i] = a.l[i] + b.l[i];
}
// r = a + K - b (normalized), K a spread multiple of p (gen_f28.py) above b's value
SSB_INL void sub(f& r, const f& a, const f& b, const uint32_t* K) {
#pragma unroll
  for (int i = 0; i < 14; ++i) r.l[i] = a.l[i] + K[i] - b.l[i];
  norm(r);
}
// r = K - b, limbs NOT normalized (< 2^29): a product operand only
SSB_INL void neg_raw(f& r, const f& b, const uint32_t* K) {
#pragma unroll
  for (int i = 0; i < 14; ++i) r.l[i] = K[i] - b.l[i];
}
SSB_INL void dbl(f& r, const f& a) { add(r, a, a); }
// r = k a (normalized), k <= 8
SSB_INL void mul_small(f& r, const f& a, uint32_t k) {
#pragma unroll
  for (int i = 0; i < 14; ++i) r.l[i] = a.l[i] * k;
  norm(r);
}
// r = 2 (a + KK - b - c) (normalized), KK a double-spread multiple of p above b + c
SSB_INL void dbl_sub_sub(f& r, const f& a, const f& b, const f& c, const uint32_t* KK) {
#pragma unroll
  for (int i = 0; i < 14; ++i) r.l[i] = 2u * (a.l[i] + KK[i] - b.l[i] - c.l[i]);
  norm(r);
}
// r = a + KK - 2 b (normalized), KK a double-spread multiple of p above 2b
SSB_INL void sub_dbl(f& r, const f& a, const f& b, const uint32_t* KK) {
#pragma unroll
  for (int i = 0; i < 14; ++i) r.l[i] = a.l[i] + KK[i] - 2u * b.l[i];
  norm(r);
}
// r == x (mod p), r < 2p; x normalized, x < 2^12 p.  q = floor((x >> 336) / ((p >> 336) + 1)) is at
// most floor(x / p) and at least floor(x / p) - 1, so x - q p lies in [0, 2p).
SSB_INL void fold(f& r, const f& x) {
  const uint64_t hi = ((uint64_t)x.l[13] << 28) | x.l[12];
  const uint32_t q = (uint32_t)((double)hi * F28_INV_PHI);
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    acc += (int64_t)x.l[i] - (int64_t)((uint64_t)q * P28[i]);
    r.l[i] = (uint32_t)acc & M28;
    acc >>= 28;   // (arithmetic)
  }
  r.l[13] = (uint32_t)(acc + (int64_t)x.l[13] - (int64_t)((uint64_t)q * P28[13]));
}
// canonical residue of x < 2p (normalized): x or x - p
SSB_INL void canon(f& r, const f& x) {
  f t;
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    const int32_t v = (int32_t)x.l[i] - (int32_t)P28[i] + br;
    t.l[i] = (uint32_t)v & M28;
    br = v >> 28;   // 0 or -1 (limbs < 2^28)
  }
  const bool keep = br != 0;   // x < p
#pragma unroll
  for (int i = 0; i < 14; ++i) r.l[i] = keep ? x.l[i] : t.l[i];
}
// x == 0 (mod p) for a normalized x < 2^12 p
SSB_INL bool is_zero(const f& x) {
  f y; fold(y, x);
  f z; canon(z, y);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) o |= z.l[i];
  return o == 0;
}
// a == b (mod p) for normalized values below 2^12 p and 63 p
SSB_INL bool eq(const f& a, const f& b) { f d; sub(d, a, b, K64P); return is_zero(d); }
SSB_INL f cst(const uint32_t* c) { f r; for (int i = 0; i < 14; ++i) r.l[i] = c[i]; return r; }
// the engine's Montgomery form (R = 2^384) -> this one (R = 2^392): value * 2^400 / 2^392, < 2p
SSB_INL void from_engine(f& r, const fp& a) { f t; from32(t, a.l); mul(r, t, cst(C_2_400)); }
// the same conversion without a product: the 12 x 32-bit limbs (a value < p) re-sliced 8 bits up
// (value * 2^8 < 2^389), then folded below 2p
SSB_INL void from_engine_shift(f& r, const fp& a) {
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const int b = 28 * k - 8;
    uint32_t v;
    if (b < 0) {
      v = a.l[0] << 8;
    } else {
      const int i = b >> 5, s = b & 31;
      v = a.l[i] >> s;
      if (s > 4 && i + 1 < 12) v |= a.l[i + 1] << (32 - s);
    }
    r.l[k] = v & M28;
  }
  fold(r, r);
}
// ... and back without a product: x 2^-8 by one 8-bit Montgomery step ((x + m p) / 2^8 < 1.01 p for a
// normalized x < 2p), then the canonical residue, re-sliced into 12 x 32-bit limbs
SSB_INL void to_engine_shift(fp& r, const f& x) {
  const uint32_t m = (x.l[0] * P28_INV) & 0xffu;
  uint32_t z[14];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    c += (uint64_t)m * P28[i] + x.l[i];
    z[i] = i < 13 ? (uint32_t)c & M28 : (uint32_t)c;
    c >>= 28;
  }
  f y;
#pragma unroll
  for (int i = 0; i < 14; ++i) y.l[i] = ((z[i] >> 8) | (i < 13 ? z[i + 1] << 20 : 0u)) & (i < 13 ? M28 : ~0u);
  f cn; canon(cn, y);
  to32(r.l, cn);
}
// ... and back, fully reduced: (x 2^392) 2^384 / 2^392 = x 2^384, canonical
SSB_INL void to_engine(fp& r, const f& a) { f t; mul(t, a, cst(C_2_384)); f c; canon(c, t); to32(r.l, c); }

// a^e for a sliding-window schedule (gen_exp_chains.py) in this representation: the engine's
// fp_pow_sw_inl body (8 odd powers picked by a switch on the uniform digit), every product a
// reduced-radix one.  In and out in the engine's Montgomery form, out fully reduced.  All values stay
// below 2p, so every product's operands satisfy a b < R p.
SSB_INL void pow_sw(fp& r, const fp& a, const uint8_t* sch, int n) {
  f t0, t1, t2, t3, t4, t5, t6, t7, a2;
  from_engine(t0, a);
  sqr(a2, t0);
  mul(t1, t0, a2); mul(t2, t1, a2); mul(t3, t2, a2); mul(t4, t3, a2);
  mul(t5, t4, a2); mul(t6, t5, a2); mul(t7, t6, a2);
  auto pick = [&](int i) -> f {
    switch (i) {
      case 0: return t0; case 1: return t1; case 2: return t2; case 3: return t3;
      case 4: return t4; case 5: return t5; case 6: return t6; default: return t7;
    }
  };
  f acc = pick((sch[1] - 1) >> 1);
  for (int s = 1; s < n; ++s) {
    const int sq = sch[2 * s], d = sch[2 * s + 1];
    for (int k = 0; k < sq; ++k) sqr(acc, acc);
    if (d) { const f m = pick((d - 1) >> 1); mul(acc, acc, m); }
  }
  to_engine(r, acc);
}

}  // namespace r28
}  // namespace ssb
