// ssb_units.h -- the per-work-unit bodies of the engine's kernels.  The gfx950 kernels in
// ssbls.hip call exactly these functions; the host op counter (tests/native/host_math.cpp,
// SSB_OPCOUNT) calls the same functions to measure the algorithmic work per unit
// (MADs/unit = 300*(Fp mul + Fp sqr) + 136*(Fr mul)).
#pragma once
#include "ssb_pairing.h"
#include "ssb_h2c.h"
#include "ssb_f28.h"

namespace ssb {

// FLAG_SUSPECT (failed batches only, ssb_k_bisect.hip): the share's job failed its committee
// consistency relation, so the share is checked on its own and left out of the exclusion check
// FLAG_DECIDED (failed batches, group-test mode): the share's verdict is final
enum : uint32_t { FLAG_CANDIDATE = 1u << 16, FLAG_SUSPECT = 1u << 17, FLAG_DECIDED = 1u << 18 };

// ---- random-linear-combination scalars -------------------------------------------------------
// lighthouse's verify_signature_sets draws one fresh non-zero 64-bit scalar per signature set from
// rand::thread_rng() (ChaCha12 keyed from the OS; RAND_BITS = 64, src/crypto/impls/blst.rs:12).
// Here: a 256-bit key drawn from getrandom() by the host for EVERY batch call (after the caller has
// handed the inputs over), passed to the kernels by value; share i's scalar is the first 64 bits
// of ChaCha12(key, counter = i, nonce = "SSB-RLC1").  The key never leaves the library, so a sender
// cannot predict k_i and cannot build shares whose errors cancel in the sums (sig_a + [k_b]D,
// sig_b - [k_a]D).  ssb_set_rlc_deterministic() switches a context to a key expanded from the
// caller's seed (reproducible runs and the forgery test only: NOT sound against chosen shares).
struct rlc_key { uint32_t w[8]; };

SSB_INL uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
#define SSB_QR(a, b, c, d)                     \
  a += b; d ^= a; d = rotl32(d, 16);           \
  c += d; b ^= c; b = rotl32(b, 12);           \
  a += b; d ^= a; d = rotl32(d, 8);            \
  c += d; b ^= c; b = rotl32(b, 7);
// words 0 and 1 of the ChaCha12 block (key, 64-bit block counter i, 64-bit nonce "SSB-RLC1")
SSB_INL uint64_t chacha12_u64(const rlc_key& key, uint64_t i) {
  const uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                           key.w[0], key.w[1], key.w[2], key.w[3], key.w[4], key.w[5], key.w[6], key.w[7],
                           (uint32_t)i, (uint32_t)(i >> 32), 0x2d425353u /* "SSB-" */, 0x31434c52u /* "RLC1" */};
  uint32_t x[16];
  for (int q = 0; q < 16; ++q) x[q] = in[q];
#pragma unroll 1
  for (int r = 0; r < 6; ++r) {             // 6 double rounds = 12 rounds
    SSB_QR(x[0], x[4], x[8], x[12]) SSB_QR(x[1], x[5], x[9], x[13])
    SSB_QR(x[2], x[6], x[10], x[14]) SSB_QR(x[3], x[7], x[11], x[15])
    SSB_QR(x[0], x[5], x[10], x[15]) SSB_QR(x[1], x[6], x[11], x[12])
    SSB_QR(x[2], x[7], x[8], x[13]) SSB_QR(x[3], x[4], x[9], x[14])
  }
  return (uint64_t)(x[0] + in[0]) | ((uint64_t)(x[1] + in[1]) << 32);
}
#undef SSB_QR

// the RLC scalars: odd, so the regular signed-window recoding applies and k != 0
// (63 secret random bits per share; lighthouse draws 64: the batch soundness error stays 2^-63)
SSB_INL uint64_t rlc_scalar_odd(const rlc_key& key, uint64_t i) { return chacha12_u64(key, i) | 1ull; }

// deterministic mode: key words = splitmix64 outputs 0..3 of the caller's seed
SSB_INL uint64_t splitmix64_at(uint64_t seed, uint64_t j) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (j + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
SSB_INL rlc_key rlc_key_from_seed(uint64_t seed) {
  rlc_key k;
  for (int j = 0; j < 4; ++j) {
    const uint64_t z = splitmix64_at(seed, (uint64_t)j);
    k.w[2 * j] = (uint32_t)z;
    k.w[2 * j + 1] = (uint32_t)(z >> 32);
  }
  return k;
}

SSB_INL g1_aff g1_neg_generator() {
  g1_aff ng; ng.x = fp_from_c(G1_GEN_X); ng.y = fp_from_c(G1_GEN_NEG_Y); ng.inf = 0;
  return ng;
}

// unit "decode": one share -> decompressed signature (+ subgroup check) and public key.
// flags: bits 0..7 signature DEC_* bits, bits 8..15 public-key DEC_* bits, bit 16 candidate
SSB_FN uint32_t unit_decode(g2_aff& sig, g1_aff& pk, const uint8_t* sig96, const uint8_t* pk48, int group_check) {
  uint32_t st = g2_decompress(sig, sig96);
  if ((st & DEC_OK) && group_check && g2_in_subgroup(sig)) st |= DEC_IN_GROUP;
  uint32_t pst = 0;
  if (pk48) pst = g1_decompress(pk, pk48);
  const bool cand = (st & DEC_OK) && !(st & DEC_INF) && (st & DEC_IN_GROUP) && (pst & DEC_OK) && !(pst & DEC_INF);
  return st | (pst << 8) | (cand ? FLAG_CANDIDATE : 0u);
}

// Split form used by the verify pipeline (independent per-share tasks, one thread each):
//   decode_sig | decode_pk   then   subgroup | rlc_sig | rlc_pk
// Inlined whole (no out-of-line call on the common path): the per-share kernels built from these
// run two waves per SIMD (SSB_LB2), which a call's frame and callee-saved registers prevent.
SSB_INL uint32_t unit_decode_sig(g2_aff& sig, const uint8_t* sig96) { return g2_decompress_inl(sig, sig96); }
SSB_INL uint32_t unit_decode_pk(g1_aff& pk, const uint8_t* pk48) { return g1_decompress_inl(pk, pk48); }
// The per-share subgroup checks run in the reduced radix (ssb_f28.h: 14 x 28-bit limbs, one
// v_mad_u64_u32 per limb product); SSB_SG_ENGINE=1 builds keep the engine's 12 x 32-bit form (A/B), and
// the op counter counts the algorithm in the engine's form (its units define the roofline's MADs).
// keep: the lane's r28::KEEP_WORDS words of LDS at stride 64 (the block's array + threadIdx.x)
SSB_INL uint32_t unit_subgroup(const g2_aff& sig, r28::keep_t* keep) {
#if defined(SSB_SG_ENGINE) || defined(SSB_OPCOUNT)
  (void)keep;
  return g2_in_subgroup_inl(sig) ? DEC_IN_GROUP : 0u;
#elif defined(__HIP_DEVICE_COMPILE__)
  return r28::g2_in_subgroup_keep<64>(sig, keep) ? DEC_IN_GROUP : 0u;
#else
  (void)keep;
  return r28::g2_in_subgroup(sig) ? DEC_IN_GROUP : 0u;
#endif
}
// (k odd: the RLC scalars are rlc_scalar_odd)
SSB_FN void unit_rlc_sig(g2_jac& r, const g2_aff& sig, uint64_t k) {
  const uint32_t kw[2] = {(uint32_t)k, (uint32_t)(k >> 32)};
  jac_mul_sw4_odd(r, sig, kw, 2);
}
SSB_FN void unit_rlc_pk(g1_jac& r, const g1_aff& pk, uint64_t k) {
  const uint32_t kw[2] = {(uint32_t)k, (uint32_t)(k >> 32)};
  jac_mul_sw4_odd(r, pk, kw, 2);
}
SSB_INL uint32_t combine_flags(uint32_t sf, uint32_t pf, uint32_t gf) {
  const uint32_t st = sf | gf;
  const bool cand = (st & DEC_OK) && !(st & DEC_INF) && (st & DEC_IN_GROUP) && (pf & DEC_OK) && !(pf & DEC_INF);
  return st | (pf << 8) | (cand ? FLAG_CANDIDATE : 0u);
}

// unit "rlc": r*sig and r*pk for the share's 64-bit RLC scalar
SSB_FN void unit_rlc(g2_jac& rsig, g1_jac& rpk, const g2_aff& sig, const g1_aff& pk, uint64_t r) {
  const uint32_t k[2] = {(uint32_t)r, (uint32_t)(r >> 32)};
  jac_mul_aff(rsig, sig, k, 2);
  jac_mul_aff(rpk, pk, k, 2);
}

// unit "verify_one": exact single-signature pairing check e(pk,H) == e(g1,sig)
SSB_FN bool unit_verify_one(const g1_aff& pk, const g2_aff& sig, const g2_aff& H) {
  fp12 f1, f2;
  miller_loop(f1, pk, H);
  g1_aff ng = g1_neg_generator();
  miller_loop(f2, ng, sig);
  fp12_mul(f1, f1, f2);
  fp12 e;
  final_exponentiation(e, f1);
  return fp12_is_one(e);
}

// unit "combine_term": lambda_i * sig_i (blst_p2_mult with 255-bit scalar).  Odd lambda: signed
// window directly; even lambda: (lambda + 1) sig - sig, exact for every point (unsafe_aggregate
// does not subgroup-check, so lambda + r would not do).  lambda < r: lambda + 1 fits 255 bits.
SSB_FN void unit_combine_term(g2_jac& r, const g2_aff& sig, const uint32_t* lam8) {
  if (sig.inf) { jac_set_inf(r); return; }
  uint32_t k[8];
  uint32_t c = (lam8[0] & 1u) ? 0u : 1u;
  const bool even = c != 0;
  for (int i = 0; i < 8; ++i) k[i] = addc(lam8[i], 0u, c, c);
  jac_mul_sw4_odd(r, sig, k, 8);
  if (even) { g2_aff n = sig; fp2_neg(n.y, n.y); jac_add_aff(r, r, n); }
}

// GLS split of a combine term for a signature KNOWN to lie in G2 (a verified candidate): on G2,
// psi acts as [x] with x = -u, u = |x| = 0xd201000000010000, and r = u^4 - u^2 + 1 < u^4, so a
// canonical scalar k < r has four base-u digits, k = d0 + d1 u + d2 u^2 + d3 u^3 (d_q < 2^64), and
//     [k] sig = [d0] sig + [d1] (-psi(sig)) + [d2] psi^2(sig) + [d3] (-psi^3(sig)).
// Each digit's 64-bit product runs on its own lane (a quarter of the 255-bit chain's latency); the
// group element is the same as blst_p2_mult(sig, k, 255), so the compressed sum is bit-identical.
// (unsafe_aggregate's shares are not group-checked: it keeps the 255-bit unit_combine_term.)
constexpr uint64_t GLS_U = 0xd201000000010000ull;
SSB_INL uint64_t gls_digit(const uint32_t* k8, int q) {
  uint64_t w[4];
  for (int i = 0; i < 4; ++i) w[i] = (uint64_t)k8[2 * i] | ((uint64_t)k8[2 * i + 1] << 32);
  uint64_t rem = 0;
  for (int step = 0; step <= q; ++step) {       // (w, rem) = divmod(w, u), q + 1 times
    uint64_t qt[4] = {0, 0, 0, 0};
    rem = 0;
    for (int i = 255; i >= 0; --i) {
      const uint64_t hi = rem >> 63;
      rem = (rem << 1) | ((w[i >> 6] >> (i & 63)) & 1ull);
      if (hi || rem >= GLS_U) { rem -= GLS_U; qt[i >> 6] |= 1ull << (i & 63); }
    }
    for (int i = 0; i < 4; ++i) w[i] = qt[i];
  }
  return rem;
}
// NAF masks of m < 2^62: m = sum_i 2^i (pos_i - neg_i), no two adjacent digits nonzero (with h = 3m:
// digit i is nonzero where bits i + 1 of h and m differ, +1 where h has the bit) -- a third of the
// positions nonzero against half for the binary digits
SSB_INL void naf_masks(uint64_t m, uint64_t& pos, uint64_t& neg) {
  const uint64_t h = 3 * m;
  pos = (h & ~m) >> 1;
  neg = (m & ~h) >> 1;
}
// [d] (+-psi^q(p)) -- digit q of a GLS split (sign as above); p in G2
SSB_FN void unit_gls_term(g2_jac& r, const g2_aff& sig, uint64_t d, int q) {
  if (sig.inf) { jac_set_inf(r); return; }
  g2_aff p = sig;
  for (int i = 0; i < q; ++i) g2_psi_aff(p, p);
  if (q & 1) fp2_neg(p.y, p.y);
  const uint32_t dw[2] = {(uint32_t)d, (uint32_t)(d >> 32)};
  jac_mul_aff(r, p, dw, 2);
}
SSB_FN void unit_combine_term_gls(g2_jac& r, const g2_aff& sig, const uint32_t* lam8, int q) {
  unit_gls_term(r, sig, gls_digit(lam8, q), q);
}

// unit "combine_sum": sum of t terms, affine, compressed (src/crypto/impls/blst.rs:74-86)
SSB_FN void unit_combine_sum(uint8_t* out96, const g2_jac* terms, uint32_t t) {
  g2_jac acc; jac_set_inf(acc);
  for (uint32_t k = 0; k < t; ++k) jac_add(acc, acc, terms[k]);
  g2_aff a; jac_to_aff(a, acc);
  g2_compress(out96, a);
}

// unit "lagrange": lambda_i = prod_{j!=i} x_j (x_j - x_i)^{-1} mod r (src/crypto/impls/blst.rs:19-39)
// with blst's inverse(0) = 0; one Fr inversion per job (Montgomery's trick).  `lam` receives
// canonical little-endian limbs (blst_scalar.b).
SSB_FN void unit_lagrange(fr* lam, const uint64_t* x, uint32_t t) {
  fr prefix = fr_one();
  for (uint32_t i = 0; i < t; ++i) {
    fr xi; fr_from_u64(xi, x[i]);
    fr den = fr_one();
    for (uint32_t k = 0; k < t; ++k) {
      if (k == i) continue;
      fr xk, d; fr_from_u64(xk, x[k]);
      fr_sub(d, xk, xi);
      fr_mul(den, den, d);
    }
    lam[i] = den;
    if (!fr_is_zero(den)) fr_mul(prefix, prefix, den);
  }
  fr inv; fr_inv(inv, prefix);            // inv = 1 / prod_{k nz} den_k
  for (int i = (int)t - 1; i >= 0; --i) {
    fr den = lam[i];
    fr out;
    if (fr_is_zero(den)) {
      out = fr_zero();
    } else {
      fr pre = fr_one();                  // prod_{k<i, nz} den_k (recomputed; t is small)
      for (int k = 0; k < i; ++k) { fr dk = lam[k]; if (!fr_is_zero(dk)) fr_mul(pre, pre, dk); }
      fr dinv; fr_mul(dinv, pre, inv);    // inv = 1/prod_{k<=i,nz} den_k  ->  pre*inv = 1/den_i
      fr_mul(inv, inv, den);
      fr xi; fr_from_u64(xi, x[i]);
      fr num = fr_one();
      for (uint32_t k = 0; k < t; ++k) {
        if ((int)k == i) continue;
        fr xk; fr_from_u64(xk, x[k]);
        fr_mul(num, num, xk);
      }
      fr_mul(out, num, dinv);
    }
    fr c; fr_from_mont(c, out);
    lam[i] = c;
  }
}

// ---- small-integer Lagrange fast path -------------------------------------------------------
// lambda_i = prod_{j!=i} x_j / (x_j - x_i) as a reduced rational, fraction by fraction (int64
// with overflow checks).  Returns true iff every lambda_i is an integer c_i (|c_i| < 2^62): then
// sum c_i sig_i == sum (lambda_i mod r) sig_i for points of order r, i.e. the reference's
// combination (src/crypto/impls/blst.rs:19-39,67-87) with t tiny scalars instead of t 255-bit
// ones.  Ids 1..t (SafeStake's usual committees) give c_i = (-1)^(i-1) binomial(t, i).
// Duplicate ids (a zero denominator) are never eligible.
SSB_INL int64_t i64_gcd(int64_t a, int64_t b) {
  if (a < 0) a = -a;
  if (b < 0) b = -b;
  while (b) { const int64_t t = a % b; a = b; b = t; }
  return a;
}
SSB_INL bool unit_lagrange_small(int64_t* c, const uint64_t* x, uint32_t t) {
  for (uint32_t i = 0; i < t; ++i) {
    int64_t num = 1, den = 1;
    for (uint32_t k = 0; k < t; ++k) {
      if (k == i) continue;
      if (x[k] >= (1ull << 62) || x[i] >= (1ull << 62)) return false;
      int64_t a = (int64_t)x[k], b = (int64_t)x[k] - (int64_t)x[i];
      if (b == 0) return false;
      int64_t g = i64_gcd(a, b); a /= g; b /= g;   // num/den and a/b both reduced: cross-reduce
      g = i64_gcd(a, den); a /= g; den /= g;
      g = i64_gcd(num, b); num /= g; b /= g;
      if (__builtin_mul_overflow(num, a, &num) || __builtin_mul_overflow(den, b, &den)) return false;
    }
    if (den == -1) { num = -num; den = 1; }
    if (den != 1 || num >= (1ll << 62) || num <= -(1ll << 62)) return false;
    c[i] = num;
  }
  return true;
}
// sum c_i P_i by interleaved signed binary (shared doublings), start at infinity; exact for every
// input (jac_add_aff handles infinity, doubling and opposite points).
SSB_FN void unit_combine_small(uint8_t* out96, const g2_aff* const* pts, const int64_t* c, uint32_t t) {
  int nb = 0;
  for (uint32_t i = 0; i < t; ++i) {
    const uint64_t m = (uint64_t)(c[i] < 0 ? -c[i] : c[i]);
    const int b = m ? 64 - __builtin_clzll(m) : 0;
    nb = b > nb ? b : nb;
  }
  g2_jac acc; jac_set_inf(acc);
  for (int b = nb - 1; b >= 0; --b) {
    jac_dbl(acc, acc);
    for (uint32_t i = 0; i < t; ++i) {
      const uint64_t m = (uint64_t)(c[i] < 0 ? -c[i] : c[i]);
      if ((m >> b) & 1ull) {
        g2_aff q = *pts[i];
        if (c[i] < 0) fp2_neg(q.y, q.y);
        jac_add_aff(acc, acc, q);
      }
    }
  }
  g2_aff a; jac_to_aff(a, acc);
  g2_compress(out96, a);
}
// the same, the points read as pts[idx[i]] (the device path: no array of point pointers in a frame)
// (NAF digits of each |c_i| -- |c_i| < 2^62 -- shared doublings: the registry ids' 48-bit
// coefficients cost ~16 additions per term instead of ~24; the group steps out of line, so the
// frame of the combine kernels holds no inlined doubling's temporaries -- round 5, private segments)
SSB_INL void combine_small_jac(g2_jac& acc, const g2_aff* __restrict__ pts, const uint32_t* __restrict__ idx,
                               const int64_t* c, uint32_t t) {
  uint64_t any = 0;
  for (uint32_t i = 0; i < t; ++i) {
    uint64_t ps, ng;
    naf_masks((uint64_t)(c[i] < 0 ? -c[i] : c[i]), ps, ng);
    any |= ps | ng;
  }
  const int nb = any ? 64 - __builtin_clzll(any) : 0;
  jac_set_inf(acc);
  for (int b = nb - 1; b >= 0; --b) {
    jac_dbl(acc, acc);
    for (uint32_t i = 0; i < t; ++i) {
      uint64_t ps, ng;
      naf_masks((uint64_t)(c[i] < 0 ? -c[i] : c[i]), ps, ng);
      const bool p1 = (ps >> b) & 1ull, n1 = (ng >> b) & 1ull;
      if (p1 || n1) {
        g2_aff q = pts[idx[i]];
        if ((c[i] < 0) != n1) fp2_neg(q.y, q.y);
        jac_add_aff(acc, acc, q);
      }
    }
  }
}
SSB_FN void unit_combine_small_at(uint8_t* out96, const g2_aff* __restrict__ pts, const uint32_t* __restrict__ idx,
                                  const int64_t* c, uint32_t t) {
  g2_jac acc;
  combine_small_jac(acc, pts, idx, c, t);
  g2_aff a; jac_to_aff(a, acc);
  g2_compress(out96, a);
}

// ---- registry-id Lagrange path ---------------------------------------------------------------
// Operator ids from the registry contract (src/node/node.rs:470-474) are arbitrary u64 (small in
// practice: < 2^16), so lambda_i is not an integer; it is a RATIO of small integers:
//     lambda_i = N_i / D_i,  N_i = prod_{j != i} x_j,  D_i = prod_{j != i} (x_j - x_i)
// (src/crypto/impls/blst.rs:19-39).  With M = lcm_i |D_i|: lambda_i = c_i / M, c_i = N_i (M / D_i),
// and for points of order r
//     sum_i lambda_i sig_i = [M^-1 mod r] (sum_i c_i sig_i)
// -- t products with small scalars (ids < 2^16, t = 3: |c_i| < 2^48) and ONE 255-bit product per job
// (its four GLS digits, unit_gls_term) instead of t of them.  Returns false when a value does not
// fit 62 bits, or ids repeat (the general path then runs).
SSB_INL bool unit_lagrange_ratio(int64_t* c, uint64_t* M, const uint64_t* x, uint32_t t) {
  int64_t L = 1;
  for (uint32_t i = 0; i < t; ++i) {
    if (x[i] >= (1ull << 62)) return false;
    int64_t d = 1;
    for (uint32_t j = 0; j < t; ++j) {
      if (j == i) continue;
      const int64_t df = (int64_t)x[j] - (int64_t)x[i];
      if (df == 0 || __builtin_mul_overflow(d, df, &d)) return false;
    }
    const int64_t a = d < 0 ? -d : d, g = i64_gcd(L, a);
    if (__builtin_mul_overflow(L / g, a, &L) || L >= (1ll << 62)) return false;
  }
  for (uint32_t i = 0; i < t; ++i) {
    int64_t d = 1, nn = 1;
    for (uint32_t j = 0; j < t; ++j) {
      if (j == i) continue;
      d *= (int64_t)x[j] - (int64_t)x[i];   // (fits: checked above)
      if (__builtin_mul_overflow(nn, (int64_t)x[j], &nn)) return false;
    }
    if (__builtin_mul_overflow(nn, L / d, &c[i]) || c[i] >= (1ll << 62) || c[i] <= -(1ll << 62)) return false;
  }
  *M = (uint64_t)L;
  return true;
}
// high 64 bits of a 64 x 64-bit product (32-bit halves)
SSB_INL uint64_t mulhi64(uint64_t a, uint64_t b) {
  const uint64_t a0 = (uint32_t)a, a1 = a >> 32, b0 = (uint32_t)b, b1 = b >> 32;
  const uint64_t p00 = a0 * b0, p01 = a0 * b1, p10 = a1 * b0, p11 = a1 * b1;
  const uint64_t mid = (p00 >> 32) + (uint32_t)p01 + (uint32_t)p10;
  return p11 + (p01 >> 32) + (p10 >> 32) + (mid >> 32);
}
// (hi:lo) / d for hi < d: quotient, *rem the remainder (shift-subtract; no 128-bit divide on the device)
SSB_INL uint64_t udiv128_64(uint64_t hi, uint64_t lo, uint64_t d, uint64_t* rem) {
  uint64_t q = 0;
  for (int i = 0; i < 64; ++i) {
    const uint64_t top = hi >> 63;
    hi = (hi << 1) | (lo >> 63);
    lo <<= 1;
    q <<= 1;
    if (top || hi >= d) { hi -= d; q |= 1ull; }
  }
  *rem = hi;
  return q;
}
// w (n little-endian 64-bit limbs) /= d, returns w mod d
SSB_INL uint64_t divmod_limbs(uint64_t* w, int n, uint64_t d) {
  uint64_t rem = 0;
  for (int i = n - 1; i >= 0; --i) w[i] = udiv128_64(rem, w[i], d, &rem);
  return rem;
}
// y = M^-1 mod r (canonical, 4 limbs) for 1 <= M < 2^62 -- without an Fr exponentiation: with
// a = r mod M and b = a^-1 mod M (extended Euclid on 64-bit integers), r b == 1 (mod M), so
// y' = (r b - 1) / M is an integer with M y' == -1 (mod r), and y = r - y'  (y' < r since b < M).
SSB_INL void inv_small_mod_r(uint64_t* y, uint64_t M) {
  uint64_t rl[4];
  for (int i = 0; i < 4; ++i) rl[i] = (uint64_t)R_LIMBS[2 * i] | ((uint64_t)R_LIMBS[2 * i + 1] << 32);
  if (M == 1) { y[0] = 1; y[1] = y[2] = y[3] = 0; return; }
  uint64_t w[4] = {rl[0], rl[1], rl[2], rl[3]};
  const uint64_t a = divmod_limbs(w, 4, M);
  int64_t t0 = 0, t1 = 1;                        // Bezout coefficients of a modulo M
  uint64_t r0 = M, r1 = a;
  while (r1) {
    const uint64_t qq = r0 / r1;
    const uint64_t r2 = r0 - qq * r1; r0 = r1; r1 = r2;
    const int64_t t2 = t0 - (int64_t)qq * t1; t0 = t1; t1 = t2;
  }
  const uint64_t b = t0 < 0 ? (uint64_t)(t0 + (int64_t)M) : (uint64_t)t0;   // (r0 == 1: r is prime, M < r)
  uint64_t v[5];                                 // r b - 1, five limbs
  uint64_t carry = 0;
  for (int i = 0; i < 4; ++i) {
    const uint64_t lo = rl[i] * b, hi = mulhi64(rl[i], b);
    v[i] = lo + carry;
    carry = hi + (v[i] < lo ? 1ull : 0ull);
  }
  v[4] = carry;
  for (int i = 0; i < 5; ++i) { const bool bw = v[i] == 0; v[i] -= 1ull; if (!bw) break; }
  divmod_limbs(v, 5, M);                         // exact: y' in v[0..3]
  uint64_t br = 0;
  for (int i = 0; i < 4; ++i) {
    const uint64_t d = rl[i] - v[i] - br;
    br = (rl[i] < v[i] || (rl[i] == v[i] && br)) ? 1ull : 0ull;
    y[i] = d;
  }
}
// the four base-u digits of k < r (the GLS split, gls_digit) in one pass: three divisions by u
SSB_INL void gls_digits4(uint64_t* d, const uint64_t* k) {
  uint64_t w[4] = {k[0], k[1], k[2], k[3]};
  for (int q = 0; q < 3; ++q) d[q] = divmod_limbs(w, 4, GLS_U);
  d[3] = w[0];   // (k < r < u^4)
}
// lambda_i mod r (canonical, unit_lagrange's output) by the ratio form when the ids allow it
// (unit_lagrange_ratio: lambda_i = c_i / M, |c_i|, M < 2^62 -- registry ids of committees up to t = 3
// and most of t = 4): M^-1 mod r by inv_small_mod_r (64-bit extended Euclid) and one Montgomery
// product per share (c_i R * M^-1 * R^-1 = c_i M^-1), instead of unit_lagrange's Fr exponentiation.
// Anything else (repeated ids, wider committees, values past 62 bits) takes unit_lagrange.
SSB_FN void unit_lagrange_fast(fr* lam, const uint64_t* x, uint32_t t) {
  constexpr uint32_t TMAX = 16;
  if (t <= TMAX) {
    int64_t c[TMAX];
    uint64_t M;
    if (unit_lagrange_ratio(c, &M, x, t)) {
      uint64_t y[4];
      inv_small_mod_r(y, M);
      fr yc;
      for (int i = 0; i < 4; ++i) { yc.l[2 * i] = (uint32_t)y[i]; yc.l[2 * i + 1] = (uint32_t)(y[i] >> 32); }
      for (uint32_t i = 0; i < t; ++i) {
        fr cm, l;
        fr_from_u64(cm, (uint64_t)(c[i] < 0 ? -c[i] : c[i]));
        fr_mul(l, cm, yc);
        if (c[i] < 0 && !fr_is_zero(l)) fr_sub(l, fr_zero(), l);
        lam[i] = l;
      }
      return;
    }
  }
  unit_lagrange(lam, x, t);
}
// ---- the ratio combine, lane-uniform (round 5) -------------------------------------------------
// sigma = [M^-1 mod r] T, T = sum_i c_i sig_i, for a job whose lambda_i = c_i / M (unit_lagrange_ratio),
// one lane per job, every lane of a wave on the same schedule (a 64-lane wave runs an addition
// wherever ANY lane needs one, so per-lane binary / NAF chains cost an addition at nearly every bit):
//   T      -- regular signed 4-bit windows (Joye-Tunstall: every digit odd, in [-15, 15], so every
//             window adds a table entry) over the t coefficients JOINTLY: one doubling chain for all
//             bases, tables of the odd multiples P, 3P, .., 15P of every base;
//   [k] T  -- k = M^-1 mod r as four base-u GLS digits (psi acts as [x] = [-u] on G2), the same
//             windows over the four digits jointly, one table of T's odd multiples normalised to
//             affine (one inversion) and its psi images: 60 doublings + 64 mixed additions for a
//             255-bit product, where four separate 64-bit binary chains cost 256 + 256.
// Per 3-of-4 registry job ~6.6k Fp products on ONE lane; the round-4 general combine ran twelve
// 64-bit binary chains (4 GLS lanes x 3 shares, ~2.9k each) on 16 lanes.  Same group element as
// blst_p2_mult(sig_i, lambda_i, 255) summed (src/crypto/impls/blst.rs:67-87): compressed bytes equal.
// Tables live in the caller's memory (device: a per-job region of the slot's workspace, read back
// with 16-byte loads; they do not fit the registers or a wave's share of LDS): RC_TAB_BYTES per job.
struct alignas(16) g2_xy { fp2 x, y; };     // affine table entry (a table entry is never infinity)
constexpr int RC_GROUP = 4;                 // bases per joint pass of T (tables 4 x 8 affine points)
// the per-job region: 32 affine entries (xy; X, Y of the Jacobian multiples until rc_normalize) | their
// Z | prefix products of the Z (2P parked there while a table is built)
constexpr size_t RC_XY_OFF = 0, RC_Z_OFF = 32 * sizeof(g2_xy), RC_PR_OFF = RC_Z_OFF + 32 * sizeof(fp2);
constexpr size_t RC_TAB_BYTES = RC_PR_OFF + 32 * sizeof(fp2);   // 12,288 B
static_assert(sizeof(g2_jac) <= 32 * sizeof(fp2), "2P fits the prefix area");

// digit j (0 = least significant) of the regular signed 4-bit recoding of an odd k < 2^(4W), read in
// any order without storing the recoding: with k_0 = k and k_{j+1} = (k_j - d_j) / 16 = 2 floor(k_j / 32) + 1,
// the low five bits of k_j are bits 4j+1 .. 4j+4 of k with bit 0 set, d_j = (k_j mod 32) - 16, and the
// top digit is k_{W-1} itself (odd, <= 15)
SSB_INL int sw4_digit(uint64_t k, int j, int W) {
  const uint64_t s = k >> (4 * j);
  return j == W - 1 ? (int)(s | 1ull) : (int)((s & 30ull) | 1ull) - 16;
}
// windows needed for an odd k: the smallest W with k < 2^(4W)
SSB_INL int sw4_windows(uint64_t k) { return k ? (64 - __builtin_clzll(k) + 3) / 4 : 1; }
// a += (+-) *qp in place (add-2007-bl, q Jacobian, read from memory where consumed; neg: -q), every
// special case (either side infinity, doubling, opposite points), few temporaries live
SSB_INL void jac_add_at(g2_jac& a, const g2_jac* __restrict__ qp, bool neg) {
  if (fp2_is_zero(qp->z)) return;
  if (jac_is_inf(a)) { a = *qp; if (neg) fp2_neg(a.y, a.y); return; }
  fp2 Z1Z1, Z2Z2, U1, S1, H, r;
  fp2_sqr(Z1Z1, a.z);
  { const fp2 z2 = qp->z; fp2_sqr(Z2Z2, z2); fp2_mul(S1, a.y, z2); }
  fp2_mul(S1, S1, Z2Z2);                                                        // Y1 Z2^3
  fp2_mul(U1, a.x, Z2Z2);                                                       // X1 Z2^2
  { const fp2 x2 = qp->x; fp2_mul(H, x2, Z1Z1); fp2_sub(H, H, U1); }            // U2 - U1
  { fp2 y2 = qp->y; if (neg) fp2_neg(y2, y2); fp2_mul(r, y2, a.z); fp2_mul(r, r, Z1Z1); fp2_sub(r, r, S1); }   // S2 - S1
  if (fp2_is_zero(H)) {
    if (fp2_is_zero(r)) jac_dbl(a, a); else jac_set_inf(a);
    return;
  }
  { const fp2 z2 = qp->z; fp2 t; fp2_add(t, a.z, z2); fp2_sqr(t, t); fp2_sub(t, t, Z1Z1); fp2_sub(t, t, Z2Z2); fp2_mul(a.z, t, H); }
  fp2_dbl(r, r);
  fp2 I; fp2_dbl(I, H); fp2_sqr(I, I);
  fp2 J; fp2_mul(J, H, I);
  fp2 V; fp2_mul(V, U1, I);
  fp2_sqr(a.x, r); fp2_sub(a.x, a.x, J); { fp2 t; fp2_dbl(t, V); fp2_sub(a.x, a.x, t); }       // r^2 - J - 2V
  fp2_sub(V, V, a.x); fp2_mul(a.y, r, V); fp2_mul(J, S1, J); fp2_dbl(J, J); fp2_sub(a.y, a.y, J);   // r (V - X3) - 2 S1 J
}
// a += (+-) *qp, q affine (madd-2007-bl, the special cases of jac_madd_at)
SSB_INL void jac_madd_xy(g2_jac& a, const g2_xy* __restrict__ qp, bool neg) {
  if (jac_is_inf(a)) { a.x = qp->x; a.y = qp->y; if (neg) fp2_neg(a.y, a.y); a.z = fp2_one(); return; }
  fp2 Z1Z1, r, H;
  fp2_sqr(Z1Z1, a.z);
  { fp2 S2, y2 = qp->y; if (neg) fp2_neg(y2, y2); fp2_mul(S2, y2, a.z); fp2_mul(S2, S2, Z1Z1); fp2_sub(r, S2, a.y); }
  { fp2 U2; const fp2 x2 = qp->x; fp2_mul(U2, x2, Z1Z1); fp2_sub(H, U2, a.x); }
  if (fp2_is_zero(H)) {
    if (fp2_is_zero(r)) jac_dbl(a, a); else jac_set_inf(a);
    return;
  }
  fp2_dbl(r, r);
  fp2 I;
  {
    fp2 HH, t;
    fp2_sqr(HH, H);
    fp2_add(t, a.z, H); fp2_sqr(t, t); fp2_sub(t, t, Z1Z1); fp2_sub(a.z, t, HH);
    fp2_dbl(I, HH); fp2_dbl(I, I);
  }
  fp2 V; fp2_mul(V, a.x, I);
  fp2 J; fp2_mul(J, H, I);
  fp2 t; fp2_mul(t, a.y, J);
  fp2_sqr(a.x, r); fp2_sub(a.x, a.x, J); fp2_dbl(J, V); fp2_sub(a.x, a.x, J);
  fp2_sub(V, V, a.x); fp2_mul(a.y, r, V); fp2_dbl(t, t); fp2_sub(a.y, a.y, t);
}
// The chains' group steps, each its own callable function (round 5).  A callable function whose
// body outgrows the +-128 KB reach of a short branch gets long branches (s_getpc / s_add / s_setpc
// through a scratch SGPR pair), and this compiler has been seen to take s[30:31] -- the return
// address -- for them without saving it: the function then "returns" into its own loop and the
// wave never finishes (rc_k_chain with inlined steps, 608 KB; build.py long_branch_clobbers fails
// the build on it).  Small out-of-line steps keep every chain loop far inside that reach, and the
// chains re-run one copy of each step's code instead of streaming megabytes of inlined copies
// through the instruction cache.
SSB_FN void rc_madd(g2_jac& a, const g2_xy* __restrict__ qp, bool neg) { jac_madd_xy(a, qp, neg); }
SSB_FN void rc_add(g2_jac& a, const g2_jac* __restrict__ qp, bool neg) { jac_add_at(a, qp, neg); }
SSB_FN void rc_dbl4(g2_jac& a) {
#pragma unroll 1
  for (int q = 0; q < 4; ++q) jac_dbl(a, a);
}
// the odd multiples (2e + 1) P, e < 8, of an affine P (not infinity): X, Y into xy[e], Z into zs[e]
// (Jacobian until rc_normalize; entry 0 is P itself, Z = 1); 2P parked at *p2
SSB_INL void rc_odd_multiples(g2_xy* __restrict__ xy, fp2* __restrict__ zs, g2_jac* __restrict__ p2, const g2_aff& P) {
  xy[0].x = P.x; xy[0].y = P.y; zs[0] = fp2_one();
  g2_jac e;
  jac_from_aff(e, P);
  jac_dbl(*p2, e);
  jac_add_aff(e, *p2, P);                   // 3P
#pragma unroll 1
  for (int i = 1; i < 8; ++i) {
    if (i > 1) rc_add(e, p2, false);
    xy[i].x = e.x; xy[i].y = e.y; zs[i] = e.z;
  }
}
// entries [0, K) to affine with ONE inversion (Montgomery's trick over their Z)
SSB_INL void rc_normalize(g2_xy* __restrict__ xy, const fp2* __restrict__ zs, fp2* __restrict__ pr, int K) {
  {
    fp2 p = zs[0];
    pr[0] = p;
#pragma unroll 1
    for (int k = 1; k < K; ++k) { const fp2 z = zs[k]; fp2_mul(p, p, z); pr[k] = p; }
  }
  fp2 inv; { const fp2 p = pr[K - 1]; fp2_inv(inv, p); }
#pragma unroll 1
  for (int k = K - 1; k >= 0; --k) {
    fp2 zi;
    if (k > 0) { const fp2 p = pr[k - 1]; fp2_mul(zi, inv, p); const fp2 z = zs[k]; fp2_mul(inv, inv, z); } else zi = inv;
    fp2 z2, z3;
    fp2_sqr(z2, zi); fp2_mul(z3, z2, zi);
    { fp2 x = xy[k].x; fp2_mul(x, x, z2); xy[k].x = x; }
    { fp2 y = xy[k].y; fp2_mul(y, y, z3); xy[k].y = y; }
  }
}

// sum_i [c_i] P_i, P_i = pts[idx[i]] (verified G2 points), |c_i| < 2^62, c_i != 0; W = a window count
// with every (|c_i| rounded up to odd) < 2^(4W) -- wave-uniform on the device (the caller takes the
// wave's maximum), so every lane runs the same doublings
// (T in memory: with more than RC_GROUP bases the groups' sums meet there, not in registers that
// would stay live across the joint loop)
SSB_INL void rc_joint_sum(g2_jac* __restrict__ T, const g2_aff* __restrict__ pts, const uint32_t* __restrict__ idx,
                          const int64_t* c, uint32_t t, int W, uint8_t* __restrict__ region) {
  g2_xy* xy = (g2_xy*)(region + RC_XY_OFF);
  fp2* zs = (fp2*)(region + RC_Z_OFF);
  fp2* pr = (fp2*)(region + RC_PR_OFF);
#pragma unroll 1
  for (uint32_t g0 = 0; g0 < t; g0 += RC_GROUP) {
    const uint32_t nb = t - g0 < (uint32_t)RC_GROUP ? t - g0 : (uint32_t)RC_GROUP;
#pragma unroll 1
    for (uint32_t b = 0; b < nb; ++b) rc_odd_multiples(xy + 8 * b, zs + 8 * b, (g2_jac*)pr, pts[idx[g0 + b]]);
    rc_normalize(xy, zs, pr, 8 * (int)nb);
    g2_jac acc;
    jac_set_inf(acc);
#pragma unroll 1
    for (int j = W - 1; j >= 0; --j) {
      if (j != W - 1) rc_dbl4(acc);
#pragma unroll 1
      for (uint32_t b = 0; b < nb; ++b) {
        const int64_t cb = c[g0 + b];
        const uint64_t m = (uint64_t)(cb < 0 ? -cb : cb) | 1ull;   // even |c|: [|c| + 1] P, and P subtracted below
        const int d = sw4_digit(m, j, W);
        const int ad = d < 0 ? -d : d;
        rc_madd(acc, xy + 8 * b + ((ad - 1) >> 1), (d < 0) != (cb < 0));
      }
    }
#pragma unroll 1
    for (uint32_t b = 0; b < nb; ++b) {     // the even coefficients' correction: - sign(c) P
      const int64_t cb = c[g0 + b];
      if (!(((uint64_t)(cb < 0 ? -cb : cb)) & 1ull)) rc_madd(acc, xy + 8 * b, cb > 0);
    }
    if (g0) rc_add(acc, T, false);
    *T = acc;
  }
}

// [k] T for k = M^-1 mod r (1 <= M < 2^62, inv_small_mod_r), T in G2 (not infinity): four base-u
// digits, one table of T's odd multiples (affine) and its signed psi images (digit q's base is
// (-1)^q psi^q(T), as in unit_gls_term), 16 windows of every digit jointly.  Two steps, out of line,
// each with its own private frame (one function held both frames' spills at once: 2.3 KB):
//   rc_k_table: the table (the digits come from rc_digits, run in phase T);
//   rc_k_chain: the joint chain from the region.
// the four base-u digits of M^-1 mod r (1 <= M < 2^62)
SSB_FN void rc_digits(uint64_t* __restrict__ kk, uint64_t M) {
  uint64_t y[4], d[4];
  inv_small_mod_r(y, M);
  gls_digits4(d, y);
  for (int q = 0; q < 4; ++q) kk[q] = d[q];
}
SSB_FN void rc_k_table(const g2_jac* __restrict__ T, uint8_t* __restrict__ region) {
  g2_xy* xy = (g2_xy*)(region + RC_XY_OFF);
  fp2* zs = (fp2*)(region + RC_Z_OFF);
  fp2* pr = (fp2*)(region + RC_PR_OFF);
  {
    g2_aff Ta;
    { const g2_jac Tv = *T; jac_to_aff(Ta, Tv); }
    rc_odd_multiples(xy, zs, (g2_jac*)pr, Ta);
  }
  rc_normalize(xy, zs, pr, 8);
  // psi images: xy[8 q + i] = (-1)^q psi^q((2i + 1) T)
#pragma unroll 1
  for (int i = 0; i < 8; ++i) {
    g2_aff p; p.x = xy[i].x; p.y = xy[i].y; p.inf = 0;
#pragma unroll 1
    for (int q = 1; q < 4; ++q) {
      g2_psi_aff(p, p);
      g2_xy o; o.x = p.x; o.y = p.y;
      if (q & 1) fp2_neg(o.y, o.y);
      xy[8 * q + i] = o;
    }
  }
}
SSB_FN void rc_k_chain(g2_jac& R, const uint8_t* __restrict__ region, const uint64_t* __restrict__ kd) {
  const g2_xy* xy = (const g2_xy*)(region + RC_XY_OFF);
  uint64_t kk[4];
  for (int q = 0; q < 4; ++q) kk[q] = kd[q];
  g2_jac acc;
  jac_set_inf(acc);
#pragma unroll 1
  for (int j = 15; j >= 0; --j) {
    if (j != 15) rc_dbl4(acc);
#pragma unroll 1
    for (int q = 0; q < 4; ++q) {
      const int d = sw4_digit(kk[q] | 1ull, j, 16);   // an even digit: d + 1, and the base subtracted below
      const int ad = d < 0 ? -d : d;
      rc_madd(acc, xy + 8 * q + ((ad - 1) >> 1), d < 0);
    }
  }
#pragma unroll 1
  for (int q = 0; q < 4; ++q)
    if (!(kk[q] & 1ull)) rc_madd(acc, xy + 8 * q, true);
  R = acc;
}

// The ratio combine in two phases, one per launch (k_combine_terms_gls' extra blocks run phase T,
// k_combine_sum's lanes of fast-2 jobs phase K), every step out of line so that no kernel holds two
// steps' private frames at once.  Phase T: T = sum c_i sig_i into *T and the digits of M^-1 into kk.
// Phase K: [M^-1] T, compressed into out96 (infinity when T is).
SSB_FN void unit_ratio_T(g2_jac* __restrict__ T, uint64_t* __restrict__ kk, const g2_aff* __restrict__ pts,
                         const uint32_t* __restrict__ idx, const int64_t* c, uint32_t t, uint64_t M, int W,
                         uint8_t* __restrict__ region) {
  rc_joint_sum(T, pts, idx, c, t, W, region);
  rc_digits(kk, M);
}
SSB_FN void rc_k_finish(uint8_t* out96, const uint8_t* __restrict__ region, const uint64_t* __restrict__ kk) {
  g2_jac R;
  rc_k_chain(R, region, kk);
  g2_aff a; jac_to_aff(a, R);
  g2_compress(out96, a);
}
SSB_INL void unit_ratio_K(uint8_t* out96, const g2_jac* __restrict__ T, const uint64_t* __restrict__ kk,
                          uint8_t* __restrict__ region) {
  if (fp2_is_zero(T->z)) {   // T = O (e.g. a zero master key): the combination is infinity
    out96[0] = 0xc0;
    for (int i = 1; i < 96; ++i) out96[i] = 0;
    return;
  }
  rc_k_table(T, region);
  rc_k_finish(out96, region, kk);
}
// the whole ratio combine of one job into out96 (host tests; the device runs the two phases)
SSB_INL void unit_combine_ratio_w4(uint8_t* out96, const g2_aff* __restrict__ pts, const uint32_t* __restrict__ idx,
                                   const int64_t* c, uint32_t t, uint64_t M, int W, uint8_t* __restrict__ region) {
  g2_jac T;
  uint64_t kk[4];
  unit_ratio_T(&T, kk, pts, idx, c, t, M, W, region);
  unit_ratio_K(out96, &T, kk, region);
}
// the window count T's coefficients need (before the wave-wide maximum)
SSB_INL int rc_windows(const int64_t* c, uint32_t t) {
  int W = 1;
  for (uint32_t i = 0; i < t; ++i) {
    const int w = sw4_windows((uint64_t)(c[i] < 0 ? -c[i] : c[i]) | 1ull);
    W = w > W ? w : W;
  }
  return W;
}

}  // namespace ssb
