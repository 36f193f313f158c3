// ssb_h2c.h -- hash_to_G2 for the suite BLS12381G2_XMD:SHA-256_SSWU_RO_ (RFC 9380), the hash
// blst computes inside Signature::verify and SecretKey::sign with the PoP DST
// (src/crypto/impls/blst.rs:11).  The engine runs it once per distinct signing root instead of
// once per partial signature.
#pragma once
#include "ssb_curve.h"

namespace ssb {

// ------------------------------------------------------------------------------------------
// SHA-256
// ------------------------------------------------------------------------------------------
constexpr uint32_t SHA256_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

SSB_INL uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

SSB_FN void sha256_compress(uint32_t* st, const uint8_t* blk) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i)
    w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) | ((uint32_t)blk[4 * i + 2] << 8) | blk[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + SHA256_K[i] + w[i];
    uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// One-shot SHA-256 of a message held in a small buffer (len <= 416 bytes).
SSB_FN void sha256(uint8_t* out, const uint8_t* msg, int len) {
  uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au, 0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  uint8_t blk[64];
  int off = 0;
  while (len - off >= 64) { sha256_compress(st, msg + off); off += 64; }
  int rem = len - off;
  for (int i = 0; i < 64; ++i) blk[i] = 0;
  for (int i = 0; i < rem; ++i) blk[i] = msg[off + i];
  blk[rem] = 0x80;
  if (rem >= 56) { sha256_compress(st, blk); for (int i = 0; i < 64; ++i) blk[i] = 0; }
  const uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; ++i) blk[63 - i] = (uint8_t)(bits >> (8 * i));
  sha256_compress(st, blk);
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)(st[i] >> 24); out[4 * i + 1] = (uint8_t)(st[i] >> 16);
    out[4 * i + 2] = (uint8_t)(st[i] >> 8); out[4 * i + 3] = (uint8_t)st[i];
  }
}

// expand_message_xmd(msg, DST, 256) -> 256 bytes   (RFC 9380 §5.3.1); msg_len <= 32 (a signing
// root is 32 bytes; shorter messages are for the RFC's own test vectors)
SSB_FN void expand_message_xmd_256(uint8_t* out, const uint8_t* msg32, const uint8_t* dst, int dst_len, int msg_len = 32) {
  uint8_t buf[64 + 32 + 3 + 256 + 1];
  int n = 0;
  for (int i = 0; i < 64; ++i) buf[n++] = 0;         // Z_pad
  for (int i = 0; i < msg_len; ++i) buf[n++] = msg32[i];  // msg
  buf[n++] = 1; buf[n++] = 0;                         // I2OSP(256, 2)
  buf[n++] = 0;                                       // I2OSP(0, 1)
  for (int i = 0; i < dst_len; ++i) buf[n++] = dst[i];
  buf[n++] = (uint8_t)dst_len;
  uint8_t b0[32];
  sha256(b0, buf, n);
  uint8_t prev[32];
  for (int i = 1; i <= 8; ++i) {
    int m = 0;
    for (int j = 0; j < 32; ++j) buf[m++] = (i == 1) ? b0[j] : (uint8_t)(b0[j] ^ prev[j]);
    buf[m++] = (uint8_t)i;
    for (int j = 0; j < dst_len; ++j) buf[m++] = dst[j];
    buf[m++] = (uint8_t)dst_len;
    sha256(prev, buf, m);
    for (int j = 0; j < 32; ++j) out[32 * (i - 1) + j] = prev[j];
  }
}

// OS2IP(64 bytes) mod p, in Montgomery form: hi(128 bit) * 2^384 + lo(384 bit)
SSB_FN void fp_from_be64_mod(fp& r, const uint8_t* b) {
  fp lo, hi;
  fp_from_be48(lo, b + 16, 0xff);  // value check result ignored: any 384-bit value is fine
  for (int i = 0; i < 12; ++i) hi.l[i] = 0;
  for (int i = 0; i < 4; ++i) {
    const uint8_t* q = b + 12 - 4 * i;
    hi.l[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
  fp a, c;
  mp_mont_mul<12>(a.l, lo.l, P_R2, P_LIMBS, P_INV32);  // lo * R
  mp_mont_mul<12>(c.l, hi.l, P_R3, P_LIMBS, P_INV32);  // hi * 2^384 * R
  fp_add(r, a, c);
}

// ------------------------------------------------------------------------------------------
// Simplified SWU onto E2': y^2 = x^3 + A'x + B', then the 3-isogeny to E2
// ------------------------------------------------------------------------------------------
SSB_FN void sswu_g(fp2& g, const fp2& x) {
  fp2 A = fp2_from_c(SSWU_A), B = fp2_from_c(SSWU_B), t;
  fp2_sqr(g, x);
  fp2_add(g, g, A);
  fp2_mul(g, g, x);
  fp2_add(g, g, B);
  (void)t;
}

SSB_FN void map_to_curve_sswu(fp2& xo, fp2& yo, const fp2& u) {
  fp2 Z = fp2_from_c(SSWU_Z);
  fp2 zu2, den, x1, t, y, g;
  fp2_sqr(zu2, u);
  fp2_mul(zu2, zu2, Z);
  fp2_sqr(den, zu2);
  fp2_add(den, den, zu2);
  if (fp2_is_zero(den)) {
    x1 = fp2_from_c(SSWU_B_OVER_ZA);
  } else {
    fp2_inv(t, den);
    fp2 one = fp2_one();
    fp2_add(t, t, one);
    fp2 nboa = fp2_from_c(SSWU_MINUS_B_OVER_A);
    fp2_mul(x1, nboa, t);
  }
  sswu_g(g, x1);
  fp2 x = x1;
  if (!fp2_sqrt(y, g)) {
    fp2_mul(x, zu2, x1);
    sswu_g(g, x);
    (void)fp2_sqrt(y, g);  // g(x2) = Z^3 u^6 g(x1) is a square when g(x1) is not
  }
  if (fp2_sgn0(u) != fp2_sgn0(y)) fp2_neg(y, y);
  xo = x; yo = y;
}

SSB_FN void iso3_poly(fp2& r, const fp2_c* k, int n, const fp2& x) {
  fp2 acc = fp2_from_c(k[n - 1]);
  for (int i = n - 2; i >= 0; --i) {
    fp2 c = fp2_from_c(k[i]);
    fp2_mul(acc, acc, x);
    fp2_add(acc, acc, c);
  }
  r = acc;
}

SSB_FN void iso3_map(g2_aff& r, const fp2& xp, const fp2& yp) {
  fp2 xn, xd, yn, yd, t;
  iso3_poly(xn, ISO_XNUM, 4, xp);
  iso3_poly(xd, ISO_XDEN, 3, xp);
  iso3_poly(yn, ISO_YNUM, 4, xp);
  iso3_poly(yd, ISO_YDEN, 4, xp);
  fp2_mul(t, xd, yd);
  if (fp2_is_zero(t)) { r.x = fp2_zero(); r.y = fp2_zero(); r.inf = 1; return; }
  fp2 ti; fp2_inv(ti, t);                 // one inversion for both denominators
  fp2 xdi, ydi;
  fp2_mul(xdi, ti, yd);
  fp2_mul(ydi, ti, xd);
  fp2_mul(r.x, xn, xdi);
  fp2_mul(t, yn, ydi);
  fp2_mul(r.y, yp, t);
  r.inf = 0;
}

// h_eff * P = [x^2-x-1]P + [x-1]psi(P) + psi^2(2P)   (RFC 9380 Appendix G.3)
SSB_FN void clear_cofactor_g2(g2_jac& r, const g2_jac& P) {
  g2_jac t1, t2, t3, n;
  jac_mul_x_abs(t1, P); jac_neg(t1, t1);  // [x]P
  g2_psi_jac(t2, P);                        // psi(P)
  jac_dbl(t3, P);                           // 2P
  g2_psi_jac(t3, t3);
  g2_psi_jac(t3, t3);                       // psi^2(2P)
  jac_neg(n, t2);
  jac_add(t3, t3, n);                       // psi^2(2P) - psi(P)
  jac_add(t2, t1, t2);                      // [x]P + psi(P)
  jac_mul_x_abs(t2, t2); jac_neg(t2, t2);   // [x^2]P + [x]psi(P)
  jac_add(t3, t3, t2);
  jac_neg(n, t1);
  jac_add(t3, t3, n);
  jac_neg(n, P);
  jac_add(r, t3, n);
}

// h_eff * (q0 + q1), the same element as clear_cofactor_g2(q0 + q1), with at most three Jacobian
// points live: h_eff P = [x]u - u + psi^2(2P) - P where u = [x]P + psi(P); u and [x]u - u go
// through *tmp (memory), P is recomputed from q0, q1.  The hash pipeline's exact redo of a root
// whose lane-group stage met an exceptional addition; its private segment is what the batch
// streams reserve per queue, so it is kept below the per-share kernels'.
#define SSB_MEM_FENCE() __asm__ volatile("" ::: "memory")
SSB_FN void h2c_clear_exact(g2_jac& r, const g2_aff& q0, const g2_aff& q1, g2_jac* tmp) {
  g2_jac p, a;
  jac_from_aff(p, q0); jac_add_aff(p, p, q1);          // P
  jac_mul_x_abs(a, p); jac_neg(a, a);                  // [x]P
  g2_psi_jac(p, p);
  jac_add(a, a, p);                                    // u = [x]P + psi(P)
  *tmp = a;
  SSB_MEM_FENCE();
  jac_mul_x_abs(p, a); jac_neg(p, p);                  // [x]u
  a = *tmp; jac_neg(a, a);
  jac_add(p, p, a);                                    // [x]u - u
  *tmp = p;
  SSB_MEM_FENCE();
  jac_from_aff(p, q0); jac_add_aff(p, p, q1);          // P again
  jac_dbl(a, p); g2_psi_jac(a, a); g2_psi_jac(a, a);   // psi^2(2P)
  jac_neg(p, p);
  jac_add(a, a, p);                                    // psi^2(2P) - P
  p = *tmp;
  jac_add(r, p, a);
}

// ---- the same hash split into the stages of the batched pipeline (ssb_k_hash.hip) ----
// stage 1: u0, u1 from expand_message_xmd
SSB_FN void h2c_field(fp2& u0, fp2& u1, const uint8_t* msg32, const uint8_t* dst, int dst_len, int msg_len = 32) {
  uint8_t uni[256];
  expand_message_xmd_256(uni, msg32, dst, dst_len, msg_len);
  fp_from_be64_mod(u0.c0, uni);
  fp_from_be64_mod(u0.c1, uni + 64);
  fp_from_be64_mod(u1.c0, uni + 128);
  fp_from_be64_mod(u1.c1, uni + 192);
}
// stage 2 (one lane per candidate): x1 (cand 0) or x2 = Z u^2 x1 (cand 1), and a square root of
// g(x); returns whether g(x) is a square.  map_to_curve_sswu takes x1 when g(x1) is a square,
// else x2 (then g(x2) is), exactly as the sequential code above.
SSB_FN bool sswu_candidate(fp2& x, fp2& y, const fp2& u, int cand) {
  fp2 Z = fp2_from_c(SSWU_Z);
  fp2 zu2, den, x1, t, g;
  fp2_sqr(zu2, u);
  fp2_mul(zu2, zu2, Z);
  fp2_sqr(den, zu2);
  fp2_add(den, den, zu2);
  if (fp2_is_zero(den)) {
    x1 = fp2_from_c(SSWU_B_OVER_ZA);
  } else {
    fp2_inv(t, den);
    fp2 one = fp2_one();
    fp2_add(t, t, one);
    fp2 nboa = fp2_from_c(SSWU_MINUS_B_OVER_A);
    fp2_mul(x1, nboa, t);
  }
  if (cand) fp2_mul(x, zu2, x1); else x = x1;
  sswu_g(g, x);
  return fp2_sqrt(y, g);
}
// stage 2 tail: sign of y, then the 3-isogeny
SSB_FN void sswu_finish(g2_aff& q, const fp2& u, const fp2& x, const fp2& y_in) {
  fp2 y = y_in;
  if (fp2_sgn0(u) != fp2_sgn0(y)) fp2_neg(y, y);
  iso3_map(q, x, y);
}

SSB_FN void hash_to_g2(g2_aff& out, const uint8_t* msg32, const uint8_t* dst, int dst_len, int msg_len = 32) {
  uint8_t uni[256];
  expand_message_xmd_256(uni, msg32, dst, dst_len, msg_len);
  fp2 u0, u1;
  fp_from_be64_mod(u0.c0, uni);
  fp_from_be64_mod(u0.c1, uni + 64);
  fp_from_be64_mod(u1.c0, uni + 128);
  fp_from_be64_mod(u1.c1, uni + 192);
  fp2 x, y;
  g2_aff q0, q1;
  map_to_curve_sswu(x, y, u0);
  iso3_map(q0, x, y);
  map_to_curve_sswu(x, y, u1);
  iso3_map(q1, x, y);
  g2_jac s;
  jac_from_aff(s, q0);
  jac_add_aff(s, s, q1);
  clear_cofactor_g2(s, s);
  jac_to_aff(out, s);
}

}  // namespace ssb
