// Host build of the device math headers, for CPU unit tests against the oracle and for the
// algorithmic op counter.  TEST INFRASTRUCTURE: not part of libssbls.so.
// Protocol: one command per stdin line, one result line per command on stdout.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <iostream>
#include <sstream>
#include "../../safestakeoperator_amd/csrc/ssb_units.h"
#include "../../safestakeoperator_amd/csrc/ssb_lane_ops.h"
#include "../../safestakeoperator_amd/csrc/ssb_f28.h"

#ifdef SSB_OPCOUNT
ssb_opcounts g_ssb_counts;
#endif
using namespace ssb;

static std::vector<uint8_t> unhex(const std::string& s) {
  std::vector<uint8_t> v(s.size() / 2);
  for (size_t i = 0; i < v.size(); ++i) v[i] = (uint8_t)std::stoi(s.substr(2 * i, 2), nullptr, 16);
  return v;
}
static std::string hex(const uint8_t* b, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; ++i) { s += d[b[i] >> 4]; s += d[b[i] & 15]; }
  return s;
}
static const char* DST = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";

// fixed pseudo-random 64-bit values for the op counter and the lane tests (splitmix64); only
// their bit patterns matter there, and keeping them fixed keeps bench_tools/opcount.json stable
static uint64_t rlc_scalar(uint64_t seed, uint64_t i) {
  uint64_t z = seed ^ (0x9E3779B97F4A7C15ull * (i + 1));
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z ? z : 1ull;
}

static bool verify_full(const g1_aff& pk, const g2_aff& sig, const g2_aff& h) {
  if (pk.inf) return false;
  if (!g2_in_subgroup(sig)) return false;
  fp12 f1, f2;
  miller_loop(f1, pk, h);
  g1_aff ng; ng.x = fp_from_c(G1_GEN_X); ng.y = fp_from_c(G1_GEN_NEG_Y); ng.inf = 0;
  miller_loop(f2, ng, sig);
  fp12_mul(f1, f1, f2);
  fp12 e; final_exponentiation(e, f1);
  return fp12_is_one(e);
}


// ---- lane-group programs (host emulation, role loop) against the single-lane code ----
struct host_group {
  std::vector<lane::lslot> K, S;
  uint32_t flag = 0;
  lane::grp g;
  host_group() : K(lane::LP_NCODE_CONST), S(lane::LP_NSCRATCH + 256) {
    g = lane::grp{K.data(), S.data(), 0, 0, 0, &flag, 0};
    lane::lp_init_consts(g);
  }
  lane::lslot* u(int i) { return &S[lane::LP_NSCRATCH + i]; }
  void put(int i, const fp& v) { lane::lp_put(u(i), lane::lv_in(v)); }
  fp get(int i) { return lane::lv_out(lane::lp_get(u(i))); }
  int U(int i) const { return lane::LP_NSCRATCH + i; }
};
template <class F> static void put_jac(host_group& h, int at, const jac<F>& p) {
  const fp* q = (const fp*)&p; for (int i = 0; i < (int)(3 * sizeof(F) / sizeof(fp)); ++i) h.put(at + i, q[i]);
}
template <class F> static bool eq_jac(host_group& h, int at, const jac<F>& p) {
  const fp* q = (const fp*)&p; bool ok = true;
  for (int i = 0; i < (int)(3 * sizeof(F) / sizeof(fp)); ++i) ok = ok && fp_eq(h.get(at + i), q[i]);
  return ok;
}
template <class F> static void put_aff(host_group& h, int at, const aff<F>& p) {
  const fp* q = (const fp*)&p; for (int i = 0; i < (int)(2 * sizeof(F) / sizeof(fp)); ++i) h.put(at + i, q[i]);
}
template <class F> static bool same_point(host_group& h, int at, const jac<F>& p) {
  jac<F> r; fp* q = (fp*)&r; for (int i = 0; i < (int)(3 * sizeof(F) / sizeof(fp)); ++i) q[i] = h.get(at + i);
  aff<F> a, b; jac_to_aff(a, r); jac_to_aff(b, p);
  return a.inf == b.inf && (a.inf || (f_eq(a.x, b.x) && f_eq(a.y, b.y)));
}

static void lane_selftest(const uint8_t* seed32) {
  int ok = 0, n = 0;
  host_group h;
  lane::grp& g = h.g;
  g2_aff P, Q, Hraw;
  uint8_t m[32];
  for (int k = 0; k < 32; ++k) m[k] = seed32[k];
  hash_to_g2(P, m, (const uint8_t*)DST, (int)strlen(DST));
  m[0] ^= 1; hash_to_g2(Q, m, (const uint8_t*)DST, (int)strlen(DST));
  { // a point on E2 that is NOT in G2: the isogeny image before cofactor clearing
    uint8_t uni[256]; m[1] ^= 7; expand_message_xmd_256(uni, m, (const uint8_t*)DST, (int)strlen(DST));
    fp2 u; fp_from_be64_mod(u.c0, uni); fp_from_be64_mod(u.c1, uni + 64);
    fp2 x, y; map_to_curve_sswu(x, y, u); iso3_map(Hraw, x, y); }
  g2_jac J1, J2, t;
  jac_from_aff(J1, P); jac_dbl(J1, J1); jac_add_aff(J1, J1, Q);        // 2P + Q, Z != 1
  jac_from_aff(J2, Q); jac_dbl(J2, J2); jac_add_aff(J2, J2, Q);        // 3Q
  uint32_t exc = 0;
  // G2 dbl / add / madd: bit-identical Jacobian coordinates
  put_jac(h, 0, J1); lane::g2_dbl(g, h.U(0), h.U(6)); jac_dbl(t, J1); ok += eq_jac(h, 6, t); ++n;
  put_jac(h, 0, J1); put_jac(h, 6, J2); lane::g2_add(g, h.U(0), h.U(6), h.U(12), exc); jac_add(t, J1, J2); ok += eq_jac(h, 12, t); ++n;
  ok += exc == 0; ++n;
  put_jac(h, 0, J1); put_aff(h, 6, Q); lane::g2_madd(g, h.U(0), h.U(6), h.U(12), exc); jac_add_aff(t, J1, Q); ok += eq_jac(h, 12, t); ++n;
  ok += exc == 0; ++n;
  // in-place (d == a)
  put_jac(h, 0, J1); put_jac(h, 6, J2); lane::g2_add(g, h.U(0), h.U(6), h.U(0), exc); jac_add(t, J1, J2); ok += eq_jac(h, 0, t); ++n;
  // exceptional: J1 + J1 and J1 + (-J1) raise exc
  { uint32_t e2 = 0; put_jac(h, 0, J1); put_jac(h, 6, J1); lane::g2_add(g, h.U(0), h.U(6), h.U(12), e2); ok += e2 == 1; ++n; }
  { uint32_t e2 = 0; g2_jac nj; jac_neg(nj, J1); put_jac(h, 0, J1); put_jac(h, 6, nj); lane::g2_add(g, h.U(0), h.U(6), h.U(12), e2); ok += e2 == 1; ++n; }
  { uint32_t e2 = 0; g2_jac inf; jac_set_inf(inf); put_jac(h, 0, inf); put_jac(h, 6, J1); lane::g2_add(g, h.U(0), h.U(6), h.U(12), e2); ok += e2 == 1; ++n; }
  // 64-bit windowed multiplication (odd scalars)
  for (int r = 0; r < 4; ++r) {
    uint64_t k = rlc_scalar(0x1234 + r, (uint64_t)r) | 1ull;
    if (r == 3) k = 1ull;
    uint32_t e = 0;
    put_aff(h, 0, P);
    lane::g2_mul_u64_odd(g, h.U(0), k, h.U(4), h.U(52), h.U(58), e);
    const uint32_t kw[2] = {(uint32_t)k, (uint32_t)(k >> 32)};
    jac_mul_aff(t, P, kw, 2);
    ok += same_point(h, 52, t) && e == 0; ++n;
  }
  // G1: generator multiples
  { g1_aff G1; G1.x = fp_from_c(G1_GEN_X); G1.y = fp_from_c(G1_GEN_Y); G1.inf = 0;
    g1_jac A1, A2, t1; jac_from_aff(A1, G1); jac_dbl(A1, A1); jac_add_aff(A1, A1, G1); jac_from_aff(A2, G1); jac_dbl(A2, A2);
    put_jac(h, 0, A1); lane::g1_dbl(g, h.U(0), h.U(3)); jac_dbl(t1, A1); ok += eq_jac(h, 3, t1); ++n;
    put_jac(h, 0, A1); put_jac(h, 3, A2); lane::g1_add(g, h.U(0), h.U(3), h.U(6), exc); jac_add(t1, A1, A2); ok += eq_jac(h, 6, t1); ++n;
    put_jac(h, 0, A1); put_aff(h, 3, G1); lane::g1_madd(g, h.U(0), h.U(3), h.U(6), exc); jac_add_aff(t1, A1, G1); ok += eq_jac(h, 6, t1); ++n;
    uint64_t k = rlc_scalar(99, 5) | 1ull; uint32_t e = 0;
    put_aff(h, 0, G1); lane::g1_mul_u64_odd(g, h.U(0), k, h.U(2), h.U(30), h.U(33), e);
    const uint32_t kw[2] = {(uint32_t)k, (uint32_t)(k >> 32)};
    jac_mul_aff(t1, G1, kw, 2); ok += same_point(h, 30, t1) && e == 0; ++n; }
  // subgroup check: a G2 point passes, the raw isogeny image fails
  { uint32_t e = 0; put_aff(h, 0, P); bool in = lane::g2_subgroup_check(g, h.U(0), h.U(4), h.U(10), e);
    ok += in && e == 0 && g2_in_subgroup(P); ++n; }
  { uint32_t e = 0; put_aff(h, 0, Hraw); bool in = lane::g2_subgroup_check(g, h.U(0), h.U(4), h.U(10), e);
    ok += !in && (e == 0) && !g2_in_subgroup(Hraw); ++n; }
  // cofactor clearing of q0 + q1 (the hash pipeline's lane-group stage) vs clear_cofactor_g2
  { uint32_t e = 0; g2_jac S; jac_from_aff(S, Hraw); jac_add_aff(S, S, Q);
    put_jac(h, 0, S); lane::g2_clear_cofactor(g, h.U(0), h.U(6), h.U(12), e);
    g2_jac R; clear_cofactor_g2(R, S); ok += same_point(h, 6, R) && e == 0; ++n;
    // the exact redo (three live points, temporaries through memory) == clear_cofactor_g2
    { auto same = [](const g2_jac& a, const g2_jac& b) { g2_aff x, y; jac_to_aff(x, a); jac_to_aff(y, b);
        uint8_t ca[96], cb[96]; g2_compress(ca, x); g2_compress(cb, y); return memcmp(ca, cb, 96) == 0; };
      g2_jac tmp, X; h2c_clear_exact(X, Hraw, Q, &tmp); ok += same(X, R); ++n;
      g2_aff Qn = Q; fp2_neg(Qn.y, Q.y); h2c_clear_exact(X, Q, Qn, &tmp); ok += jac_is_inf(X) != 0; ++n;  // q0 = -q1
      g2_jac D; jac_from_aff(D, Q); jac_dbl(D, D); clear_cofactor_g2(D, D); h2c_clear_exact(X, Q, Q, &tmp); ok += same(X, D); ++n; }  // q0 = q1
    // staged hash == hash_to_g2
    fp2 u0, u1; h2c_field(u0, u1, m, (const uint8_t*)DST, (int)strlen(DST));
    g2_aff q[2]; const fp2* us[2] = {&u0, &u1};
    for (int j = 0; j < 2; ++j) {
      fp2 x0, y0, x1, y1; bool ok0 = sswu_candidate(x0, y0, *us[j], 0); bool ok1 = sswu_candidate(x1, y1, *us[j], 1);
      sswu_finish(q[j], *us[j], ok0 ? x0 : x1, ok0 ? y0 : y1); (void)ok1; }
    g2_jac T; jac_from_aff(T, q[0]); jac_add_aff(T, T, q[1]);
    put_jac(h, 0, T); lane::g2_clear_cofactor(g, h.U(0), h.U(6), h.U(12), e);
    g2_aff want; hash_to_g2(want, m, (const uint8_t*)DST, (int)strlen(DST));
    g2_jac wj; jac_from_aff(wj, want); ok += same_point(h, 6, wj) && e == 0; ++n; }
  ok += exc == 0; ++n;
  // Fp12 programs, the lane final exponentiation and Miller loop
  { g1_aff pk; pk.x = fp_from_c(G1_GEN_X); pk.y = fp_from_c(G1_GEN_Y); pk.inf = 0;
    fp12 f1, f2, r1, r2; miller_loop(f1, pk, P); g1_aff ng = g1_neg_generator(); miller_loop(f2, ng, Q);
    lane::st12(g.s + h.U(0), f1); lane::st12(g.s + h.U(12), f2);
    lane::f12_mul(g, h.U(0), h.U(12), h.U(24)); fp12_mul(r1, f1, f2); lane::ld12(r2, g.s + h.U(24)); ok += fp12_eq(r1, r2); ++n;
    g.a = h.U(0); g.d = h.U(24); lane::lp_fp12_sqr(g); fp12_sqr(r1, f1); lane::ld12(r2, g.s + h.U(24)); ok += fp12_eq(r1, r2); ++n;
    for (int k = 1; k <= 3; ++k) { lane::f12_frob(g, k, h.U(0), h.U(24)); fp12_frob(r1, f1, k); lane::ld12(r2, g.s + h.U(24)); ok += fp12_eq(r1, r2); ++n; }
    { fp12 t0, t1, cy; fp12_conj(t0, f1); fp12_inv(t1, f1); fp12_mul(cy, t0, t1); fp12_frob(t0, cy, 2); fp12_mul(cy, t0, cy);
      lane::st12(g.s + h.U(0), cy); lane::f12_cyc_sqr(g, h.U(0), h.U(24)); fp12_cyc_sqr(r1, cy); lane::ld12(r2, g.s + h.U(24)); ok += fp12_eq(r1, r2); ++n; }
    { fp12 m; fp12_mul(m, f1, f2); final_exponentiation(r1, m);
      lane::st12(g.s + h.U(0), m); lane::f12_final_exp(g, h.U(0), h.U(12)); lane::ld12(r2, g.s + h.U(0)); ok += fp12_eq(r1, r2); ++n; }
    { // Miller loop of (pk, P)
      const int F = h.U(100), Bq = h.U(130);
      lane::lp_put(g.s + Bq, lane::lv_in(P.x.c0)); lane::lp_put(g.s + Bq + 1, lane::lv_in(P.x.c1)); lane::lp_put(g.s + Bq + 2, lane::lv_in(P.y.c0)); lane::lp_put(g.s + Bq + 3, lane::lv_in(P.y.c1)); lane::lp_put(g.s + Bq + 4, lane::lv_in(pk.x)); lane::lp_put(g.s + Bq + 5, lane::lv_in(pk.y));
      // (the lane loop runs homogeneous-projective steps, the single-lane one Jacobian: the Miller
      // values differ by an Fp2 factor per line, which the final exponentiation removes)
      lane::f12_miller(g, F, Bq); lane::ld12(r2, g.s + F);
      fp12 e1, e2; final_exponentiation(e1, f1); final_exponentiation(e2, r2); ok += fp12_eq(e1, e2); ++n;
      ok += !fp12_eq(f1, r2); ++n; }
    { // two-pair Miller loop of (pk, P) and (-g1, Q): == the product of the two single loops after
      // the final exponentiation
      const int F = h.U(100), Bq = h.U(130), Bp = h.U(142);
      lane::lp_put(g.s + Bq, lane::lv_in(P.x.c0)); lane::lp_put(g.s + Bq + 1, lane::lv_in(P.x.c1)); lane::lp_put(g.s + Bq + 2, lane::lv_in(P.y.c0)); lane::lp_put(g.s + Bq + 3, lane::lv_in(P.y.c1)); lane::lp_put(g.s + Bq + 4, lane::lv_in(pk.x)); lane::lp_put(g.s + Bq + 5, lane::lv_in(pk.y));
      lane::lp_put(g.s + Bq + 6, lane::lv_in(Q.x.c0)); lane::lp_put(g.s + Bq + 7, lane::lv_in(Q.x.c1)); lane::lp_put(g.s + Bq + 8, lane::lv_in(Q.y.c0)); lane::lp_put(g.s + Bq + 9, lane::lv_in(Q.y.c1)); lane::lp_put(g.s + Bq + 10, lane::lv_in(ng.x)); lane::lp_put(g.s + Bq + 11, lane::lv_in(ng.y));
      lane::f12_miller2(g, F, Bq, Bp); lane::ld12(r2, g.s + F);
      fp12 m, e1, e2; fp12_mul(m, f1, f2); final_exponentiation(e1, m); final_exponentiation(e2, r2); ok += fp12_eq(e1, e2); ++n;
      // and (pk, P) with (-pk, P): a check that holds, e(pk, P) e(-pk, P) == 1
      g1_aff npk = pk; fp_neg(npk.y, pk.y);
      lane::lp_put(g.s + Bq + 6, lane::lv_in(P.x.c0)); lane::lp_put(g.s + Bq + 7, lane::lv_in(P.x.c1)); lane::lp_put(g.s + Bq + 8, lane::lv_in(P.y.c0)); lane::lp_put(g.s + Bq + 9, lane::lv_in(P.y.c1)); lane::lp_put(g.s + Bq + 10, lane::lv_in(npk.x)); lane::lp_put(g.s + Bq + 11, lane::lv_in(npk.y));
      lane::f12_miller2(g, F, Bq, Bp); lane::f12_final_exp(g, F, h.U(12)); lane::ld12(r2, g.s + F); ok += fp12_is_one(r2); ++n; } }
  printf("%d %d\n", ok, n);
}

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    std::istringstream is(line);
    std::string cmd; is >> cmd;
    if (cmd == "h2g2") {  // h2g2 <msghex, <= 32 bytes; "-" = empty> [dsthex]
      std::string m, d; is >> m >> d;
      auto msg = m == "-" ? std::vector<uint8_t>() : unhex(m);
      const int mlen = (int)msg.size();
      msg.resize(32, 0);
      std::vector<uint8_t> dst = d.empty() ? std::vector<uint8_t>(DST, DST + strlen(DST)) : unhex(d);
      g2_aff h; hash_to_g2(h, msg.data(), dst.data(), (int)dst.size(), mlen);
      uint8_t out[192]; g2_serialize(out, h);
      printf("%s\n", hex(out, 192).c_str());
    } else if (cmd == "g2dec") {
      std::string s; is >> s; auto b = unhex(s);
      g2_aff p; uint32_t st = g2_decompress(p, b.data());
      uint32_t sub = (st & DEC_OK) && g2_in_subgroup(p) ? 1 : 0;
      uint8_t out[192]; g2_serialize(out, p); uint8_t cmp[96]; g2_compress(cmp, p);
      printf("%u %u %s %s\n", st, sub, hex(out, 192).c_str(), hex(cmp, 96).c_str());
    } else if (cmd == "g1dec") {
      std::string s; is >> s; auto b = unhex(s);
      g1_aff p; uint32_t st = g1_decompress(p, b.data());
      uint8_t cmp[48]; g1_compress(cmp, p);
      fp x, y; fp_from_mont(x, p.x); fp_from_mont(y, p.y);
      uint8_t xb[48], yb[48]; fp_to_be48(xb, x); fp_to_be48(yb, y);
      printf("%u %s %s %s\n", st, hex(cmp, 48).c_str(), hex(xb, 48).c_str(), hex(yb, 48).c_str());
    } else if (cmd == "verify") {  // verify pk48 sig96 msg32
      std::string a, b, c; is >> a >> b >> c;
      auto pkb = unhex(a), sb = unhex(b), mb = unhex(c);
      g1_aff pk; g2_aff sig, h;
      bool ok = (g1_decompress(pk, pkb.data()) & DEC_OK) && (g2_decompress(sig, sb.data()) & DEC_OK);
      if (ok) { hash_to_g2(h, mb.data(), (const uint8_t*)DST, (int)strlen(DST)); ok = verify_full(pk, sig, h); }
      printf("%d\n", ok ? 1 : 0);
    } else if (cmd == "mul") {  // mul <g2 compressed> <scalar 32B LE hex> -> compressed
      std::string a, b; is >> a >> b;
      auto pb = unhex(a), kb = unhex(b);
      g2_aff p; g2_decompress(p, pb.data());
      uint32_t k[8]; for (int i = 0; i < 8; ++i) k[i] = kb[4*i] | (kb[4*i+1] << 8) | (kb[4*i+2] << 16) | ((uint32_t)kb[4*i+3] << 24);
      g2_jac r1, r2; jac_mul_aff(r1, p, k, 8); jac_mul_w4(r2, p, k, 8);
      g2_aff a1, a2; jac_to_aff(a1, r1); jac_to_aff(a2, r2);
      uint8_t o1[96], o2[96]; g2_compress(o1, a1); g2_compress(o2, a2);
      printf("%s %s\n", hex(o1, 96).c_str(), hex(o2, 96).c_str());
    } else if (cmd == "sg28") {  // sg28 <n> -> "<agree> <total> <in> <out>": reduced-radix subgroup test vs the engine's
      int n = 0; is >> n;
      int agree = 0, tot = 0, nin = 0, nout = 0;
      uint8_t m[32];
      for (int k = 0; k < 32; ++k) m[k] = (uint8_t)(0x5b * k + 7);
      auto check = [&](const g2_aff& P) {
        const bool a = g2_in_subgroup_inl(P), b = r28::g2_in_subgroup(P);
        agree += a == b; ++tot; nin += a; nout += !a;
      };
      g2_aff inf; inf.inf = 1; inf.x = fp2_zero(); inf.y = fp2_zero();
      check(inf);
      for (int i = 0; i < n; ++i) {
        m[0] = (uint8_t)i; m[1] = (uint8_t)(i >> 8);
        g2_aff P, Hraw;
        hash_to_g2(P, m, (const uint8_t*)DST, (int)strlen(DST));                // in G2
        check(P);
        uint8_t uni[256]; expand_message_xmd_256(uni, m, (const uint8_t*)DST, (int)strlen(DST));
        fp2 u; fp_from_be64_mod(u.c0, uni); fp_from_be64_mod(u.c1, uni + 64);
        fp2 x, y; map_to_curve_sswu(x, y, u); iso3_map(Hraw, x, y);              // on E2, not in G2
        check(Hraw);
        g2_jac j; jac_from_aff(j, P); jac_add_aff(j, j, Hraw); g2_aff S; jac_to_aff(S, j);   // P + Hraw: not in G2
        check(S);
        g2_aff nP = P; fp2_neg(nP.y, nP.y); check(nP);                          // -P: in G2
        const uint32_t kw[2] = {(uint32_t)(0x9e3779b9u * (i + 1)), (uint32_t)i};
        jac_mul_aff(j, P, kw, 2); g2_aff kP; jac_to_aff(kP, j); if (!kP.inf) check(kP);   // [k]P: in G2
      }
      // the reduced-radix arithmetic itself: products, two-product sums, fold / canon against the engine
      int aok = 0, an = 0;
      uint64_t z = 0x9E3779B97F4A7C15ull;
      auto rnd = [&](fp& v) { for (int k = 0; k < 12; ++k) { z ^= z << 13; z ^= z >> 7; z ^= z << 17; v.l[k] = (uint32_t)z; } v.l[11] &= 0x0fffffffu; fp t; fp_to_mont(t, v); v = t; };
      auto back = [&](const r28::f& a) { r28::f y; r28::fold(y, a); r28::f c; r28::canon(c, y); fp o; r28::to32(o.l, c);
                                         fp k = fp_zero(); k.l[11] = 1u << 24; fp t; fp_mul(t, o, k); return t; };   // (x 2^392) 2^376 / 2^384 = x 2^384: engine form
      for (int i = 0; i < 2000; ++i) {
        fp a, b, c, d; rnd(a); rnd(b); rnd(c); rnd(d);
        r28::f A, B, C, D, R; r28::from_engine(A, a); r28::from_engine(B, b); r28::from_engine(C, c); r28::from_engine(D, d);
        fp want; fp_mul(want, a, b);
        r28::mul(R, A, B); aok += fp_eq(back(R), want); ++an;
        fp w2; fp_mul(w2, c, d); fp_add(w2, w2, want);
        r28::mul2(R, A, B, C, D); aok += fp_eq(back(R), w2); ++an;
        // a value near the bounds: A + 64 p, folded
        r28::f Big; for (int k = 0; k < 14; ++k) Big.l[k] = A.l[k] + r28::K64P[k]; r28::norm(Big);
        aok += fp_eq(back(Big), a); ++an;
        // the squaring (cross products once, doubled) == the product a a; and at the top of its range:
        // a 2p - 1 operand (limbs of 2p - 1, normalized)
        fp sq; fp_mul(sq, a, a);
        r28::sqr(R, A); aok += fp_eq(back(R), sq); ++an;
        r28::f T2; r28::add(T2, r28::cst(r28::P28), r28::cst(r28::P28)); T2.l[0] -= 1;   // 2p - 1
        r28::f S1, S2; r28::sqr(S1, T2); r28::mul(S2, T2, T2); aok += fp_eq(back(S1), back(S2)); ++an;
      }
      printf("%d %d %d %d %d %d\n", agree, tot, nin, nout, aok, an);
    } else if (cmd == "invtest") {  // invtest N -> "<ok> <n>": fp_inv (safegcd) == Fermat, a * a^-1 == 1
      int n = 0; is >> n;
      uint64_t z = 0x243F6A8885A308D3ull;
      int ok = 0, cnt = 0;
      for (int i = 0; i < n + 6; ++i) {
        fp c;
        for (int k = 0; k < 12; ++k) { z = z * 6364136223846793005ull + 1442695040888963407ull; c.l[k] = (uint32_t)(z >> 32); }
        c.l[11] &= 0x1fffffffu;
        if (!mp_gt<12>(P_LIMBS, c.l)) c.l[11] &= 0x0fffffffu;
        if (i >= n) {                  // edge cases: 1, 2, p - 1, p - 2, 2^32, 2^380
          for (int k = 0; k < 12; ++k) c.l[k] = 0;
          if (i == n) c.l[0] = 1;
          if (i == n + 1) c.l[0] = 2;
          if (i == n + 2 || i == n + 3) { for (int k = 0; k < 12; ++k) c.l[k] = P_LIMBS[k]; c.l[0] -= (uint32_t)(i - n - 1); }
          if (i == n + 4) c.l[1] = 1;
          if (i == n + 5) c.l[11] = 1u << 28;
        }
        fp a; fp_to_mont(a, c);
        fp x, y, one;
        fp_inv(x, a); fp_inv_fermat(y, a); fp_mul(one, x, a);
        ok += fp_eq(x, y) && fp_eq(one, fp_one());
        ++cnt;
      }
      fp zi; fp_inv(zi, fp_zero());
      ok += fp_is_zero(zi); ++cnt;
      printf("%d %d\n", ok, cnt);
    } else if (cmd == "opcount") {  // opcount pk48 sig96 msg32 -> JSON of per-unit op counts
#ifdef SSB_OPCOUNT
      std::string a, b, c; is >> a >> b >> c;
      auto pkb = unhex(a), sb = unhex(b), mb = unhex(c);
      std::string js = "{";
      auto rec = [&](const char* name, double reps) {
        char tmp[256];
        snprintf(tmp, sizeof tmp, "%s\"%s\": {\"fp_mul\": %.1f, \"fp_sqr\": %.1f, \"fr_mul\": %.1f}",
                 js.size() > 1 ? ", " : "", name, g_ssb_counts.fp_mul / reps, g_ssb_counts.fp_sqr / reps,
                 g_ssb_counts.fr_mul / reps);
        js += tmp;
        g_ssb_counts = {};
      };
      g2_aff sig, H; g1_aff pk;
      g_ssb_counts = {};
      const int NR = 4;
      for (int i = 0; i < NR; ++i) { uint8_t m[32]; for (int k = 0; k < 32; ++k) m[k] = mb[k] ^ (uint8_t)i; hash_to_g2(H, m, (const uint8_t*)DST, (int)strlen(DST)); }
      rec("hash_to_g2", NR);
      hash_to_g2(H, mb.data(), (const uint8_t*)DST, (int)strlen(DST));
      g_ssb_counts = {};
      uint32_t fl = unit_decode(sig, pk, sb.data(), pkb.data(), 1);
      rec("decode", 1);
      if (!(fl & FLAG_CANDIDATE)) { printf("ERR not a candidate\n"); fflush(stdout); continue; }
      unit_decode_sig(sig, sb.data()); rec("decode_sig", 1);
      unit_decode_pk(pk, pkb.data()); rec("decode_pk", 1);
      unit_subgroup(sig, nullptr); rec("subgroup", 1);
      const int NS = 16;
      g2_jac rs; g1_jac rp;
      for (int i = 0; i < NS; ++i) unit_rlc_sig(rs, sig, rlc_scalar(0x5AFE57A4Eull, (uint64_t)i));
      rec("rlc_sig", NS);
      for (int i = 0; i < NS; ++i) unit_rlc_pk(rp, pk, rlc_scalar(0x5AFE57A4Eull, (uint64_t)i));
      rec("rlc_pk", NS);
      for (int i = 0; i < NS; ++i) unit_rlc(rs, rp, sig, pk, rlc_scalar(0x5AFE57A4Eull, (uint64_t)i));
      rec("rlc", NS);
      g1_jac acc1; jac_set_inf(acc1); jac_add(acc1, acc1, rp); g_ssb_counts = {};
      for (int i = 0; i < NS; ++i) jac_add(acc1, acc1, rp);
      rec("sum_g1_add", NS);
      g2_jac acc2; jac_set_inf(acc2); jac_add(acc2, acc2, rs); jac_dbl(acc2, acc2); g_ssb_counts = {};
      for (int i = 0; i < NS; ++i) jac_add(acc2, acc2, rs);
      rec("sum_g2_add", NS);
      for (int i = 0; i < NS; ++i) jac_add_aff(acc1, acc1, pk);
      rec("madd_g1", NS);
      for (int i = 0; i < NS; ++i) jac_add_aff(acc2, acc2, sig);
      rec("madd_g2", NS);
      for (int i = 0; i < NS; ++i) jac_dbl(acc1, acc1);
      rec("dbl_g1", NS);
      for (int i = 0; i < NS; ++i) jac_dbl(acc2, acc2);
      rec("dbl_g2", NS);
      { g1_aff a1; jac_to_aff(a1, acc1); } rec("to_affine_g1", 1);
      { g2_aff a2; jac_to_aff(a2, acc2); } rec("to_affine_g2", 1);
      fp12 f; miller_loop(f, pk, H); rec("miller_pair", 1);
      fp12 f2; fp12_mul(f2, f, f); rec("fp12_mul", 1);
      fp12 e; final_exponentiation(e, f2); rec("final_exp", 1);
      bool ok = unit_verify_one(pk, sig, H); rec("verify_one", 1);
      const uint64_t ids3[3] = {1, 2, 3}, ids5[5] = {1, 2, 3, 4, 5}, ids10[10] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10};
      fr lam[10];
      unit_lagrange(lam, ids3, 3); rec("lagrange_t3", 1);
      unit_lagrange(lam, ids5, 5); rec("lagrange_t5", 1);
      unit_lagrange(lam, ids10, 10); rec("lagrange_t10", 1);
      g2_jac terms[10];
      for (int i = 0; i < NS; ++i) { uint32_t l8[8]; for (int k = 0; k < 8; ++k) l8[k] = (uint32_t)rlc_scalar(77, 8 * i + k); l8[7] &= 0x73eda752u; unit_combine_term(terms[i % 10], sig, l8); }
      rec("combine_term", NS);
      uint8_t o96[96];
      unit_combine_sum(o96, terms, 3); rec("combine_sum_t3", 1);
      unit_combine_sum(o96, terms, 10); rec("combine_sum_t10", 1);
      { // small-integer Lagrange path (ids 1..t): coefficients + the shared-doubling combination
        const g2_aff* pp[10] = {&sig, &H, &sig, &H, &sig, &H, &sig, &H, &sig, &H};
        int64_t c[10];
        unit_lagrange_small(c, ids3, 3); unit_combine_small(o96, pp, c, 3); rec("combine_small_t3", 1);
        unit_lagrange_small(c, ids5, 5); unit_combine_small(o96, pp, c, 5); rec("combine_small_t5", 1);
        unit_lagrange_small(c, ids10, 10); unit_combine_small(o96, pp, c, 10); rec("combine_small_t10", 1); }
      js += ok ? ", \"verify_ok\": true}" : ", \"verify_ok\": false}";
      printf("%s\n", js.c_str());
#else
      printf("disabled\n");
#endif
    } else if (cmd == "rlc") {  // rlc <seed> <i> [key 8 words hex]: the device RLC scalar derivation
      std::string a, b; is >> a >> b;
      const uint64_t seed = std::stoull(a, nullptr, 0), i = std::stoull(b, nullptr, 0);
      rlc_key k = rlc_key_from_seed(seed);
      std::string w;
      for (int q = 0; q < 8 && (is >> w); ++q) k.w[q] = (uint32_t)std::stoul(w, nullptr, 16);
      printf("%llu\n", (unsigned long long)rlc_scalar_odd(k, i));
    } else if (cmd == "lagsmall") {  // lagsmall t id1 .. idt : fast integer path vs 255-bit path
      int t; is >> t; std::vector<uint64_t> ids(t); for (int i = 0; i < t; ++i) is >> ids[i];
      std::vector<g2_aff> P(t); std::vector<const g2_aff*> pp(t);
      for (int i = 0; i < t; ++i) { uint8_t m[32] = {0}; m[0] = (uint8_t)i; m[1] = 0x77; hash_to_g2(P[i], m, (const uint8_t*)DST, (int)strlen(DST)); pp[i] = &P[i]; }
      std::vector<int64_t> c(t); std::vector<fr> lam(t);
      const bool elig = unit_lagrange_small(c.data(), ids.data(), (uint32_t)t);
      unit_lagrange(lam.data(), ids.data(), (uint32_t)t);
      std::vector<g2_jac> terms(t);
      for (int i = 0; i < t; ++i) unit_combine_term(terms[i], P[i], lam[i].l);
      uint8_t a[96], b[96]; unit_combine_sum(a, terms.data(), (uint32_t)t);
      int same = -1;
      if (elig) { unit_combine_small(b, pp.data(), c.data(), (uint32_t)t); same = memcmp(a, b, 96) == 0; }
      printf("%d %d\n", elig ? 1 : 0, same);
    } else if (cmd == "lagratio") {  // lagratio t id1 .. idt : registry ratio path vs 255-bit path
      int t; is >> t; std::vector<uint64_t> ids(t); for (int i = 0; i < t; ++i) is >> ids[i];
      std::vector<g2_aff> P(t); std::vector<uint32_t> idx(t);
      for (int i = 0; i < t; ++i) { uint8_t m[32] = {0}; m[0] = (uint8_t)i; m[1] = 0x5a; hash_to_g2(P[i], m, (const uint8_t*)DST, (int)strlen(DST)); idx[i] = (uint32_t)i; }
      std::vector<int64_t> c(t); std::vector<fr> lam(t); uint64_t M = 0;
      const bool elig = unit_lagrange_ratio(c.data(), &M, ids.data(), (uint32_t)t);
      unit_lagrange(lam.data(), ids.data(), (uint32_t)t);
      std::vector<g2_jac> terms(t);
      for (int i = 0; i < t; ++i) unit_combine_term(terms[i], P[i], lam[i].l);
      uint8_t a[96], b[96]; unit_combine_sum(a, terms.data(), (uint32_t)t);
      int same = -1;
      if (elig) {
        // the lane-uniform windowed combine (k_combine_ratio), at the job's own window count and at a
        // wider one (the wave's maximum on the device), with the table region in host memory
        std::vector<uint8_t> region(RC_TAB_BYTES);
        const int W = rc_windows(c.data(), (uint32_t)t);
        unit_combine_ratio_w4(b, P.data(), idx.data(), c.data(), (uint32_t)t, M, W, region.data());
        same = memcmp(a, b, 96) == 0;
        unit_combine_ratio_w4(b, P.data(), idx.data(), c.data(), (uint32_t)t, M, 16, region.data());
        same = same && memcmp(a, b, 96) == 0;
      }
      printf("%d %d %llu\n", elig ? 1 : 0, same, (unsigned long long)M);
    } else if (cmd == "ratiozero") {  // ratiozero t id1 .. idt: P_i = [x_i] P, so T = sum c_i x_i P = O -> infinity
      int t; is >> t; std::vector<uint64_t> ids(t); for (int i = 0; i < t; ++i) is >> ids[i];
      g2_aff H; { uint8_t m[32] = {0}; m[0] = 0x33; hash_to_g2(H, m, (const uint8_t*)DST, (int)strlen(DST)); }
      std::vector<g2_aff> P(t); std::vector<uint32_t> idx(t);
      for (int i = 0; i < t; ++i) {
        const uint32_t kw[2] = {(uint32_t)ids[i], (uint32_t)(ids[i] >> 32)};
        g2_jac r; jac_mul_aff(r, H, kw, 2); jac_to_aff(P[i], r); idx[i] = (uint32_t)i;
      }
      std::vector<int64_t> c(t); uint64_t M = 0;
      const bool elig = unit_lagrange_ratio(c.data(), &M, ids.data(), (uint32_t)t);
      uint8_t b[96] = {0};
      std::vector<uint8_t> region(RC_TAB_BYTES);
      if (elig) unit_combine_ratio_w4(b, P.data(), idx.data(), c.data(), (uint32_t)t, M, rc_windows(c.data(), (uint32_t)t), region.data());
      printf("%d %s\n", elig ? 1 : 0, hex(b, 96).c_str());
    } else if (cmd == "lagfast") {  // lagfast t id1 .. idt : unit_lagrange_fast's lambda_i (canonical hex, one per share)
      int t; is >> t; std::vector<uint64_t> ids(t); for (int i = 0; i < t; ++i) is >> ids[i];
      std::vector<fr> lam(t);
      unit_lagrange_fast(lam.data(), ids.data(), (uint32_t)t);
      std::string o;
      for (int i = 0; i < t; ++i) {
        char buf[72];
        for (int k = 7; k >= 0; --k) snprintf(buf + 8 * (7 - k), 9, "%08x", lam[i].l[k]);
        o += (i ? " " : ""); o += buf;
      }
      printf("%s\n", o.c_str());
    } else if (cmd == "invsmall") {  // invsmall M: M^-1 mod r (4 limbs hex, most significant first) and its GLS digits
      std::string a; is >> a;
      const uint64_t M = std::stoull(a, nullptr, 0);
      uint64_t y[4], d[4];
      inv_small_mod_r(y, M);
      gls_digits4(d, y);
      printf("%016llx%016llx%016llx%016llx %llu %llu %llu %llu\n", (unsigned long long)y[3], (unsigned long long)y[2],
             (unsigned long long)y[1], (unsigned long long)y[0], (unsigned long long)d[0], (unsigned long long)d[1],
             (unsigned long long)d[2], (unsigned long long)d[3]);
    } else if (cmd == "madd") {  // madd <trials>: jac_madd_at (bucket loops) vs jac_add_aff_inl, incl. special cases
      int trials; is >> trials;
      int bad = 0, n = 0;
      auto same = [](const auto& a, const auto& b) { return memcmp(&a, &b, sizeof(a)) == 0; };
      for (int tr = 0; tr < trials; ++tr) {
        uint8_t m[32] = {0}; m[0] = (uint8_t)tr; m[1] = (uint8_t)(tr >> 8); m[2] = 0x3c;
        g2_aff P, Q; hash_to_g2(P, m, (const uint8_t*)DST, (int)strlen(DST));
        m[3] = 1; hash_to_g2(Q, m, (const uint8_t*)DST, (int)strlen(DST));
        g2_jac A; jac_from_aff(A, P); jac_dbl(A, A); jac_add_aff(A, A, Q);    // Z != 1
        g2_aff Aa; jac_to_aff(Aa, A);
        g2_aff nAa = Aa; fp2_neg(nAa.y, nAa.y);
        g2_aff inf = Q; inf.inf = 1;
        g2_jac I; jac_set_inf(I);
        const g2_jac accs[4] = {A, A, A, I};
        const g2_aff qs[4] = {Q, Aa, nAa, Q};
        for (int c = 0; c < 5; ++c) {
          const g2_jac a0 = c < 4 ? accs[c] : A;
          const g2_aff q = c < 4 ? qs[c] : inf;
          g2_jac want; jac_add_aff_inl(want, a0, q);
          g2_jac got = a0; jac_madd_at(got, &q);
          ++n; if (!same(want, got)) ++bad;
        }
        // G1 (the cached keys' bases): the same over Fp
        g1_aff g = g1_neg_generator(); fp_neg(g.y, g.y);
        g1_jac B; jac_from_aff(B, g); for (int k = 0; k <= tr % 7; ++k) jac_dbl(B, B);
        g1_aff Ba; jac_to_aff(Ba, B);
        g1_jac w1; jac_add_aff_inl(w1, B, g); g1_jac g1v = B; jac_madd_at(g1v, &g);
        g1_jac w2; jac_add_aff_inl(w2, B, Ba); g1_jac g2v = B; jac_madd_at(g2v, &Ba);
        n += 2; bad += !same(w1, g1v); bad += !same(w2, g2v);
      }
      printf("%d %d\n", n - bad, n);
    } else if (cmd == "pt28") {  // pt28 <trials>: the MSM's reduced-radix complete additions vs the engine's
      int trials; is >> trials;
      int bad = 0, n = 0;
      auto eqp = [](const g2_jac& a, const g2_jac& b) {   // the same point (affine compare)
        g2_aff x, y; jac_to_aff(x, a); jac_to_aff(y, b);
        return x.inf == y.inf && (x.inf || (fp2_eq(x.x, y.x) && fp2_eq(x.y, y.y)));
      };
      uint32_t keep[r28::KEEP_WORDS];
      for (int tr = 0; tr < trials; ++tr) {
        uint8_t m[32] = {0}; m[0] = (uint8_t)tr; m[1] = (uint8_t)(tr >> 8); m[2] = 0x51;
        g2_aff P, Q; hash_to_g2(P, m, (const uint8_t*)DST, (int)strlen(DST));
        m[3] = 1; hash_to_g2(Q, m, (const uint8_t*)DST, (int)strlen(DST));
        g2_jac A; jac_from_aff(A, P); jac_dbl(A, A); jac_add_aff(A, A, Q);   // Z != 1
        g2_aff Aa; jac_to_aff(Aa, A);
        g2_aff nAa = Aa; fp2_neg(nAa.y, nAa.y);
        g2_aff infa = Q; infa.inf = 1;
        g2_jac I; jac_set_inf(I);
        g2_jac B; jac_from_aff(B, Q); jac_dbl(B, B); jac_dbl(B, B);          // another Z != 1
        g2_jac nA = A; fp2_neg(nA.y, A.y);
        // madd: random, acc == P (doubling), acc == -P (infinity), acc at infinity, P at infinity; chained
        const g2_jac accs[5] = {A, A, A, I, A};
        const g2_aff qs[5] = {Q, Aa, nAa, Q, infa};
        for (int c = 0; c < 5; ++c) {
          g2_jac want; jac_add_aff_inl(want, accs[c], qs[c]);
          r28::pt2 a; r28::pt2_from_engine(a, accs[c]);
          r28::pt2_madd<1>(a, qs[c], keep);
          g2_jac got; r28::pt2_to_engine(got, a);
          ++n; bad += !eqp(want, got);
        }
        { r28::pt2 a; r28::pt2_set_inf(a); g2_jac want; jac_set_inf(want);
          for (int k = 0; k < 9; ++k) { const g2_aff& q = (k % 3 == 2) ? nAa : (k & 1 ? Q : P);
            r28::pt2_madd<1>(a, q, keep); jac_add_aff_inl(want, want, q); }
          g2_jac got; r28::pt2_to_engine(got, a); ++n; bad += !eqp(want, got); }
        // add: random, a == b (doubling), a == -b, either at infinity; dbl
        const g2_jac xs[5] = {A, A, A, I, A}, ys[5] = {B, A, nA, B, I};
        for (int c = 0; c < 5; ++c) {
          g2_jac want; jac_add_inl(want, xs[c], ys[c]);
          r28::pt2 a, b; r28::pt2_from_engine(a, xs[c]); r28::pt2_from_engine(b, ys[c]);
          r28::pt2_add(a, b);
          g2_jac got; r28::pt2_to_engine(got, a);
          ++n; bad += !eqp(want, got);
        }
        { g2_jac want; jac_dbl(want, B); r28::pt2 a; r28::pt2_from_engine(a, B); r28::pt2_dbl(a);
          g2_jac got; r28::pt2_to_engine(got, a); ++n; bad += !eqp(want, got); }
        // G1: the merged MSM's bucket additions (pt1_madd): random, a == P, a == -P, a at infinity, chained
        { g1_aff g = g1_neg_generator(); fp_neg(g.y, g.y);
          g1_jac B1; jac_from_aff(B1, g); for (int k = 0; k <= tr % 5 + 1; ++k) jac_dbl(B1, B1);   // Z != 1
          g1_aff Ba; jac_to_aff(Ba, B1); g1_aff nBa = Ba; fp_neg(nBa.y, Ba.y);
          g1_jac I1; jac_set_inf(I1);
          const g1_jac as1[4] = {B1, B1, B1, I1}; const g1_aff qs1[4] = {g, Ba, nBa, g};
          auto eq1 = [](const g1_jac& a, const g1_jac& b) { g1_aff x, y; jac_to_aff(x, a); jac_to_aff(y, b);
                                                         return x.inf == y.inf && (x.inf || (fp_eq(x.x, y.x) && fp_eq(x.y, y.y))); };
          for (int c = 0; c < 4; ++c) {
            g1_jac want; jac_add_aff_inl(want, as1[c], qs1[c]);
            r28::pt1 a; a.inf = jac_is_inf(as1[c]);
            r28::from_engine_shift(a.x, as1[c].x); r28::from_engine_shift(a.y, as1[c].y); r28::from_engine_shift(a.z, as1[c].z);
            r28::pt1_madd(a, qs1[c]);
            g1_jac got; r28::pt1_to_engine(got, a); ++n; bad += !eq1(want, got);
          }
          r28::pt1 a; a.inf = true; g1_jac want; jac_set_inf(want);
          for (int k = 0; k < 7; ++k) { const g1_aff& q = (k % 3 == 2) ? nBa : (k & 1 ? g : Ba);
            r28::pt1_madd(a, q); jac_add_aff_inl(want, want, q); }
          g1_jac got; r28::pt1_to_engine(got, a); ++n; bad += !eq1(want, got); }
        // a running window sum in both forms (the window kernel's S / U recurrences)
        { r28::pt2 S, U, o; r28::pt2_set_inf(S); r28::pt2_set_inf(U); g2_jac Se, Ue; jac_set_inf(Se); jac_set_inf(Ue);
          const g2_jac bk[4] = {A, B, I, nA};
          for (int e = 3; e >= 0; --e) { r28::pt2_from_engine(o, bk[e]); r28::pt2_add(S, o); r28::pt2_add(U, S);
            jac_add_inl(Se, Se, bk[e]); jac_add_inl(Ue, Ue, Se); }
          g2_jac got; r28::pt2_to_engine(got, U); ++n; bad += !eqp(Ue, got); }
      }
      printf("%d %d\n", n - bad, n);
    } else if (cmd == "lafin") {  // lafin <trials>: accumulator engine (reduced radix) vs repeated modular add/sub
      int trials; is >> trials;
      uint64_t st = 0x9E3779B97F4A7C15ull;
      auto rnd = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
      int bad = 0;
      lane::lv pm1 = r28::cst(r28::P28); pm1.l[0] -= 1;                 // p - 1
      lane::lv tpm1; r28::add(tpm1, pm1, r28::cst(r28::P28));             // 2p - 1 (the slot bound)
      for (int tr = 0; tr < trials; ++tr) {
        const int t = 1 + (int)(rnd() % 16);
        lane::lacc A; lane::la_zero(A);
        uint32_t K = 0;
        fp want = fp_zero();
        for (int k = 0; k < t; ++k) {
          lane::lv v;
          const int kind = (int)(rnd() % 4);
          if (kind == 0) v = lane::lv_zero();
          else if (kind == 1) v = pm1;
          else if (kind == 2) v = tpm1;
          else { fp e; for (int i = 0; i < 12; ++i) e.l[i] = (uint32_t)rnd(); e.l[11] &= 0x0fffffffu; v = lane::lv_in(e); }
          const fp ve = lane::lv_out(v);
          const int m = (tr & 1) ? 1 + (int)(rnd() % 60) : 1 + (int)(rnd() % 3);
          const bool neg = rnd() & 1;
          if (neg) { lane::la_neg(A, v, (uint32_t)m); K += (uint32_t)m; } else lane::la_pos(A, v, (uint32_t)m);
          for (int j = 0; j < m; ++j) { if (neg) fp_sub(want, want, ve); else fp_add(want, want, ve); }
        }
        lane::lv r, r2; lane::la_fin(r, A, K, true); lane::la_fin(r2, A, K, false);
        lane::lv r2f; r28::fold(r2f, r2);
        if (!fp_eq(lane::lv_out(r), want) || !fp_eq(lane::lv_out(r2f), want)) ++bad;
        // the fold's bound: r <= 2p - 1 (normalized limbs, compared from the top)
        int cmp = 0;
        for (int i = 13; i >= 0 && cmp == 0; --i) cmp = r.l[i] < tpm1.l[i] ? -1 : (r.l[i] > tpm1.l[i] ? 1 : 0);
        for (int i = 0; i < 13; ++i) if (r.l[i] >> 28) cmp = 1;
        if (cmp > 0) ++bad;
      }
      printf("%d\n", bad);
    } else if (cmd == "lane") {  // lane <seed32hex>: lane-group programs vs single-lane code
      std::string s; is >> s; auto b = unhex(s);
      lane_selftest(b.data());
    } else if (cmd.empty()) {
      continue;
    } else {
      printf("ERR unknown %s\n", cmd.c_str());
    }
    fflush(stdout);
  }
  return 0;
}
