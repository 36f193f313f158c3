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
#include "../../safestakeoperator_amd/csrc/ssb_wave.h"

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

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    std::istringstream is(line);
    std::string cmd; is >> cmd;
    if (cmd == "h2g2") {  // h2g2 <msg32hex> [dsthex]
      std::string m, d; is >> m >> d;
      auto msg = unhex(m);
      std::vector<uint8_t> dst = d.empty() ? std::vector<uint8_t>(DST, DST + strlen(DST)) : unhex(d);
      g2_aff h; hash_to_g2(h, msg.data(), dst.data(), (int)dst.size());
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
      unit_subgroup(sig); rec("subgroup", 1);
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
      js += ok ? ", \"verify_ok\": true}" : ", \"verify_ok\": false}";
      printf("%s\n", js.c_str());
#else
      printf("disabled\n");
#endif
    } else if (cmd == "wave") {  // wave pk48 sig96 msg32: wave programs vs single-lane code
      std::string a, b, c; is >> a >> b >> c;
      auto pkb = unhex(a), sb = unhex(b), mb = unhex(c);
      g1_aff pk; g2_aff sig, H;
      g1_decompress(pk, pkb.data()); g2_decompress(sig, sb.data());
      hash_to_g2(H, mb.data(), (const uint8_t*)DST, (int)strlen(DST));
      std::vector<fp> slots(wave::S_USER + 256);
      wave::ws w{slots.data()};
      wave::init(w, 0, 1);
      const int U = wave::S_USER;
      fp12 f1, f2, r1, r2;
      miller_loop(f1, pk, H);
      g1_aff ng = g1_neg_generator();
      miller_loop(f2, ng, sig);
      int ok = 0, n = 0;
      // FP12_MUL, FP12_SQR
      wave::store12(w, U, f1); wave::store12(w, U + 12, f2);
      wave::run(w, wave::FP12_MUL, U, U + 12, U + 24, 0, 1);
      fp12_mul(r1, f1, f2); wave::load12(r2, w, U + 24); ok += fp12_eq(r1, r2); ++n;
      wave::run(w, wave::FP12_SQR, U, 0, U + 24, 0, 1);
      fp12_sqr(r1, f1); wave::load12(r2, w, U + 24); ok += fp12_eq(r1, r2); ++n;
      // frobenius, conj
      for (int k = 1; k <= 3; ++k) {
        wave::run(w, k == 1 ? wave::FP12_FROB1 : k == 2 ? wave::FP12_FROB2 : wave::FP12_FROB3, U, 0, U + 24, 0, 1);
        fp12_frob(r1, f1, k); wave::load12(r2, w, U + 24); ok += fp12_eq(r1, r2); ++n;
      }
      wave::run(w, wave::FP12_CONJ, U, 0, U + 24, 0, 1);
      fp12_conj(r1, f1); wave::load12(r2, w, U + 24); ok += fp12_eq(r1, r2); ++n;
      // sparse line multiply (in place)
      { fp2 l0 = H.x, l1 = H.y, l4 = sig.x;
        for (int k = 0; k < 6; ++k) {}
        w.s[U + 36] = l0.c0; w.s[U + 37] = l0.c1; w.s[U + 38] = l1.c0; w.s[U + 39] = l1.c1; w.s[U + 40] = l4.c0; w.s[U + 41] = l4.c1;
        wave::store12(w, U + 24, f1);
        wave::run(w, wave::FP12_MUL_014, U + 24, U + 36, U + 24, 0, 1);
        fp12_mul_014(r1, f1, l0, l1, l4); wave::load12(r2, w, U + 24); ok += fp12_eq(r1, r2); ++n; }
      // cyclotomic square on a cyclotomic element: f^((p^6-1)(p^2+1))
      { fp12 t0, t1, g; fp12_conj(t0, f1); fp12_inv(t1, f1); fp12_mul(g, t0, t1); fp12_frob(t0, g, 2); fp12_mul(g, t0, g);
        wave::store12(w, U, g); wave::run(w, wave::FP12_CYC_SQR, U, 0, U + 24, 0, 1);
        fp12_cyc_sqr(r1, g); wave::load12(r2, w, U + 24); ok += fp12_eq(r1, r2); ++n;
        fp12 g2; fp12_sqr(g2, g); ok += fp12_eq(g2, r1); ++n; }
      // final exponentiation
      { fp12 m; fp12_mul(m, f1, f2); final_exponentiation(r1, m);
        wave::store12(w, U, m); wave::final_exp(w, U, U + 12, 0, 1); wave::load12(r2, w, U);
        ok += fp12_eq(r1, r2); ++n; ok += fp12_is_one(r2); ++n; }
      // Miller loop for the pair (pk, H)
      { const int B0 = U + 120;
        w.s[B0 + 24] = H.x.c0; w.s[B0 + 25] = H.x.c1; w.s[B0 + 26] = H.y.c0; w.s[B0 + 27] = H.y.c1;
        w.s[B0 + 28] = pk.x; w.s[B0 + 29] = pk.y;
        wave::miller(w, B0, 0, 1);
        wave::load12(r2, w, B0); ok += fp12_eq(f1, r2); ++n; }
      printf("%d %d\n", ok, n);
    } else if (cmd.empty()) {
      continue;
    } else {
      printf("ERR unknown %s\n", cmd.c_str());
    }
    fflush(stdout);
  }
  return 0;
}
