// Host build of the device math headers, for CPU unit tests against the oracle and for the
// algorithmic op counter.  TEST INFRASTRUCTURE: not part of libssbls.so.
// Protocol: one command per stdin line, one result line per command on stdout.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <iostream>
#include <sstream>
#include "../../safestakeoperator_amd/csrc/ssb_pairing.h"
#include "../../safestakeoperator_amd/csrc/ssb_h2c.h"

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
    } else if (cmd == "opcount") {  // opcount <what>
#ifdef SSB_OPCOUNT
      std::string what; is >> what;
      g_ssb_counts = {};
      printf("n/a\n");
#else
      printf("disabled\n");
#endif
    } else if (cmd.empty()) {
      continue;
    } else {
      printf("ERR unknown %s\n", cmd.c_str());
    }
    fflush(stdout);
  }
  return 0;
}
