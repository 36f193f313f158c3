// ssb_wave.h -- wave-cooperative execution of the tower programs in ssb_wave_tables.h.
//
// The latency-bound parts of the batch check (one final exponentiation per batch, one Miller
// loop per (root, sum) pair) are long chains of Fp12 / Miller-step operations.  Run on a single
// lane, each Fp12 multiply is 54 dependent-issue Fp multiplies.  Here a whole wavefront
// cooperates on one operation: every lane computes one independent Fp product of the current
// phase (operands are +-sums of LDS slots), then a few lanes form the linear outputs.  The
// programs are generated from the same formulas (gen_wave_tables.py) and checked against the
// single-lane code (tests/native).
//
// The executor is written against (lane, nlanes): on the device lane = threadIdx.x,
// nlanes = 64 and SSB_WAVE_SYNC() is a workgroup barrier; on the host (tests) lane = 0,
// nlanes = 1 and the loops run every entry in order.
#pragma once
#include "ssb_pairing.h"
#include "ssb_wave_tables.h"

#if defined(__HIP_DEVICE_COMPILE__)
#define SSB_WAVE_SYNC() __syncthreads()
#else
#define SSB_WAVE_SYNC() ((void)0)
#endif

namespace ssb {
namespace wave {

// LDS layout of one wave's working set (in Fp slots)
enum : int {
  S_ZERO = 0,
  S_FROB = 1,                       // 3 x 10: gamma_{n,k} components, n = 1..3, k = 1..5
  S_PSCR = S_FROB + 30,             // products
  S_MSCR = S_PSCR + MAX_PROD,       // materialisations
  S_OSCR = S_MSCR + MAX_MAT,        // output staging
  S_USER = S_OSCR + MAX_OUT,        // caller-owned values start here
};

struct ws { fp* s; };  // slot array (LDS on the device)

SSB_INL int kslot(const prog& pg, int k) {
  const int n = pg.kconst[3 * k], kk = pg.kconst[3 * k + 1], c = pg.kconst[3 * k + 2];
  return S_FROB + (n - 1) * 10 + (kk - 1) * 2 + c;
}

SSB_INL int map_slot(const prog& pg, int i, int a, int b) {
  if (i == 0) return S_ZERO;
  i -= 1;
  if (i < pg.na) return a + i;
  i -= pg.na;
  if (i < pg.nb) return b + i;
  i -= pg.nb;
  if (i < pg.nk) return kslot(pg, i);
  i -= pg.nk;
  if (i < pg.nprod) return S_PSCR + i;
  i -= pg.nprod;
  return S_MSCR + i;
}

SSB_INL void form(fp& r, const ws& w, const prog& pg, const uint8_t* t, int np, int nn, int a, int b) {
  fp acc = fp_zero(), neg = fp_zero();
  for (int i = 0; i < np; ++i) fp_add(acc, acc, w.s[map_slot(pg, t[i], a, b)]);
  for (int i = 0; i < nn; ++i) fp_add(neg, neg, w.s[map_slot(pg, t[np + i], a, b)]);
  fp_sub(r, acc, neg);
}

// Run program `pg` with inputs at slots [a, a+na), [b, b+nb); outputs to [dst, dst+nout).
// dst may alias the inputs.
SSB_FN void run(const ws& w, const prog& pg, int a, int b, int dst, int lane, int nlanes) {
  int p0 = 0, m0 = 0, li = 0;
  for (int ph = 0; ph < pg.nphase; ++ph) {
    const int p1 = pg.phase_end[ph];
    for (int L = p0 + lane; L < p1; L += nlanes) {
      const uint8_t* c = pg.cnt + 4 * L;
      const uint8_t* t = pg.terms + pg.off[L];
      fp x, y;
      form(x, w, pg, t, c[0], c[1], a, b);
      form(y, w, pg, t + c[0] + c[1], c[2], c[3], a, b);
      fp_mul(w.s[S_PSCR + L], x, y);
    }
    SSB_WAVE_SYNC();
    p0 = p1;
    for (; li < pg.nlin && pg.lin[2 * li] == ph; ++li) {  // linear stages (levels) after this phase
      const int m1 = pg.lin[2 * li + 1];
      for (int M = m0 + lane; M < m1; M += nlanes) {
        fp r;
        form(r, w, pg, pg.terms + pg.ooff[M], pg.ocnt[2 * M], pg.ocnt[2 * M + 1], a, b);
        w.s[S_MSCR + M] = r;
      }
      SSB_WAVE_SYNC();
      m0 = m1;
    }
  }
  for (int j = lane; j < pg.nout; j += nlanes) {
    const int o = pg.nmat + j;
    fp r;
    form(r, w, pg, pg.terms + pg.ooff[o], pg.ocnt[2 * o], pg.ocnt[2 * o + 1], a, b);
    w.s[S_OSCR + j] = r;
  }
  SSB_WAVE_SYNC();
  for (int j = lane; j < pg.nout; j += nlanes) w.s[dst + j] = w.s[S_OSCR + j];
  SSB_WAVE_SYNC();
}

SSB_FN void init(const ws& w, int lane, int nlanes) {
  for (int i = lane; i < 31; i += nlanes) {
    if (i == 0) { w.s[S_ZERO] = fp_zero(); continue; }
    const int j = i - 1, n = j / 10 + 1, k = (j % 10) / 2 + 1, c = j % 2;
    const fp2_c& g = (n == 1) ? FROB1[k] : (n == 2) ? FROB2[k] : FROB3[k];
    w.s[i] = fp_from_c(c ? g.c1 : g.c0);
  }
  SSB_WAVE_SYNC();
}

// Fp12 value <-> 12 consecutive slots (c0.c0.c0, c0.c0.c1, c0.c1.c0, ..., c1.c2.c1)
SSB_INL void store12(const ws& w, int at, const fp12& f) {
  const fp2* q = &f.c0.c0;
  const fp2 v[6] = {f.c0.c0, f.c0.c1, f.c0.c2, f.c1.c0, f.c1.c1, f.c1.c2};
  (void)q;
  for (int k = 0; k < 6; ++k) { w.s[at + 2 * k] = v[k].c0; w.s[at + 2 * k + 1] = v[k].c1; }
}
SSB_INL void load12(fp12& f, const ws& w, int at) {
  fp2* v[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int k = 0; k < 6; ++k) { v[k]->c0 = w.s[at + 2 * k]; v[k]->c1 = w.s[at + 2 * k + 1]; }
}

SSB_FN void copy12(const ws& w, int dst, int src, int lane, int nlanes) {
  for (int j = lane; j < 12; j += nlanes) w.s[dst + j] = w.s[src + j];
  SSB_WAVE_SYNC();
}

SSB_FN void set_one12(const ws& w, int dst, int lane, int nlanes) {
  for (int j = lane; j < 12; j += nlanes) w.s[dst + j] = (j == 0) ? fp_one() : fp_zero();
  SSB_WAVE_SYNC();
}

// r = f^x (x = -0xd201000000010000), f cyclotomic; r must differ from f
SSB_FN void cyc_exp_x(const ws& w, int r, int f, int lane, int nlanes) {
  copy12(w, r, f, lane, nlanes);
  for (int i = 62; i >= 0; --i) {
    run(w, FP12_CYC_SQR, r, 0, r, lane, nlanes);
    if ((BLS_X_ABS >> i) & 1ull) run(w, FP12_MUL, r, f, r, lane, nlanes);
  }
  run(w, FP12_CONJ, r, 0, r, lane, nlanes);
}

// Final exponentiation of the value at slot `f` (12 slots), result in place.
// Uses 8 x 12 scratch slots starting at `tmp`.  Same chain as ssb::final_exponentiation.
SSB_FN void final_exp(const ws& w, int f, int tmp, int lane, int nlanes) {
  const int t0 = tmp, t1 = tmp + 12, t2 = tmp + 24, t3 = tmp + 36, t4 = tmp + 48, t5 = tmp + 60, t6 = tmp + 72;
  run(w, FP12_CONJ, f, 0, t0, lane, nlanes);
  if (lane == 0) {  // one inversion: a single lane
    fp12 x, xi;
    load12(x, w, f);
    fp12_inv(xi, x);
    store12(w, t1, xi);
  }
  SSB_WAVE_SYNC();
  run(w, FP12_MUL, t0, t1, t2, lane, nlanes);
  copy12(w, t1, t2, lane, nlanes);
  run(w, FP12_FROB2, t2, 0, t2, lane, nlanes);
  run(w, FP12_MUL, t2, t1, t2, lane, nlanes);
  run(w, FP12_CYC_SQR, t2, 0, t1, lane, nlanes);
  run(w, FP12_CONJ, t1, 0, t1, lane, nlanes);
  cyc_exp_x(w, t3, t2, lane, nlanes);
  run(w, FP12_CYC_SQR, t3, 0, t4, lane, nlanes);
  run(w, FP12_MUL, t1, t3, t5, lane, nlanes);
  cyc_exp_x(w, t1, t5, lane, nlanes);
  cyc_exp_x(w, t0, t1, lane, nlanes);
  cyc_exp_x(w, t6, t0, lane, nlanes);
  run(w, FP12_MUL, t6, t4, t6, lane, nlanes);
  cyc_exp_x(w, t4, t6, lane, nlanes);
  run(w, FP12_CONJ, t5, 0, t5, lane, nlanes);
  run(w, FP12_MUL, t5, t2, t5, lane, nlanes);
  run(w, FP12_MUL, t4, t5, t4, lane, nlanes);
  run(w, FP12_CONJ, t2, 0, t5, lane, nlanes);
  run(w, FP12_MUL, t1, t2, t1, lane, nlanes);
  run(w, FP12_FROB3, t1, 0, t1, lane, nlanes);
  run(w, FP12_MUL, t6, t5, t6, lane, nlanes);
  run(w, FP12_FROB1, t6, 0, t6, lane, nlanes);
  run(w, FP12_MUL, t3, t0, t3, lane, nlanes);
  run(w, FP12_FROB2, t3, 0, t3, lane, nlanes);
  run(w, FP12_MUL, t3, t1, t3, lane, nlanes);
  run(w, FP12_MUL, t3, t6, t3, lane, nlanes);
  run(w, FP12_MUL, t3, t4, f, lane, nlanes);
}

// Miller loop f_{|x|,Q}(P) (conjugated) for one pair.  Slot layout at `base`:
// [0,12) f   [12,18) T   [18,24) line   [24,28) Q (xQ, yQ)   [28,30) P (xP, yP)
// The caller stores Q and P first.  Same schedule as ssb::miller_loop.
SSB_FN void miller(const ws& w, int base, int lane, int nlanes) {
  const int F = base, T = base + 12, LN = base + 18, Q = base + 24, PP = base + 28;
  set_one12(w, F, lane, nlanes);
  for (int j = lane; j < 6; j += nlanes) w.s[T + j] = (j < 4) ? w.s[Q + j] : ((j == 4) ? fp_one() : fp_zero());
  SSB_WAVE_SYNC();
  bool first = true;
  for (int i = 62; i >= 0; --i) {
    if (!first) run(w, FP12_SQR, F, 0, F, lane, nlanes);
    run(w, MILLER_DBL, T, PP, T, lane, nlanes);     // writes T (6) and the line (6) at T + 6 = LN
    run(w, FP12_MUL_014, F, LN, F, lane, nlanes);
    first = false;
    if ((BLS_X_ABS >> i) & 1ull) {
      run(w, MILLER_ADD, T, Q, T, lane, nlanes);    // B = (xQ, yQ, xP, yP) at Q
      run(w, FP12_MUL_014, F, LN, F, lane, nlanes);
    }
  }
  run(w, FP12_CONJ, F, 0, F, lane, nlanes);
}

}  // namespace wave
}  // namespace ssb
