// ssb_field.h -- BLS12-381 field tower for the MI355X threshold-BLS engine.
//
// Fp: 12 x 32-bit limbs, Montgomery form (R = 2^384), CIOS multiplication on v_mad_u64_u32
// chains; every value is kept fully reduced (< p).  Fr: 8 x 32-bit limbs, R = 2^256.
// Tower: Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3 - (1+u)), Fp12 = Fp6[w]/(w^2 - v).
//
// These replace the blst 0.3.10 field layer the reference calls through lighthouse `bls`
// (SURVEY.md §2, F2): blst_sk_* (src/crypto/impls/blst.rs:19-39) and the Fp/Fp2/Fp12 arithmetic
// inside blst_p2_mult / verify.  The same source compiles for gfx950 (kernels) and, for the
// host-side unit tests and op counter only, for the CPU.
#pragma once
#include <cstdint>
#include "ssb_consts.h"
#include "ssb_exp_chains.h"

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define SSB_INL __host__ __device__ __forceinline__
// Kernel launch bounds: workgroup size n and a minimum of SSB_WAVES_PER_EU waves per SIMD, which
// caps every kernel of the TU (and, through the attributor, its out-of-line callees) at
// 512 / SSB_WAVES_PER_EU registers per lane (VGPR + AGPR).
#ifndef SSB_WAVES_PER_EU
#define SSB_WAVES_PER_EU 1
#endif
#define SSB_LB(n) __attribute__((amdgpu_flat_work_group_size(1, n), amdgpu_waves_per_eu(SSB_WAVES_PER_EU)))
// Throughput kernels with every routine inlined: at most 256 registers per lane (VGPR + AGPR), so
// two waves share each SIMD and hide each other's dependent-chain latency.  Measured on MI355X
// (bench_tools/sg_bench.hip, G2 subgroup check over 262,144 points = 4 waves per SIMD):
// 9.52 ms at one wave per SIMD, 7.10 ms at two.
#ifndef SSB_LB2_WAVES
#define SSB_LB2_WAVES 2
#endif
#define SSB_LB2(n) __attribute__((amdgpu_flat_work_group_size(1, n), amdgpu_waves_per_eu(SSB_LB2_WAVES)))
#ifdef SSB_FN_INLINE  // experiment: every routine inlined (code size explodes; microbenchmarks only)
#define SSB_FN __host__ __device__ __forceinline__
#else
#define SSB_FN __host__ __device__ inline __attribute__((noinline))
#endif
#else
#define SSB_INL inline
#define SSB_FN inline
#endif

#ifdef SSB_OPCOUNT
// Host-only instrumented build (tests/native): counts the algorithmic work per operation.
struct ssb_opcounts { unsigned long long fp_mul, fp_sqr, fr_mul; };
extern ssb_opcounts g_ssb_counts;
#define SSB_CNT(f) (g_ssb_counts.f++)
#else
#define SSB_CNT(f) ((void)0)
#endif

namespace ssb {

// ------------------------------------------------------------------------------------------
// carry helpers (lower to v_add_co_u32 / v_addc_co_u32 / v_sub_co_u32 / v_subb_co_u32)
// ------------------------------------------------------------------------------------------
SSB_INL uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t& cout) {
  return __builtin_addc(a, b, cin, &cout);
}
SSB_INL uint32_t subb(uint32_t a, uint32_t b, uint32_t bin, uint32_t& bout) {
  return __builtin_subc(a, b, bin, &bout);
}

// ------------------------------------------------------------------------------------------
// Generic N-limb Montgomery arithmetic (N = 12 for Fp, 8 for Fr)
// ------------------------------------------------------------------------------------------
template <int N>
SSB_INL void mp_add_mod(uint32_t* r, const uint32_t* a, const uint32_t* b, const uint32_t* m) {
  uint32_t t[N], s[N];
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) t[i] = addc(a[i], b[i], c, c);
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) s[i] = subb(t[i], m[i], br, br);
  // a + b < 2m < 2^(32N): no carry out; keep t if t < m (borrow), else s.
  const bool keep = br != 0;
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = keep ? t[i] : s[i];
}

template <int N>
SSB_INL void mp_sub_mod(uint32_t* r, const uint32_t* a, const uint32_t* b, const uint32_t* m) {
  uint32_t t[N];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) t[i] = subb(a[i], b[i], br, br);
  const uint32_t mask = 0u - br;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = addc(t[i], m[i] & mask, c, c);
}

// CIOS Montgomery product r = a*b/2^(32N) mod m, for m < 2^(32N-2) (no top-word carry).
// The outer loop is kept rolled (b is rotated so every access is a static register index):
// the unrolled 12x12 body inlined at every call site made kernels ~12x larger.
template <int N>
SSB_INL void mp_mont_mul_cios(uint32_t* r, const uint32_t* a, const uint32_t* b_in, const uint32_t* m,
                              uint32_t minv) {
  uint32_t t[N], b[N];
  uint32_t tN = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) { t[j] = 0; b[j] = b_in[j]; }
#pragma nounroll
  for (int i = 0; i < N; ++i) {
    uint32_t carry = 0;
    const uint32_t bi = b[0];
#pragma unroll
    for (int j = 0; j < N - 1; ++j) b[j] = b[j + 1];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      uint64_t s = (uint64_t)a[j] * bi + t[j] + carry;
      t[j] = (uint32_t)s;
      carry = (uint32_t)(s >> 32);
    }
    tN += carry;  // t < 2^(32N) + m*2^32: never overflows 32 bits
    const uint32_t q = t[0] * minv;
    uint64_t s = (uint64_t)q * m[0] + t[0];
    carry = (uint32_t)(s >> 32);
#pragma unroll
    for (int j = 1; j < N; ++j) {
      s = (uint64_t)q * m[j] + t[j] + carry;
      t[j - 1] = (uint32_t)s;
      carry = (uint32_t)(s >> 32);
    }
    s = (uint64_t)tN + carry;
    t[N - 1] = (uint32_t)s;
    tN = (uint32_t)(s >> 32);
  }
  // t < 2m: conditional subtraction
  uint32_t s2[N];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) s2[i] = subb(t[i], m[i], br, br);
  const bool keep = (br != 0) && (tN == 0);
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = keep ? t[i] : s2[i];
}

#if defined(__HIP_DEVICE_COMPILE__)
// (acc, top) += x * y : one v_mad_u64_u32 with its carry-out captured by v_addc into `top`.
#define SSB_MAC(acc, top, x, y)                                                        \
  do {                                                                                 \
    uint64_t c_;                                                                       \
    asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32_e64 %2, %1, 0, %2, %1"      \
        : "+v"(acc), "=&s"(c_), "+v"(top) : "v"(x), "v"(y));                           \
  } while (0)
#define SSB_MACS(acc, top, x, y)                                                       \
  do {                                                                                 \
    uint64_t c_;                                                                       \
    asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32_e64 %2, %1, 0, %2, %1"      \
        : "+v"(acc), "=&s"(c_), "+v"(top) : "v"(x), "s"(y));                           \
  } while (0)
// four MACs into the same accumulator in ONE asm statement (one hipcc boundary pad per 4)
#define SSB_MAC_STEP(X, Y) "v_mad_u64_u32 %0, %1, " X ", " Y ", %0\n\tv_addc_co_u32_e64 %2, %1, 0, %2, %1\n\t"
#define SSB_MAC4(CX, CY, acc, top, x0, y0, x1, y1, x2, y2, x3, y3)                     \
  do {                                                                                 \
    uint64_t c_;                                                                       \
    asm(SSB_MAC_STEP("%3", "%4") SSB_MAC_STEP("%5", "%6") SSB_MAC_STEP("%7", "%8")      \
        SSB_MAC_STEP("%9", "%10")                                                      \
        : "+v"(acc), "=&s"(c_), "+v"(top)                                              \
        : CX(x0), CY(y0), CX(x1), CY(y1), CX(x2), CY(y2), CX(x3), CY(y3));             \
  } while (0)
#define SSB_MAC2(CX, CY, acc, top, x0, y0, x1, y1)                                     \
  do {                                                                                 \
    uint64_t c_;                                                                       \
    asm(SSB_MAC_STEP("%3", "%4") SSB_MAC_STEP("%5", "%6")                              \
        : "+v"(acc), "=&s"(c_), "+v"(top) : CX(x0), CY(y0), CX(x1), CY(y1));           \
  } while (0)
// two independent accumulator chains interleaved instruction by instruction (ILP 2 in one wave)
#define SSB_MAC2X2(CX, CY, a0, t0, a1, t1, x0, y0, x1, y1, x2, y2, x3, y3)               \
  do {                                                                                 \
    uint64_t c0_, c1_;                                                                 \
    asm("v_mad_u64_u32 %0, %2, %6, %7, %0\n\tv_mad_u64_u32 %3, %5, %8, %9, %3\n\t"      \
        "v_addc_co_u32_e64 %1, %2, 0, %1, %2\n\tv_addc_co_u32_e64 %4, %5, 0, %4, %5\n\t"  \
        "v_mad_u64_u32 %0, %2, %10, %11, %0\n\tv_mad_u64_u32 %3, %5, %12, %13, %3\n\t"    \
        "v_addc_co_u32_e64 %1, %2, 0, %1, %2\n\tv_addc_co_u32_e64 %4, %5, 0, %4, %5"       \
        : "+v"(a0), "+v"(t0), "=&s"(c0_), "+v"(a1), "+v"(t1), "=&s"(c1_)                 \
        : CX(x0), CY(y0), CX(x1), CY(y1), CX(x2), CY(y2), CX(x3), CY(y3));             \
  } while (0)
#define SSB_V(x) "v"(x)
#define SSB_S(x) "s"(x)
#else
#define SSB_MAC(acc, top, x, y)                                                        \
  do {                                                                                 \
    unsigned __int128 s_ = (unsigned __int128)(uint64_t)(x) * (uint32_t)(y) + (acc);   \
    acc = (uint64_t)s_; top += (uint32_t)(s_ >> 64);                                   \
  } while (0)
#define SSB_MACS SSB_MAC
#define SSB_MAC4(CX, CY, acc, top, x0, y0, x1, y1, x2, y2, x3, y3)                     \
  do { SSB_MAC(acc, top, x0, y0); SSB_MAC(acc, top, x1, y1);                           \
       SSB_MAC(acc, top, x2, y2); SSB_MAC(acc, top, x3, y3); } while (0)
#define SSB_MAC2(CX, CY, acc, top, x0, y0, x1, y1)                                     \
  do { SSB_MAC(acc, top, x0, y0); SSB_MAC(acc, top, x1, y1); } while (0)
#define SSB_MAC2X2(CX, CY, a0, t0, a1, t1, x0, y0, x1, y1, x2, y2, x3, y3)               \
  do { SSB_MAC(a0, t0, x0, y0); SSB_MAC(a1, t1, x1, y1);                               \
       SSB_MAC(a0, t0, x2, y2); SSB_MAC(a1, t1, x3, y3); } while (0)
#endif

// Montgomery product by product scanning (FIPS): column k accumulates every a_j*b_{k-j} and
// m_j*p_{k-j} into a 96-bit (acc, top) accumulator -- one v_mad_u64_u32 + one v_addc per
// limb product -- then either fixes m_k (k < N) or emits r_{k-N}.  Fully unrolled.
// Inputs < m < 2^(32N-2); output fully reduced.
template <int N>
SSB_INL void mp_mont_mul_fips(uint32_t* r, const uint32_t* a, const uint32_t* b, const uint32_t* mod,
                              uint32_t minv) {
  uint32_t m[N], t[N];
  uint64_t acc = 0;
  uint32_t top = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; ++k) {
#pragma unroll
    for (int j = 0; j < N; ++j)
      if (k - j >= 0 && k - j < N) SSB_MAC(acc, top, a[j], b[k - j]);
#pragma unroll
    for (int j = 0; j < N; ++j)
      if (j < k && k - j < N) SSB_MACS(acc, top, m[j], mod[k - j]);
    if (k < N) {
      m[k] = (uint32_t)acc * minv;
      SSB_MACS(acc, top, m[k], mod[0]);  // low word becomes 0
    } else {
      t[k - N] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
  t[N - 1] = (uint32_t)acc;  // acc < 2^32 here since the result < 2m < 2^(32N)
  uint32_t s2[N];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) s2[i] = subb(t[i], mod[i], br, br);
  const bool keep = br != 0;
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = keep ? t[i] : s2[i];
}

// Same product, two interleaved accumulators per column (even / odd j): consecutive MACs touch
// different registers, which removes hipcc's post-asm wait-state pad and doubles the ILP.
template <int N>
SSB_INL void mp_mont_mul_fips2(uint32_t* r, const uint32_t* a, const uint32_t* b, const uint32_t* mod,
                               uint32_t minv) {
  uint32_t m[N], t[N];
  uint64_t acc0 = 0, acc1 = 0;
  uint32_t top0 = 0, top1 = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; ++k) {
    int q = 0;
#pragma unroll
    for (int j = 0; j < N; ++j)
      if (k - j >= 0 && k - j < N) {
        if (q++ & 1) SSB_MAC(acc1, top1, a[j], b[k - j]); else SSB_MAC(acc0, top0, a[j], b[k - j]);
      }
#pragma unroll
    for (int j = 0; j < N; ++j)
      if (j < k && k - j < N) {
        if (q++ & 1) SSB_MACS(acc1, top1, m[j], mod[k - j]); else SSB_MACS(acc0, top0, m[j], mod[k - j]);
      }
    // merge: (acc0, top0) += (acc1, top1)
    {
      uint32_t lo = (uint32_t)acc0, hi = (uint32_t)(acc0 >> 32), c;
      lo = addc(lo, (uint32_t)acc1, 0u, c);
      hi = addc(hi, (uint32_t)(acc1 >> 32), c, c);
      top0 = top0 + top1 + c;
      acc0 = ((uint64_t)hi << 32) | lo;
      acc1 = 0; top1 = 0;
    }
    if (k < N) {
      m[k] = (uint32_t)acc0 * minv;
      SSB_MACS(acc0, top0, m[k], mod[0]);  // low word becomes 0
    } else {
      t[k - N] = (uint32_t)acc0;
    }
    acc0 = (acc0 >> 32) | ((uint64_t)top0 << 32);
    top0 = 0;
  }
  t[N - 1] = (uint32_t)acc0;
  uint32_t s2[N];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) s2[i] = subb(t[i], mod[i], br, br);
  const bool keep = br != 0;
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = keep ? t[i] : s2[i];
}

// FIPS with the column MACs issued four per asm statement.
template <int N>
SSB_INL void mp_mont_mul_fips4(uint32_t* r, const uint32_t* a, const uint32_t* b, const uint32_t* mod,
                               uint32_t minv) {
  uint32_t m[N], t[N];
  uint64_t acc = 0;
  uint32_t top = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; ++k) {
    const int jlo = k - (N - 1) > 0 ? k - (N - 1) : 0;
    const int jhi = k < N - 1 ? k : N - 1;  // a_j b_{k-j}, j in [jlo, jhi]
#pragma unroll
    for (int j = jlo; j <= jhi; j += 4) {
      const int left = jhi - j + 1;
      if (left >= 4) SSB_MAC4(SSB_V, SSB_V, acc, top, a[j], b[k - j], a[j + 1], b[k - j - 1], a[j + 2], b[k - j - 2], a[j + 3], b[k - j - 3]);
      else if (left >= 2) { SSB_MAC2(SSB_V, SSB_V, acc, top, a[j], b[k - j], a[j + 1], b[k - j - 1]); if (left == 3) SSB_MAC(acc, top, a[j + 2], b[k - j - 2]); }
      else SSB_MAC(acc, top, a[j], b[k - j]);
    }
    const int mhi = k - 1 < N - 1 ? k - 1 : N - 1;  // m_j p_{k-j}, j in [jlo, min(k-1, N-1)]
#pragma unroll
    for (int j = jlo; j <= mhi; j += 4) {
      const int left = mhi - j + 1;
      if (left >= 4) SSB_MAC4(SSB_V, SSB_S, acc, top, m[j], mod[k - j], m[j + 1], mod[k - j - 1], m[j + 2], mod[k - j - 2], m[j + 3], mod[k - j - 3]);
      else if (left >= 2) { SSB_MAC2(SSB_V, SSB_S, acc, top, m[j], mod[k - j], m[j + 1], mod[k - j - 1]); if (left == 3) SSB_MACS(acc, top, m[j + 2], mod[k - j - 2]); }
      else SSB_MACS(acc, top, m[j], mod[k - j]);
    }
    if (k < N) {
      m[k] = (uint32_t)acc * minv;
      SSB_MACS(acc, top, m[k], mod[0]);  // low word becomes 0
    } else {
      t[k - N] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
  t[N - 1] = (uint32_t)acc;
  uint32_t s2[N];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) s2[i] = subb(t[i], mod[i], br, br);
  const bool keep = br != 0;
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = keep ? t[i] : s2[i];
}

// r = (a*b + c*d) / 2^(32N) mod m: the FIPS product with BOTH products summed into each column
// before the column's reduction MACs -- one Montgomery reduction for a sum of two products (lazy
// reduction).  Inputs a, b, c < m and d <= m: a*b + c*d < 2 m^2 < m 2^(32N), so the result is < 2m
// before the final conditional subtraction; a column holds at most 3N products, (acc, top) 96 bits.
// The columns are generated by template recursion (a plain unrolled loop of this size is not
// unrolled by the compiler, and the limb arrays then go to scratch).
template <int N, int K>
struct mont2_col {
  SSB_INL static void run(uint32_t* m, uint32_t* t, uint64_t& acc, uint32_t& top, const uint32_t* a, const uint32_t* b,
                          const uint32_t* c, const uint32_t* d, const uint32_t* mod, uint32_t minv) {
    constexpr int jlo = K - (N - 1) > 0 ? K - (N - 1) : 0;
    constexpr int jhi = K < N - 1 ? K : N - 1;
    constexpr int mhi = K - 1 < N - 1 ? K - 1 : N - 1;
#pragma unroll
    for (int j = jlo; j <= jhi; j += 4) {
      const int left = jhi - j + 1;
      if (left >= 4) SSB_MAC4(SSB_V, SSB_V, acc, top, a[j], b[K - j], a[j + 1], b[K - j - 1], a[j + 2], b[K - j - 2], a[j + 3], b[K - j - 3]);
      else if (left >= 2) { SSB_MAC2(SSB_V, SSB_V, acc, top, a[j], b[K - j], a[j + 1], b[K - j - 1]); if (left == 3) SSB_MAC(acc, top, a[j + 2], b[K - j - 2]); }
      else SSB_MAC(acc, top, a[j], b[K - j]);
    }
#pragma unroll
    for (int j = jlo; j <= jhi; j += 4) {
      const int left = jhi - j + 1;
      if (left >= 4) SSB_MAC4(SSB_V, SSB_V, acc, top, c[j], d[K - j], c[j + 1], d[K - j - 1], c[j + 2], d[K - j - 2], c[j + 3], d[K - j - 3]);
      else if (left >= 2) { SSB_MAC2(SSB_V, SSB_V, acc, top, c[j], d[K - j], c[j + 1], d[K - j - 1]); if (left == 3) SSB_MAC(acc, top, c[j + 2], d[K - j - 2]); }
      else SSB_MAC(acc, top, c[j], d[K - j]);
    }
#pragma unroll
    for (int j = jlo; j <= mhi; j += 4) {
      const int left = mhi - j + 1;
      if (left >= 4) SSB_MAC4(SSB_V, SSB_S, acc, top, m[j], mod[K - j], m[j + 1], mod[K - j - 1], m[j + 2], mod[K - j - 2], m[j + 3], mod[K - j - 3]);
      else if (left >= 2) { SSB_MAC2(SSB_V, SSB_S, acc, top, m[j], mod[K - j], m[j + 1], mod[K - j - 1]); if (left == 3) SSB_MACS(acc, top, m[j + 2], mod[K - j - 2]); }
      else SSB_MACS(acc, top, m[j], mod[K - j]);
    }
    if (K < N) {
      m[K < N ? K : 0] = (uint32_t)acc * minv;
      SSB_MACS(acc, top, m[K < N ? K : 0], mod[0]);  // low word becomes 0
    } else {
      t[K >= N ? K - N : 0] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
    mont2_col<N, K + 1>::run(m, t, acc, top, a, b, c, d, mod, minv);
  }
};
template <int N>
struct mont2_col<N, 2 * N - 1> {
  SSB_INL static void run(uint32_t*, uint32_t*, uint64_t&, uint32_t&, const uint32_t*, const uint32_t*, const uint32_t*,
                          const uint32_t*, const uint32_t*, uint32_t) {}
};
template <int N>
SSB_INL void mp_mont_mul2_fips4(uint32_t* r, const uint32_t* a, const uint32_t* b, const uint32_t* c,
                                const uint32_t* d, const uint32_t* mod, uint32_t minv) {
  uint32_t m[N], t[N];
  uint64_t acc = 0;
  uint32_t top = 0;
  mont2_col<N, 0>::run(m, t, acc, top, a, b, c, d, mod, minv);
  t[N - 1] = (uint32_t)acc;
  uint32_t s2[N];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) s2[i] = subb(t[i], mod[i], br, br);
  const bool keep = br != 0;
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = keep ? t[i] : s2[i];
}

// FIPS, two accumulators interleaved inside each asm chunk (halves the dependent chain).
template <int N>
SSB_INL void mp_mont_mul_fips4x2(uint32_t* r, const uint32_t* a, const uint32_t* b, const uint32_t* mod,
                                 uint32_t minv) {
  uint32_t m[N], t[N];
  uint64_t acc = 0, acc1 = 0;
  uint32_t top = 0, top1 = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; ++k) {
    const int jlo = k - (N - 1) > 0 ? k - (N - 1) : 0;
    const int jhi = k < N - 1 ? k : N - 1;
#pragma unroll
    for (int j = jlo; j <= jhi; j += 4) {
      const int left = jhi - j + 1;
      if (left >= 4) SSB_MAC2X2(SSB_V, SSB_V, acc, top, acc1, top1, a[j], b[k - j], a[j + 1], b[k - j - 1], a[j + 2], b[k - j - 2], a[j + 3], b[k - j - 3]);
      else if (left >= 2) { SSB_MAC2(SSB_V, SSB_V, acc1, top1, a[j], b[k - j], a[j + 1], b[k - j - 1]); if (left == 3) SSB_MAC(acc, top, a[j + 2], b[k - j - 2]); }
      else SSB_MAC(acc, top, a[j], b[k - j]);
    }
    const int mhi = k - 1 < N - 1 ? k - 1 : N - 1;
#pragma unroll
    for (int j = jlo; j <= mhi; j += 4) {
      const int left = mhi - j + 1;
      if (left >= 4) SSB_MAC2X2(SSB_V, SSB_S, acc, top, acc1, top1, m[j], mod[k - j], m[j + 1], mod[k - j - 1], m[j + 2], mod[k - j - 2], m[j + 3], mod[k - j - 3]);
      else if (left >= 2) { SSB_MAC2(SSB_V, SSB_S, acc1, top1, m[j], mod[k - j], m[j + 1], mod[k - j - 1]); if (left == 3) SSB_MACS(acc, top, m[j + 2], mod[k - j - 2]); }
      else SSB_MACS(acc, top, m[j], mod[k - j]);
    }
    {  // merge the second chain
      uint32_t lo = (uint32_t)acc, hi = (uint32_t)(acc >> 32), c;
      lo = addc(lo, (uint32_t)acc1, 0u, c);
      hi = addc(hi, (uint32_t)(acc1 >> 32), c, c);
      top = top + top1 + c;
      acc = ((uint64_t)hi << 32) | lo;
      acc1 = 0; top1 = 0;
    }
    if (k < N) {
      m[k] = (uint32_t)acc * minv;
      SSB_MACS(acc, top, m[k], mod[0]);
    } else {
      t[k - N] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
  t[N - 1] = (uint32_t)acc;
  uint32_t s2[N];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) s2[i] = subb(t[i], mod[i], br, br);
  const bool keep = br != 0;
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = keep ? t[i] : s2[i];
}

// The engine's Montgomery product: FIPS with 4-MAC asm chunks.  Measured on MI355X
// (bench_tools/fpmul_bench.hip, profiles/r01_fpmul_variants.json): 1.66x the throughput and
// 0.55x the single-wave latency of the CIOS form above, bit-identical results.
template <int N>
SSB_INL void mp_mont_mul(uint32_t* r, const uint32_t* a, const uint32_t* b, const uint32_t* m, uint32_t minv) {
  mp_mont_mul_fips4<N>(r, a, b, m, minv);
}

template <int N>
SSB_INL bool mp_is_zero(const uint32_t* a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) acc |= a[i];
  return acc == 0;
}

template <int N>
SSB_INL bool mp_eq(const uint32_t* a, const uint32_t* b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) acc |= a[i] ^ b[i];
  return acc == 0;
}

// a > b (canonical integers)
template <int N>
SSB_INL bool mp_gt(const uint32_t* a, const uint32_t* b) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) (void)subb(b[i], a[i], br, br);
  return br != 0;  // b - a borrowed  <=>  a > b
}

// ------------------------------------------------------------------------------------------
// Fp
// ------------------------------------------------------------------------------------------
struct alignas(16) fp { uint32_t l[12]; };  // 16-B aligned: ds_read_b128 / dwordx4 moves

SSB_INL fp fp_from_c(const fp_c& c) { fp r; for (int i = 0; i < 12; ++i) r.l[i] = c.l[i]; return r; }
SSB_INL fp fp_zero() { fp r; for (int i = 0; i < 12; ++i) r.l[i] = 0; return r; }
SSB_INL fp fp_one() { fp r; for (int i = 0; i < 12; ++i) r.l[i] = P_ONE[i]; return r; }
SSB_INL bool fp_is_zero(const fp& a) { return mp_is_zero<12>(a.l); }
SSB_INL bool fp_eq(const fp& a, const fp& b) { return mp_eq<12>(a.l, b.l); }
SSB_INL void fp_add(fp& r, const fp& a, const fp& b) { mp_add_mod<12>(r.l, a.l, b.l, P_LIMBS); }
SSB_INL void fp_sub(fp& r, const fp& a, const fp& b) { mp_sub_mod<12>(r.l, a.l, b.l, P_LIMBS); }
SSB_INL void fp_dbl(fp& r, const fp& a) { mp_add_mod<12>(r.l, a.l, a.l, P_LIMBS); }
SSB_INL void fp_neg(fp& r, const fp& a) { fp z = fp_zero(); fp_sub(r, z, a); }
#if defined(SSB_FPMUL_CALL) && SSB_FPMUL_CALL == 2
// experiment: one out-of-line Montgomery product, operands and result in VGPRs (by value)
SSB_FN fp fp_mul_v(fp a, fp b) { fp r; mp_mont_mul<12>(r.l, a.l, b.l, P_LIMBS, P_INV32); return r; }
SSB_INL void fp_mul(fp& r, const fp& a, const fp& b) { SSB_CNT(fp_mul); r = fp_mul_v(a, b); }
SSB_INL void fp_sqr(fp& r, const fp& a) { SSB_CNT(fp_sqr); r = fp_mul_v(a, a); }
#elif defined(SSB_FPMUL_CALL)
SSB_FN void fp_mul_r(fp& r, const fp& a, const fp& b) { mp_mont_mul<12>(r.l, a.l, b.l, P_LIMBS, P_INV32); }
SSB_INL void fp_mul(fp& r, const fp& a, const fp& b) { SSB_CNT(fp_mul); fp_mul_r(r, a, b); }
SSB_INL void fp_sqr(fp& r, const fp& a) { SSB_CNT(fp_sqr); fp_mul_r(r, a, a); }
#else
SSB_INL void fp_mul(fp& r, const fp& a, const fp& b) {
  SSB_CNT(fp_mul);
  mp_mont_mul<12>(r.l, a.l, b.l, P_LIMBS, P_INV32);
}
SSB_INL void fp_sqr(fp& r, const fp& a) {
  SSB_CNT(fp_sqr);
  mp_mont_mul<12>(r.l, a.l, a.l, P_LIMBS, P_INV32);
}
#endif
SSB_INL void fp_cmov(fp& r, const fp& a, bool c) {
  for (int i = 0; i < 12; ++i) r.l[i] = c ? a.l[i] : r.l[i];
}
// canonical integer (< 2^384) -> Montgomery form (reduces mod p)
SSB_INL void fp_to_mont(fp& r, const fp& a) { mp_mont_mul<12>(r.l, a.l, P_R2, P_LIMBS, P_INV32); }
SSB_INL void fp_from_mont(fp& r, const fp& a) {
  uint32_t one[12] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  mp_mont_mul<12>(r.l, a.l, one, P_LIMBS, P_INV32);
}

// a^e for a fixed (wave-uniform) exponent given as 12 LE limbs
SSB_FN void fp_pow(fp& r, const fp& a, const uint32_t* e) {
  fp acc = fp_one();
  bool started = false;
  for (int i = 383; i >= 0; --i) {
    if (started) fp_sqr(acc, acc);
    if ((e[i >> 5] >> (i & 31)) & 1u) {
      if (started) fp_mul(acc, acc, a); else acc = a;
      started = true;
    }
  }
  r = acc;
}
SSB_INL void fp_inv_fermat(fp& r, const fp& a) { fp_pow(r, a, EXP_P_MINUS_2); }  // inv(0) = 0

// a^e for a fixed exponent given as a sliding-window schedule (gen_exp_chains.py): 8 odd powers,
// then per step `sq` squarings and a multiplication by a^digit.  The schedule index is uniform,
// so the table pick is a select chain, not an indexed (scratch) access.
SSB_INL fp fp_pick8(const fp* t, int i) {
  fp r = t[0];
  for (int k = 1; k < 8; ++k) if (i == k) r = t[k];
  return r;
}
// (_inl twins: bodies for the occupancy-2 per-share kernels, which must not call out of line --
// a call's callee-saved registers and frame keep the kernel at one wave per SIMD)
// (the odd powers as eight named values picked by a switch on the uniform digit: as an array indexed
// by it, the compiler kept the table in scratch and every multiplication of the loop reloaded an
// entry from there -- 12 scratch loads per step in each of the decompression's square roots, round 5)
}  // namespace ssb
#include "ssb_f28_field.h"
namespace ssb {
// The square roots' exponentiations run in the reduced radix (ssb_f28_field.h, r28::pow_sw: one
// v_mad_u64_u32 per limb product); SSB_POW_ENGINE=1 builds keep the engine's products (A/B), and the op
// counter counts the engine's form.
SSB_INL void fp_pow_sw_inl(fp& r, const fp& a, const uint8_t* sch, int n) {
#if !defined(SSB_POW_ENGINE) && !defined(SSB_OPCOUNT)
  r28::pow_sw(r, a, sch, n);
  return;
#endif
  fp t0 = a, t1, t2, t3, t4, t5, t6, t7, a2;
  fp_sqr(a2, a);
  fp_mul(t1, t0, a2); fp_mul(t2, t1, a2); fp_mul(t3, t2, a2); fp_mul(t4, t3, a2);
  fp_mul(t5, t4, a2); fp_mul(t6, t5, a2); fp_mul(t7, t6, a2);
  auto pick = [&](int i) -> fp {
    switch (i) {
      case 0: return t0; case 1: return t1; case 2: return t2; case 3: return t3;
      case 4: return t4; case 5: return t5; case 6: return t6; default: return t7;
    }
  };
  fp acc = pick((sch[1] - 1) >> 1);
  for (int s = 1; s < n; ++s) {
    const int sq = sch[2 * s], d = sch[2 * s + 1];
    for (int k = 0; k < sq; ++k) fp_sqr(acc, acc);
    if (d) { const fp m = pick((d - 1) >> 1); fp_mul(acc, acc, m); }
  }
  r = acc;
}
SSB_FN void fp_pow_sw(fp& r, const fp& a, const uint8_t* sch, int n) { fp_pow_sw_inl(r, a, sch, n); }
// INL = false: the power out of line.  The callable square roots and decompression take that form --
// four inline powers put their function past the 128 KB reach of a short branch, and a callable
// function's long branch overwrites its return address (build.py, long_branch_clobbers).
template <bool INL>
SSB_INL void fp_pow_sw_sel(fp& r, const fp& a, const uint8_t* sch, int n) {
  if constexpr (INL) fp_pow_sw_inl(r, a, sch, n); else fp_pow_sw(r, a, sch, n);
}

// Binary extended Euclid (variable time: inputs on this path are public).  For the Montgomery
// form aR it returns (aR)^{-1} * R^3 / R = a^{-1} R.  inv(0) = 0.  About 4x fewer dependent
// instructions than the Fermat chain, which matters on the single-lane inversions of the
// latency-bound stages (to-affine of the RLC sums, SSWU, isogeny, final exponentiation).
template <int N>
SSB_INL void mp_shr1(uint32_t* a) {
#pragma unroll
  for (int i = 0; i < N - 1; ++i) a[i] = (a[i] >> 1) | (a[i + 1] << 31);
  a[N - 1] >>= 1;
}
// x/2 mod p for x < p
SSB_INL void fp_half_mod(uint32_t* x) {
  if (x[0] & 1u) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) x[i] = addc(x[i], P_LIMBS[i], c, c);
    mp_shr1<12>(x);
    x[11] |= c << 31;
  } else {
    mp_shr1<12>(x);
  }
}
SSB_FN void fp_inv_bgcd(fp& r, const fp& a) {
  uint32_t u[12], v[12], x1[12], x2[12];
  for (int i = 0; i < 12; ++i) { u[i] = a.l[i]; v[i] = P_LIMBS[i]; x1[i] = 0; x2[i] = 0; }
  x1[0] = 1;
  if (mp_is_zero<12>(u)) { r = fp_zero(); return; }
  uint32_t one[12] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  while (!mp_eq<12>(u, one) && !mp_eq<12>(v, one)) {
    while (!(u[0] & 1u)) { mp_shr1<12>(u); fp_half_mod(x1); }
    while (!(v[0] & 1u)) { mp_shr1<12>(v); fp_half_mod(x2); }
    if (!mp_gt<12>(v, u)) {  // u >= v
      uint32_t br = 0;
      for (int i = 0; i < 12; ++i) u[i] = subb(u[i], v[i], br, br);
      mp_sub_mod<12>(x1, x1, x2, P_LIMBS);
    } else {
      uint32_t br = 0;
      for (int i = 0; i < 12; ++i) v[i] = subb(v[i], u[i], br, br);
      mp_sub_mod<12>(x2, x2, x1, P_LIMBS);
    }
  }
  fp t;
  for (int i = 0; i < 12; ++i) t.l[i] = mp_eq<12>(u, one) ? x1[i] : x2[i];
  mp_mont_mul<12>(r.l, t.l, P_R3, P_LIMBS, P_INV32);
}

// ---- Bernstein-Yang "safegcd" inversion (variable time; every input on this path is public) ----
// The binary Euclid above branches per bit, so the 64 lanes of a wave (distinct inputs) diverge:
// measured on MI355X (bench_tools/inv_bench.hip) 734 us per inversion per wave -- one inversion
// was ~0.75 ms of every latency-bound stage that ends in to-affine.  Here the work is batches of
// 30 "divsteps" on the low 30 bits of (f, g) with branch-free selects, each batch folded into the
// full-width values as one 2x2 matrix of int32 entries (|u| + |v| <= 2^30), applied with
// v_mad_i64_i32 over 13 signed 30-bit limbs.  At most 1101 divsteps are needed for 381-bit inputs
// ((49 d + 57) / 17), so 37 batches always suffice; a lane whose g reached 0 stops early.
//   invariant: f = d x (mod p), g = e x (mod p); start f = p, g = x, d = 0, e = 1, delta = 1;
//   end: g = 0, f = +-1, so x^-1 = +-d.
struct s30 { int32_t v[13]; };
constexpr uint32_t SG_M30 = 0x3fffffffu;
struct sg_tables { int32_t pk[7][13]; };   // 2^j p, j = 0..6, as 13 x 30-bit limbs
constexpr sg_tables make_sg_tables() {
  sg_tables t{};
  for (int j = 0; j < 7; ++j)
    for (int l = 0; l < 13; ++l) {
      uint32_t v = 0;
      for (int b = 0; b < 30; ++b) {
        const int bit = 30 * l + b - j;                       // bit of p feeding bit 30 l + b of 2^j p
        if (bit >= 0 && bit < 384 && ((P_LIMBS[bit >> 5] >> (bit & 31)) & 1u)) v |= 1u << b;
      }
      t.pk[j][l] = (int32_t)v;
    }
  return t;
}
constexpr sg_tables SG_T = make_sg_tables();

SSB_INL void s30_from_u32(s30& r, const uint32_t* l) {
  uint64_t acc = 0;
  int bits = 0, k = 0;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    if (bits < 30 && k < 12) { acc |= (uint64_t)l[k++] << bits; bits += 32; }
    r.v[i] = (int32_t)(acc & SG_M30);
    acc >>= 30; bits -= 30;
  }
}
// a non-negative s30 value < 2^384 -> 12 x 32-bit limbs
SSB_INL void s30_to_u32(uint32_t* l, const s30& a) {
  uint64_t acc = 0;
  int bits = 0, k = 0;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    acc |= (uint64_t)(uint32_t)a.v[i] << bits; bits += 30;
    if (bits >= 32 && k < 12) { l[k++] = (uint32_t)acc; acc >>= 32; bits -= 32; }
  }
}
// 30 divsteps on the low bits; returns the new delta and the transition matrix (scaled by 2^30)
SSB_INL int32_t sg_divsteps30(int32_t delta, uint32_t f, uint32_t g, int32_t& u, int32_t& v, int32_t& q, int32_t& r) {
  int32_t uu = 1, vv = 0, qq = 0, rr = 1;
#pragma unroll
  for (int i = 0; i < 30; ++i) {
    const bool odd = (g & 1u) != 0;
    const bool sw = odd && delta > 0;
    // swap:  (f, g) <- (g, (g - f)/2),  (u, v) <- 2(q, r), (q, r) <- (q - u, r - v), delta <- 1 - delta
    // odd:   g <- (g + f)/2,            (u, v) <- 2(u, v), (q, r) <- (q + u, r + v), delta <- 1 + delta
    // even:  g <- g/2,                  (u, v) <- 2(u, v),                           delta <- 1 + delta
    const uint32_t gs = sw ? g - f : (odd ? g + f : g);
    const int32_t qs = sw ? qq - uu : (odd ? qq + uu : qq);
    const int32_t rs = sw ? rr - vv : (odd ? rr + vv : rr);
    const int32_t us = sw ? qq : uu, vs = sw ? rr : vv;
    f = sw ? g : f;
    delta = (sw ? -delta : delta) + 1;
    g = gs >> 1;
    uu = us * 2; vv = vs * 2; qq = qs; rr = rs;
  }
  u = uu; v = vv; q = qq; r = rr;
  return delta;
}
// (f, g) <- (u f + v g, q f + r g) / 2^30  (exact)
SSB_INL void sg_update_fg(s30& f, s30& g, int32_t u, int32_t v, int32_t q, int32_t r) {
  int64_t cf = (int64_t)u * f.v[0] + (int64_t)v * g.v[0];
  int64_t cg = (int64_t)q * f.v[0] + (int64_t)r * g.v[0];
  cf >>= 30; cg >>= 30;
#pragma unroll
  for (int i = 1; i < 13; ++i) {
    cf += (int64_t)u * f.v[i] + (int64_t)v * g.v[i];
    cg += (int64_t)q * f.v[i] + (int64_t)r * g.v[i];
    f.v[i - 1] = (int32_t)((uint32_t)cf & SG_M30);
    g.v[i - 1] = (int32_t)((uint32_t)cg & SG_M30);
    cf >>= 30; cg >>= 30;
  }
  f.v[12] = (int32_t)cf; g.v[12] = (int32_t)cg;
}
// (d, e) <- (u d + v e + md p, q d + r e + me p) / 2^30, md / me in [0, 2^30) chosen so the
// divisions are exact (P_INV32 = -p^-1 mod 2^32).  |d'| <= max(|d|, |e|) + p.
SSB_INL void sg_update_de(s30& d, s30& e, int32_t u, int32_t v, int32_t q, int32_t r) {
  const uint32_t dl = (uint32_t)u * (uint32_t)d.v[0] + (uint32_t)v * (uint32_t)e.v[0];
  const uint32_t el = (uint32_t)q * (uint32_t)d.v[0] + (uint32_t)r * (uint32_t)e.v[0];
  const int32_t md = (int32_t)((dl * P_INV32) & SG_M30), me = (int32_t)((el * P_INV32) & SG_M30);
  int64_t cd = (int64_t)u * d.v[0] + (int64_t)v * e.v[0] + (int64_t)md * SG_T.pk[0][0];
  int64_t ce = (int64_t)q * d.v[0] + (int64_t)r * e.v[0] + (int64_t)me * SG_T.pk[0][0];
  cd >>= 30; ce >>= 30;
#pragma unroll
  for (int i = 1; i < 13; ++i) {
    cd += (int64_t)u * d.v[i] + (int64_t)v * e.v[i] + (int64_t)md * SG_T.pk[0][i];
    ce += (int64_t)q * d.v[i] + (int64_t)r * e.v[i] + (int64_t)me * SG_T.pk[0][i];
    d.v[i - 1] = (int32_t)((uint32_t)cd & SG_M30);
    e.v[i - 1] = (int32_t)((uint32_t)ce & SG_M30);
    cd >>= 30; ce >>= 30;
  }
  d.v[12] = (int32_t)cd; e.v[12] = (int32_t)ce;
}
// r = a + s * b (s = +-1 or 0), limbs renormalised
SSB_INL void s30_addmul(s30& r, const s30& a, const int32_t* b, int32_t s) {
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    c += (int64_t)a.v[i] + (int64_t)s * b[i];
    r.v[i] = (int32_t)((uint32_t)c & SG_M30);
    c >>= 30;
  }
  r.v[12] = (int32_t)(c + (int64_t)a.v[12] + (int64_t)s * b[12]);
}
SSB_FN void fp_inv(fp& r, const fp& a) {
  if (mp_is_zero<12>(a.l)) { r = fp_zero(); return; }      // inv(0) = 0, as blst
  s30 f, g, d, e;
#pragma unroll
  for (int i = 0; i < 13; ++i) { f.v[i] = SG_T.pk[0][i]; d.v[i] = 0; e.v[i] = 0; }
  e.v[0] = 1;
  s30_from_u32(g, a.l);
  int32_t delta = 1;
  for (int it = 0; it < 37; ++it) {
    int32_t any = 0;
#pragma unroll
    for (int i = 0; i < 13; ++i) any |= g.v[i];
    if (!any) break;
    int32_t u, v, q, w;
    delta = sg_divsteps30(delta, (uint32_t)f.v[0], (uint32_t)g.v[0], u, v, q, w);
    sg_update_de(d, e, u, v, q, w);
    sg_update_fg(f, g, u, v, q, w);
  }
  // x^-1 = d * f (f = +-1); |d| <= 37 p: shift into (0, 128 p) with +64 p, then reduce mod p
  s30 zero;
#pragma unroll
  for (int i = 0; i < 13; ++i) zero.v[i] = 0;
  if (f.v[12] < 0) s30_addmul(d, zero, d.v, -1);
  s30_addmul(d, d, SG_T.pk[6], 1);
#pragma unroll
  for (int j = 6; j >= 0; --j) {
    s30 t;
    s30_addmul(t, d, SG_T.pk[j], -1);
    if (t.v[12] >= 0) d = t;
  }
  fp t;
  s30_to_u32(t.l, d);
  mp_mont_mul<12>(r.l, t.l, P_R3, P_LIMBS, P_INV32);        // (aR)^-1 -> a^-1 R
}
// returns true iff a is a square; r = a^((p+1)/4) (a root when it is)
template <bool INL = true>
SSB_INL bool fp_sqrt_inl(fp& r, const fp& a) {
  fp s, s2;
  fp_pow_sw_sel<INL>(s, a, EXPW_P_PLUS_1_DIV_4, EXPW_P_PLUS_1_DIV_4_N);
  fp_sqr(s2, s);
  r = s;
  return fp_eq(s2, a);
}
SSB_FN bool fp_sqrt(fp& r, const fp& a) { return fp_sqrt_inl<false>(r, a); }
// ZCash sign: canonical(a) > (p-1)/2
SSB_INL bool fp_lex_largest(const fp& a) {
  fp c; fp_from_mont(c, a);
  return mp_gt<12>(c.l, P_HALF_CANON);
}
SSB_INL uint32_t fp_parity(const fp& a) { fp c; fp_from_mont(c, a); return c.l[0] & 1u; }

// big-endian 48 bytes -> canonical limbs (no reduction); returns true iff value < p
SSB_INL bool fp_from_be48(fp& r, const uint8_t* b, uint8_t top_mask) {
  for (int i = 0; i < 12; ++i) {
    const uint8_t* q = b + 44 - 4 * i;
    uint32_t v = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
    r.l[i] = v;
  }
  r.l[11] &= ((uint32_t)top_mask << 24) | 0x00ffffffu;
  return mp_gt<12>(P_LIMBS, r.l);
}
SSB_INL void fp_to_be48(uint8_t* b, const fp& canon) {
  for (int i = 0; i < 12; ++i) {
    uint32_t v = canon.l[i];
    uint8_t* q = b + 44 - 4 * i;
    q[0] = (uint8_t)(v >> 24); q[1] = (uint8_t)(v >> 16); q[2] = (uint8_t)(v >> 8); q[3] = (uint8_t)v;
  }
}

// ------------------------------------------------------------------------------------------
// Fr (scalar field), used for the Lagrange coefficients (src/crypto/impls/blst.rs:19-39)
// ------------------------------------------------------------------------------------------
struct fr { uint32_t l[8]; };

SSB_INL fr fr_zero() { fr r; for (int i = 0; i < 8; ++i) r.l[i] = 0; return r; }
SSB_INL fr fr_one() { fr r; for (int i = 0; i < 8; ++i) r.l[i] = R_ONE[i]; return r; }
SSB_INL bool fr_is_zero(const fr& a) { return mp_is_zero<8>(a.l); }
SSB_INL void fr_sub(fr& r, const fr& a, const fr& b) { mp_sub_mod<8>(r.l, a.l, b.l, R_LIMBS); }
SSB_INL void fr_mul(fr& r, const fr& a, const fr& b) {
  SSB_CNT(fr_mul);
  mp_mont_mul<8>(r.l, a.l, b.l, R_LIMBS, R_INV32);
}
// u64 -> Montgomery Fr (blst_scalar_from_uint64, src/utils/blst_utils.rs:15-21); u64 < r always
SSB_INL void fr_from_u64(fr& r, uint64_t v) {
  uint32_t c[8] = {(uint32_t)v, (uint32_t)(v >> 32), 0, 0, 0, 0, 0, 0};
  mp_mont_mul<8>(r.l, c, R_R2, R_LIMBS, R_INV32);
}
SSB_INL void fr_from_mont(fr& r, const fr& a) {
  uint32_t one[8] = {1, 0, 0, 0, 0, 0, 0, 0};
  mp_mont_mul<8>(r.l, a.l, one, R_LIMBS, R_INV32);
}
SSB_FN void fr_inv(fr& r, const fr& a) {  // Fermat; inv(0) = 0 like blst_sk_inverse
  fr acc = fr_one();
  bool started = false;
  for (int i = 255; i >= 0; --i) {
    if (started) fr_mul(acc, acc, acc);
    if ((EXP_R_MINUS_2[i >> 5] >> (i & 31)) & 1u) {
      if (started) fr_mul(acc, acc, a); else acc = a;
      started = true;
    }
  }
  r = acc;
}

// ------------------------------------------------------------------------------------------
// Fp2
// ------------------------------------------------------------------------------------------
struct fp2 { fp c0, c1; };

SSB_INL fp2 fp2_from_c(const fp2_c& c) { fp2 r; r.c0 = fp_from_c(c.c0); r.c1 = fp_from_c(c.c1); return r; }
SSB_INL fp2 fp2_zero() { fp2 r; r.c0 = fp_zero(); r.c1 = fp_zero(); return r; }
SSB_INL fp2 fp2_one() { fp2 r; r.c0 = fp_one(); r.c1 = fp_zero(); return r; }
SSB_INL bool fp2_is_zero(const fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
SSB_INL bool fp2_eq(const fp2& a, const fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
SSB_INL void fp2_add(fp2& r, const fp2& a, const fp2& b) { fp_add(r.c0, a.c0, b.c0); fp_add(r.c1, a.c1, b.c1); }
SSB_INL void fp2_sub(fp2& r, const fp2& a, const fp2& b) { fp_sub(r.c0, a.c0, b.c0); fp_sub(r.c1, a.c1, b.c1); }
SSB_INL void fp2_dbl(fp2& r, const fp2& a) { fp_dbl(r.c0, a.c0); fp_dbl(r.c1, a.c1); }
SSB_INL void fp2_neg(fp2& r, const fp2& a) { fp_neg(r.c0, a.c0); fp_neg(r.c1, a.c1); }
SSB_INL void fp2_conj(fp2& r, const fp2& a) { r.c0 = a.c0; fp_neg(r.c1, a.c1); }
// Schoolbook with lazy reduction: c0 = a0 b0 + a1 (p - b1), c1 = a0 b1 + a1 b0, each ONE Montgomery
// reduction of a sum of two products (mp_mont_mul2_fips4): four products and two reductions, no
// modular additions, instead of Karatsuba's three Montgomery products and five modular additions.
// (Counted as three products, the algorithmic unit of the op counter.)
SSB_INL void fp2_mul(fp2& r, const fp2& a, const fp2& b) {
  SSB_CNT(fp_mul); SSB_CNT(fp_mul); SSB_CNT(fp_mul);
  fp nb1, c0, c1;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) nb1.l[i] = subb(P_LIMBS[i], b.c1.l[i], br, br);   // p - b1 in (0, p]
  mp_mont_mul2_fips4<12>(c0.l, a.c0.l, b.c0.l, a.c1.l, nb1.l, P_LIMBS, P_INV32);
  mp_mont_mul2_fips4<12>(c1.l, a.c0.l, b.c1.l, a.c1.l, b.c0.l, P_LIMBS, P_INV32);
  r.c0 = c0;
  r.c1 = c1;
}
// (a0 + a1)(a0 - a1) with both factors left unreduced (< 2p): the Montgomery product accepts them
// (4p^2 < p 2^384, the result is < 2p before its final subtraction), which saves the two modular
// corrections of the sum and the difference
SSB_INL void fp2_sqr(fp2& r, const fp2& a) {
  fp s, d, m;
  uint32_t c = 0, br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) s.l[i] = addc(a.c0.l[i], a.c1.l[i], c, c);          // a0 + a1 < 2p
#pragma unroll
  for (int i = 0; i < 12; ++i) d.l[i] = subb(P_LIMBS[i], a.c1.l[i], br, br);      // p - a1 in (0, p]
  c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) d.l[i] = addc(d.l[i], a.c0.l[i], c, c);             // a0 - a1 + p < 2p
  fp_mul(m, a.c0, a.c1);
  fp_mul(r.c0, s, d);
  fp_dbl(r.c1, m);
}
SSB_INL void fp2_mul_fp(fp2& r, const fp2& a, const fp& b) { fp_mul(r.c0, a.c0, b); fp_mul(r.c1, a.c1, b); }
// (a0 + a1 u)(1 + u)
SSB_INL void fp2_mul_xi(fp2& r, const fp2& a) {
  fp t0, t1;
  fp_sub(t0, a.c0, a.c1);
  fp_add(t1, a.c0, a.c1);
  r.c0 = t0; r.c1 = t1;
}
SSB_INL void fp2_cmov(fp2& r, const fp2& a, bool c) { fp_cmov(r.c0, a.c0, c); fp_cmov(r.c1, a.c1, c); }
SSB_FN void fp2_inv(fp2& r, const fp2& a) {
  fp t0, t1;
  fp_sqr(t0, a.c0);
  fp_sqr(t1, a.c1);
  fp_add(t0, t0, t1);
  fp_inv(t1, t0);
  fp_mul(r.c0, a.c0, t1);
  fp_mul(t0, a.c1, t1);
  fp_neg(r.c1, t0);
}
// Square root in Fp2 by the norm method (p = 3 mod 4).  Any root is returned; the caller fixes
// the sign.  Returns false iff a is not a square.
template <bool INL = true>
SSB_INL bool fp2_sqrt_inl(fp2& r, const fp2& a) {
  if (fp_is_zero(a.c1)) {
    fp s;
    if (fp_sqrt_inl<INL>(s, a.c0)) { r.c0 = s; r.c1 = fp_zero(); return true; }
    fp na; fp_neg(na, a.c0);
    bool ok = fp_sqrt_inl<INL>(s, na);
    r.c0 = fp_zero(); r.c1 = s;
    return ok;
  }
  fp n, t, s;
  fp_sqr(n, a.c0);
  fp_sqr(t, a.c1);
  fp_add(n, n, t);
  if (!fp_sqrt_inl<INL>(s, n)) return false;
  fp c, half = fp_from_c(FP_HALF);
  fp_add(c, a.c0, s);
  fp_mul(c, c, half);                       // c = (a0 + s)/2  (nonzero since a1 != 0)
  fp_pow_sw_sel<INL>(t, c, EXPW_P_MINUS_3_DIV_4, EXPW_P_MINUS_3_DIV_4_N);  // t = c^((p-3)/4)
  fp x, x2;
  fp_mul(x, c, t);                          // x^2 = c if c is a square, else -c
  fp_sqr(x2, x);
  fp2 y;
  if (fp_eq(x2, c)) {
    y.c0 = x;                               // x0 = sqrt(c), 1/x0 = t
    fp_mul(y.c1, a.c1, t);
    fp_mul(y.c1, y.c1, half);               // x1 = a1 / (2 x0)
  } else {
    fp nt; fp_neg(nt, t);
    fp_mul(y.c0, a.c1, nt);
    fp_mul(y.c0, y.c0, half);               // x0 = a1 / (2 sqrt(-c)) = -a1 t / 2
    y.c1 = x;                               // x1 = sqrt(-c)
  }
  fp2 chk; fp2_sqr(chk, y);
  r = y;
  return fp2_eq(chk, a);
}
SSB_FN bool fp2_sqrt(fp2& r, const fp2& a) { return fp2_sqrt_inl<false>(r, a); }
// ZCash sign for Fp2: c1 > (p-1)/2, or c0 > (p-1)/2 when c1 == 0
SSB_INL bool fp2_lex_largest(const fp2& a) {
  if (!fp_is_zero(a.c1)) return fp_lex_largest(a.c1);
  return fp_lex_largest(a.c0);
}
// RFC 9380 sgn0 for Fp2
SSB_INL uint32_t fp2_sgn0(const fp2& a) {
  fp c0, c1;
  fp_from_mont(c0, a.c0);
  fp_from_mont(c1, a.c1);
  const uint32_t sign0 = c0.l[0] & 1u;
  const uint32_t zero0 = mp_is_zero<12>(c0.l) ? 1u : 0u;
  const uint32_t sign1 = c1.l[0] & 1u;
  return sign0 | (zero0 & sign1);
}

// ------------------------------------------------------------------------------------------
// Fp6
// ------------------------------------------------------------------------------------------
struct fp6 { fp2 c0, c1, c2; };

SSB_INL fp6 fp6_zero() { fp6 r; r.c0 = fp2_zero(); r.c1 = fp2_zero(); r.c2 = fp2_zero(); return r; }
SSB_INL fp6 fp6_one() { fp6 r; r.c0 = fp2_one(); r.c1 = fp2_zero(); r.c2 = fp2_zero(); return r; }
SSB_INL void fp6_add(fp6& r, const fp6& a, const fp6& b) { fp2_add(r.c0, a.c0, b.c0); fp2_add(r.c1, a.c1, b.c1); fp2_add(r.c2, a.c2, b.c2); }
SSB_INL void fp6_sub(fp6& r, const fp6& a, const fp6& b) { fp2_sub(r.c0, a.c0, b.c0); fp2_sub(r.c1, a.c1, b.c1); fp2_sub(r.c2, a.c2, b.c2); }
SSB_INL void fp6_neg(fp6& r, const fp6& a) { fp2_neg(r.c0, a.c0); fp2_neg(r.c1, a.c1); fp2_neg(r.c2, a.c2); }
SSB_INL bool fp6_eq(const fp6& a, const fp6& b) { return fp2_eq(a.c0, b.c0) && fp2_eq(a.c1, b.c1) && fp2_eq(a.c2, b.c2); }
SSB_FN void fp6_mul(fp6& r, const fp6& a, const fp6& b) {
  fp2 t0, t1, t2, s0, s1, u;
  fp2_mul(t0, a.c0, b.c0);
  fp2_mul(t1, a.c1, b.c1);
  fp2_mul(t2, a.c2, b.c2);
  fp6 o;
  // c0 = ((a1+a2)(b1+b2) - t1 - t2) xi + t0
  fp2_add(s0, a.c1, a.c2); fp2_add(s1, b.c1, b.c2); fp2_mul(u, s0, s1);
  fp2_sub(u, u, t1); fp2_sub(u, u, t2); fp2_mul_xi(u, u); fp2_add(o.c0, u, t0);
  // c1 = (a0+a1)(b0+b1) - t0 - t1 + xi t2
  fp2_add(s0, a.c0, a.c1); fp2_add(s1, b.c0, b.c1); fp2_mul(u, s0, s1);
  fp2_sub(u, u, t0); fp2_sub(u, u, t1); fp2 x2; fp2_mul_xi(x2, t2); fp2_add(o.c1, u, x2);
  // c2 = (a0+a2)(b0+b2) - t0 - t2 + t1
  fp2_add(s0, a.c0, a.c2); fp2_add(s1, b.c0, b.c2); fp2_mul(u, s0, s1);
  fp2_sub(u, u, t0); fp2_sub(u, u, t2); fp2_add(o.c2, u, t1);
  r = o;
}
SSB_INL void fp6_mul_v(fp6& r, const fp6& a) {  // * v
  fp2 t; fp2_mul_xi(t, a.c2);
  fp2 a0 = a.c0, a1 = a.c1;
  r.c0 = t; r.c1 = a0; r.c2 = a1;
}
// a * (b0 + b1 v)
SSB_FN void fp6_mul_01(fp6& r, const fp6& a, const fp2& b0, const fp2& b1) {
  fp2 aa, bb, t1, t2, t3, s0, s1;
  fp2_mul(aa, a.c0, b0);
  fp2_mul(bb, a.c1, b1);
  fp2_mul(t1, a.c2, b1); fp2_mul_xi(t1, t1); fp2_add(t1, t1, aa);
  fp2_add(s0, b0, b1); fp2_add(s1, a.c0, a.c1); fp2_mul(t2, s0, s1); fp2_sub(t2, t2, aa); fp2_sub(t2, t2, bb);
  fp2_mul(t3, a.c2, b0); fp2_add(t3, t3, bb);
  r.c0 = t1; r.c1 = t2; r.c2 = t3;
}
// a * (b1 v)
SSB_FN void fp6_mul_1(fp6& r, const fp6& a, const fp2& b1) {
  fp2 t0, t1, t2;
  fp2_mul(t0, a.c2, b1); fp2_mul_xi(t0, t0);
  fp2_mul(t1, a.c0, b1);
  fp2_mul(t2, a.c1, b1);
  r.c0 = t0; r.c1 = t1; r.c2 = t2;
}
SSB_FN void fp6_inv(fp6& r, const fp6& a) {
  fp2 c0, c1, c2, t, u;
  fp2_sqr(c0, a.c0); fp2_mul(t, a.c1, a.c2); fp2_mul_xi(t, t); fp2_sub(c0, c0, t);
  fp2_sqr(c1, a.c2); fp2_mul_xi(c1, c1); fp2_mul(t, a.c0, a.c1); fp2_sub(c1, c1, t);
  fp2_sqr(c2, a.c1); fp2_mul(t, a.c0, a.c2); fp2_sub(c2, c2, t);
  fp2_mul(t, a.c2, c1); fp2_mul(u, a.c1, c2); fp2_add(t, t, u); fp2_mul_xi(t, t);
  fp2_mul(u, a.c0, c0); fp2_add(t, t, u);
  fp2_inv(t, t);
  fp2_mul(r.c0, c0, t); fp2_mul(r.c1, c1, t); fp2_mul(r.c2, c2, t);
}

// ------------------------------------------------------------------------------------------
// Fp12
// ------------------------------------------------------------------------------------------
struct fp12 { fp6 c0, c1; };

SSB_INL fp12 fp12_one() { fp12 r; r.c0 = fp6_one(); r.c1 = fp6_zero(); return r; }
SSB_INL bool fp12_eq(const fp12& a, const fp12& b) { return fp6_eq(a.c0, b.c0) && fp6_eq(a.c1, b.c1); }
SSB_INL bool fp12_is_one(const fp12& a) { fp12 o = fp12_one(); return fp12_eq(a, o); }
SSB_INL void fp12_conj(fp12& r, const fp12& a) { r.c0 = a.c0; fp6_neg(r.c1, a.c1); }
SSB_FN void fp12_mul(fp12& r, const fp12& a, const fp12& b) {
  fp6 t0, t1, s0, s1, c1;
  fp6_mul(t0, a.c0, b.c0);
  fp6_mul(t1, a.c1, b.c1);
  fp6_add(s0, a.c0, a.c1);
  fp6_add(s1, b.c0, b.c1);
  fp6_mul(c1, s0, s1);
  fp6_sub(c1, c1, t0);
  fp6_sub(r.c1, c1, t1);
  fp6_mul_v(t1, t1);
  fp6_add(r.c0, t0, t1);
}
SSB_FN void fp12_sqr(fp12& r, const fp12& a) {
  fp6 ab, s0, s1, t;
  fp6_mul(ab, a.c0, a.c1);
  fp6_add(s0, a.c0, a.c1);
  fp6_mul_v(t, a.c1);
  fp6_add(s1, a.c0, t);
  fp6_mul(s0, s0, s1);
  fp6_sub(s0, s0, ab);
  fp6_mul_v(t, ab);
  fp6_sub(r.c0, s0, t);
  fp6_add(r.c1, ab, ab);
}
SSB_FN void fp12_inv(fp12& r, const fp12& a) {
  fp6 t0, t1;
  fp6_mul(t0, a.c0, a.c0);
  fp6_mul(t1, a.c1, a.c1);
  fp6_mul_v(t1, t1);
  fp6_sub(t0, t0, t1);
  fp6_inv(t1, t0);
  fp6_mul(r.c0, a.c0, t1);
  fp6_mul(t0, a.c1, t1);
  fp6_neg(r.c1, t0);
}
// f * (o0 + o1 v + o4 v w): the sparse line value (positions 0, 1, 4)
SSB_FN void fp12_mul_014(fp12& r, const fp12& f, const fp2& o0, const fp2& o1, const fp2& o4) {
  fp6 aa, bb, s;
  fp6_mul_01(aa, f.c0, o0, o1);
  fp6_mul_1(bb, f.c1, o4);
  fp2 o; fp2_add(o, o1, o4);
  fp6_add(s, f.c1, f.c0);
  fp6_mul_01(s, s, o0, o);
  fp6_sub(s, s, aa);
  fp6_sub(r.c1, s, bb);
  fp6_mul_v(bb, bb);
  fp6_add(r.c0, bb, aa);
}
// Frobenius^n, n = 1, 2, 3: coefficient of w^k -> (conj^n) * xi^(k (p^n-1)/6)
SSB_FN void fp12_frob(fp12& r, const fp12& a, int n) {
  const fp2_c* g = (n == 1) ? FROB1 : (n == 2) ? FROB2 : FROB3;
  fp2 c[6] = {a.c0.c0, a.c1.c0, a.c0.c1, a.c1.c1, a.c0.c2, a.c1.c2};  // w^0..w^5
  for (int k = 0; k < 6; ++k) {
    if (n & 1) fp2_conj(c[k], c[k]);
    if (k) { fp2 gk = fp2_from_c(g[k]); fp2_mul(c[k], c[k], gk); }
  }
  r.c0.c0 = c[0]; r.c1.c0 = c[1]; r.c0.c1 = c[2]; r.c1.c1 = c[3]; r.c0.c2 = c[4]; r.c1.c2 = c[5];
}
// Granger-Scott squaring in the cyclotomic subgroup
SSB_INL void fp4_sqr(fp2& c0, fp2& c1, const fp2& a, const fp2& b) {
  fp2 t0, t1, t2;
  fp2_sqr(t0, a);
  fp2_sqr(t1, b);
  fp2_mul_xi(t2, t1);
  fp2_add(c0, t2, t0);
  fp2_add(t2, a, b);
  fp2_sqr(t2, t2);
  fp2_sub(t2, t2, t0);
  fp2_sub(c1, t2, t1);
}
SSB_FN void fp12_cyc_sqr(fp12& r, const fp12& f) {
  fp2 z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2, z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
  fp2 t0, t1, t2, t3;
  fp4_sqr(t0, t1, z0, z1);
  fp2_sub(z0, t0, z0); fp2_dbl(z0, z0); fp2_add(z0, z0, t0);
  fp2_add(z1, t1, z1); fp2_dbl(z1, z1); fp2_add(z1, z1, t1);
  fp4_sqr(t0, t1, z2, z3);
  fp4_sqr(t2, t3, z4, z5);
  fp2_sub(z4, t0, z4); fp2_dbl(z4, z4); fp2_add(z4, z4, t0);
  fp2_add(z5, t1, z5); fp2_dbl(z5, z5); fp2_add(z5, z5, t1);
  fp2_mul_xi(t0, t3);
  fp2_add(z2, t0, z2); fp2_dbl(z2, z2); fp2_add(z2, z2, t0);
  fp2_sub(z3, t2, z3); fp2_dbl(z3, z3); fp2_add(z3, z3, t2);
  r.c0.c0 = z0; r.c0.c1 = z4; r.c0.c2 = z3; r.c1.c0 = z2; r.c1.c1 = z1; r.c1.c2 = z5;
}
// f^x for x = -0xd201000000010000 (f in the cyclotomic subgroup)
SSB_FN void fp12_cyc_exp_x(fp12& r, const fp12& f) {
  fp12 acc = f;
  for (int i = 62; i >= 0; --i) {
    fp12_cyc_sqr(acc, acc);
    if ((BLS_X_ABS >> i) & 1ull) fp12_mul(acc, acc, f);
  }
  fp12_conj(r, acc);
}

}  // namespace ssb
