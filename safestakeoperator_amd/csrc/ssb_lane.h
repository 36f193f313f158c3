// ssb_lane.h -- runtime of the lane-group programs generated into ssb_lane_progs.h.
//
// A program runs one point / tower operation on a GROUP of G lanes: in every product round each
// lane ("role") computes one Fp Montgomery product whose operands are short +-sums of LDS slots;
// in every linear stage some lanes materialise longer forms (reduced mod p) into slots.  The
// 64/G groups of a wave run independent operations in lockstep.  Slot codes (8 bit) select:
//   0..47    shared constants of the workgroup (0 = zero)          -> g.k[code]
//   48..447  the group's scratch                                    -> g.s[code - 48]
//   448..479 input A, 480..511 input B, 512..543 output D          -> g.s[g.a/b/d + ...]
// (A, B, D are group-relative slot indices chosen by the caller, beyond the scratch area.)
//
// Values in slots are fully reduced (< p).  A product operand of up to 3 terms is formed WITHOUT
// reduction (negative terms enter as p - v, so the value is <= 3p); 3p * 3p < p * 2^384 keeps the
// Montgomery product's output < 2p before its final conditional subtraction, so fp_mul accepts
// it.  Materialised forms have up to 8 terms (<= 8p < 2^384) and are reduced by conditional
// subtraction of 4p, 2p, p, p.
//
// The same source runs on the host (tests): LP_FOR loops over the roles of one group, and the
// stores of a pass happen after every role computed, like the lockstep lanes of a wave.
#pragma once
#include "ssb_curve.h"

namespace ssb {
namespace lane {

constexpr int LP_NCODE_CONST = 48, LP_NSCRATCH = 400;

// LDS pointers carry address space 3 on the device, so slot traffic is ds_read/ds_write_b128
// (generic pointers would compile to flat_* accesses).
#if defined(__HIP_DEVICE_COMPILE__)
#define SSB_LDS __attribute__((address_space(3)))
#else
#define SSB_LDS
#endif
typedef SSB_LDS fp lfp;
typedef SSB_LDS uint32_t lu32;

struct grp {       // passed BY VALUE to the programs (lives in registers)
  lfp* k;          // shared constants (LP_NCODE_CONST slots)
  lfp* s;          // this group's slots: [0, scratch) program scratch, then caller-owned
  int a, b, d;     // group-relative slot index of input A, input B, output D
  lu32* flag;      // this group's check word (bit per check component)
  int role;        // lane index inside the group (device)
};

#if (defined(__HIPCC__) || defined(__HIP__)) && defined(SSB_LP_INLINE)
#define SSB_LP_FN __host__ __device__ __forceinline__
#elif defined(__HIPCC__) || defined(__HIP__)
#define SSB_LP_FN __host__ __device__ __noinline__
#else
#define SSB_LP_FN inline
#endif
#define SSB_LP_TABLE alignas(16) constexpr
#if defined(__HIP_DEVICE_COMPILE__)
#define LP_DECL_T fp T_
#define LP_FOR(G) for (int role = g.role, once_ = 1; once_; once_ = 0)
#define LP_T T_
#define LP_SYNC() __syncthreads()
#define LP_FOR_ALL_CONSTS(i) for (int i = threadIdx.x; i < LP_NCODE_CONST; i += blockDim.x)
#else
#define LP_DECL_T fp T_[64]
#define LP_FOR(G) for (int role = 0; role < (G); ++role)
#define LP_T T_[role]
#define LP_SYNC() ((void)0)
#define LP_FOR_ALL_CONSTS(i) for (int i = 0; i < LP_NCODE_CONST; ++i)
#endif

#define LP_SEL8(imm) ((uint32_t)((imm) >> (8 * role)) & 0xffu)
#define LP_SEL16(imm) ((uint32_t)((imm) >> (16 * role)) & 0xffffu)
#define LP_SEL16X2(lo, hi) ((uint32_t)((role < 4 ? (lo) : (hi)) >> (16 * (role & 3))) & 0xffffu)
#define LP_SELT(tab) ((uint32_t)(tab)[role])
// Per-stage code rows of the G = 64 programs: tab[role * nw .. + nw) holds the lane's 16-bit codes of
// one stage, two per word.  The device loads its row once at the top of the stage (nw / 4 16-byte
// loads, one memory round trip); the host reads the table directly inside its role loop.
#if defined(__HIP_DEVICE_COMPILE__)
#define LP_CODES(tab, nw) lp_u4c cw_[(nw) / 4]; lp_load_codes<(nw) / 4>(cw_, (tab) + (size_t)g.role * (nw))
#define LP_CW(tab, nw, i) ((cw_[(i) / 8][((i) / 2) & 3] >> (16 * ((i) & 1))) & 0xffffu)
#else
#define LP_CODES(tab, nw) ((void)0)
#define LP_CW(tab, nw, i) (((uint32_t)(tab)[role * (nw) + (i) / 2] >> (16 * ((i) & 1))) & 0xffffu)
#endif
#define LP_BIT(imm) ((uint32_t)((imm) >> role) & 1u)

SSB_INL lfp* lp_ptr(const grp& g, uint32_t c) {
  const int base = c >= 512u ? g.d - 512 : (c >= 480u ? g.b - 480 : (c >= 448u ? g.a - 448 : -48));
  return c < (uint32_t)LP_NCODE_CONST ? g.k + c : g.s + ((int)c + base);
}
// Slot moves as three 16-byte LDS accesses (ds_read_b128 / ds_write_b128): through a computed slot
// pointer the compiler no longer sees fp's 16-byte alignment and splits a plain struct copy into
// ds_read2_b32 pairs (six per slot, each a separate LDS round trip when its limbs are consumed).
#if defined(__HIP_DEVICE_COMPILE__)
typedef uint32_t lp_u4 __attribute__((ext_vector_type(4)));
typedef uint32_t lp_u4c __attribute__((ext_vector_type(4)));
template <int N> SSB_INL void lp_load_codes(lp_u4c* cw, const uint32_t* row) {
  const lp_u4c* p = (const lp_u4c*)row;
#pragma unroll
  for (int k = 0; k < N; ++k) cw[k] = p[k];
}
SSB_INL fp lp_get(const lfp* p) {
  const SSB_LDS lp_u4* q = (const SSB_LDS lp_u4*)p;
  const lp_u4 a = q[0], b = q[1], c = q[2];
  fp r;
  r.l[0] = a.x; r.l[1] = a.y; r.l[2] = a.z; r.l[3] = a.w;
  r.l[4] = b.x; r.l[5] = b.y; r.l[6] = b.z; r.l[7] = b.w;
  r.l[8] = c.x; r.l[9] = c.y; r.l[10] = c.z; r.l[11] = c.w;
  return r;
}
SSB_INL void lp_put(lfp* p, const fp& v) {
  SSB_LDS lp_u4* q = (SSB_LDS lp_u4*)p;
  q[0] = lp_u4{v.l[0], v.l[1], v.l[2], v.l[3]};
  q[1] = lp_u4{v.l[4], v.l[5], v.l[6], v.l[7]};
  q[2] = lp_u4{v.l[8], v.l[9], v.l[10], v.l[11]};
}
#else
SSB_INL fp lp_get(const lfp* p) { return *p; }
SSB_INL void lp_put(lfp* p, const fp& v) { *p = v; }
#endif

// ---- 12-limb helpers without modular reduction ----
SSB_INL void lp_add_raw(fp& x, const fp& v) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) x.l[i] = addc(x.l[i], v.l[i], c, c);
}
SSB_INL void lp_pminus(fp& r, const fp& v) {  // p - v (v < p)
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.l[i] = subb(P_LIMBS[i], v.l[i], br, br);
}
SSB_INL void lp_sel(fp& r, const fp& a, const fp& b, uint32_t s) {  // r = s ? a : b
#pragma unroll
  for (int i = 0; i < 12; ++i) r.l[i] = s ? a.l[i] : b.l[i];
}

template <class GR> SSB_INL void lp_ld(fp& x, const GR& g, uint32_t c) { x = lp_get(lp_ptr(g, c)); }
template <class GR> SSB_INL void lp_ld_neg(fp& x, const GR& g, uint32_t c) { lp_pminus(x, lp_get(lp_ptr(g, c))); }
template <class GR> SSB_INL void lp_ld_sgn(fp& x, const GR& g, uint32_t c, uint32_t s) {
  const fp v = lp_get(lp_ptr(g, c));
  fp n; lp_pminus(n, v);
  lp_sel(x, n, v, s);
}
template <class GR> SSB_INL void lp_acc(fp& x, const GR& g, uint32_t c) { lp_add_raw(x, lp_get(lp_ptr(g, c))); }
template <class GR> SSB_INL void lp_acc_neg(fp& x, const GR& g, uint32_t c) {
  fp n; lp_pminus(n, lp_get(lp_ptr(g, c)));
  lp_add_raw(x, n);
}
template <class GR> SSB_INL void lp_acc_sgn(fp& x, const GR& g, uint32_t c, uint32_t s) {
  const fp v = lp_get(lp_ptr(g, c));
  fp n; lp_pminus(n, v);
  fp t; lp_sel(t, n, v, s);
  lp_add_raw(x, t);
}
template <class GR> SSB_INL void lp_st(const GR& g, uint32_t c, const fp& v) { lp_put(lp_ptr(g, c), v); }

// modular doubling / addition of reduced values (< p)
SSB_INL void lp_csub(fp& x, const uint32_t* mp);
SSB_INL void lp_dbl_mod(fp& u) { fp t = u; lp_add_raw(u, t); lp_csub(u, P_LIMBS); }
SSB_INL void lp_add_mod(fp& u, const fp& v) { lp_add_raw(u, v); lp_csub(u, P_LIMBS); }
SSB_INL void lp_add_mod_sel(fp& u, const fp& v, uint32_t s) { fp t = u; lp_add_mod(t, v); lp_sel(u, t, u, s); }

// x >= m*p ? x - m*p : x   (m*p given as limbs)
SSB_INL void lp_csub(fp& x, const uint32_t* mp) {
  fp t;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) t.l[i] = subb(x.l[i], mp[i], br, br);
  lp_sel(x, x, t, br);
}
constexpr uint32_t LP_P2[12] = {0xffff5556u, 0x73fdffffu, 0x62a7ffffu, 0x3d57fffdu, 0xed61ec48u, 0xce61a541u,
                                0xe70a257eu, 0xc8ee9709u, 0x869759aeu, 0x96374f6cu, 0x72ffcd34u, 0x340223d4u};
constexpr uint32_t LP_P4[12] = {0xfffeaaacu, 0xe7fbffffu, 0xc54ffffeu, 0x7aaffffau, 0xdac3d890u, 0x9cc34a83u,
                                0xce144afdu, 0x91dd2e13u, 0x0d2eb35du, 0x2c6e9ed9u, 0xe5ff9a69u, 0x680447a8u};
SSB_INL void lp_reduce1(fp& x) { lp_csub(x, P_LIMBS); }
SSB_INL void lp_reduce2(fp& x) { lp_csub(x, P_LIMBS); lp_csub(x, P_LIMBS); }
SSB_INL void lp_reduce3(fp& x) { lp_csub(x, LP_P2); lp_csub(x, P_LIMBS); lp_csub(x, P_LIMBS); }
SSB_INL void lp_reduce4(fp& x) { lp_csub(x, LP_P4); lp_csub(x, LP_P2); lp_csub(x, P_LIMBS); lp_csub(x, P_LIMBS); }

// ---- the accumulator engine for long / scaled forms ----------------------------------------
// value = sum_pos c v + sum_neg |c| (p - v), per 32-bit limb in 64-bit accumulators (ONE
// v_mad_u64_u32 per limb and term, no carry chain), then a signed carry propagation and one
// Barrett-style step: q = floor(top / (p_hi + 1)) underestimates value / p, so value - q p lies in
// [0, 2p) (an operand for fp_mul) and one conditional subtraction makes it < p (a stored value).
struct lacc { uint64_t a[12], b[12]; };
SSB_INL void la_zero(lacc& x) {
#pragma unroll
  for (int i = 0; i < 12; ++i) { x.a[i] = 0; x.b[i] = 0; }
}
SSB_INL void la_pos(lacc& x, const fp& v, uint32_t c) {
#pragma unroll
  for (int i = 0; i < 12; ++i) x.a[i] = (uint64_t)v.l[i] * c + x.a[i];
}
SSB_INL void la_neg(lacc& x, const fp& v, uint32_t c) {
#pragma unroll
  for (int i = 0; i < 12; ++i) x.b[i] = (uint64_t)v.l[i] * c + x.b[i];
}
SSB_INL void la_mix(lacc& x, const fp& v, uint32_t cp, uint32_t cn) { la_pos(x, v, cp); la_neg(x, v, cn); }
template <class GR> SSB_INL void la_ld_pos(lacc& x, const GR& g, uint32_t code, uint32_t c) { la_pos(x, lp_get(lp_ptr(g, code)), c); }
template <class GR> SSB_INL void la_ld_neg(lacc& x, const GR& g, uint32_t code, uint32_t c) { la_neg(x, lp_get(lp_ptr(g, code)), c); }
template <class GR> SSB_INL void la_ld_mix(lacc& x, const GR& g, uint32_t code, uint32_t cp, uint32_t cn) {
  la_mix(x, lp_get(lp_ptr(g, code)), cp, cn);
}
constexpr double LA_INV_PHI = 1.0 / (436277738.0 + 1.0) * (1.0 - 1e-12);  // 1 / ((p >> 352) + 1), rounded down
SSB_INL void la_fin(fp& r, const lacc& x, uint32_t K, bool exact) {
  int64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const uint64_t t = (uint64_t)P_LIMBS[i] * K + x.a[i];
    const int64_t d = (int64_t)(t - x.b[i]) + carry;
    r.l[i] = (uint32_t)d;
    carry = d >> 32;
  }
  const uint64_t hi = ((uint64_t)carry << 32) | r.l[11];  // value >> 352 (carry >= 0: value >= 0)
  const uint32_t q = (uint32_t)((double)hi * LA_INV_PHI);
  uint64_t pc = 0;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const uint64_t pr = (uint64_t)P_LIMBS[i] * q + pc;
    pc = pr >> 32;
    r.l[i] = subb(r.l[i], (uint32_t)pr, br, br);
  }
  if (exact) { lp_csub(r, P_LIMBS); lp_csub(r, P_LIMBS); }
}

template <class GR> SSB_INL void lp_chk(const GR& g, const fp& v, uint32_t bit) {
  if (bit < 31u && fp_is_zero(v)) {
#if defined(__HIP_DEVICE_COMPILE__)
    atomicOr((uint32_t*)g.flag, 1u << bit);
#else
    *g.flag |= 1u << bit;
#endif
  }
}

// true iff one of the program's checks fired (all components of some check were zero)
SSB_INL bool lp_fired(uint32_t flag, const uint32_t* masks, int n) {
  bool f = false;
  for (int i = 0; i < n; ++i) f = f || ((flag & masks[i]) == masks[i] && masks[i] != 0u);
  return f;
}

}  // namespace lane
}  // namespace ssb

#include "ssb_lane_progs.h"
