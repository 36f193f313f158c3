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
// Values live in the reduced radix (ssb_f28_field.h: 14 x 28-bit limbs, Montgomery R = 2^392, one
// v_mad_u64_u32 per limb product -- 496 VALU instructions per product against the 12 x 32-bit
// engine's 671), lazily reduced: a slot holds a normalized value < 2p.  A product operand of up to
// 3 terms is formed WITHOUT reduction (a negative term enters as K4P - v, K4P a 'spread' 4p whose
// limbs dominate v's, so a term is < 4p and the form < 12p; 12p * 12p < p * 2^392 keeps the product's
// output < 2p); the generator normalizes an operand whose limbs would make a limb product >= 2^60.
// Materialised forms (up to 8 terms, every limb < 2^32) are normalized and folded below 2p (one
// quotient estimate from the top limbs).  Values enter and leave the slots through lv_in / lv_out
// (the engine's 12 x 32-bit Montgomery form, R = 2^384: a shift by 8 bits and a fold in, an 8-bit
// Montgomery step and a conditional subtraction out), so the kernels' global data stays in the
// engine's form.
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
using lv = r28::f;                                  // a lane value (registers)
struct alignas(16) lslot { uint32_t w[16]; };       // its LDS slot: 14 limbs, padded to four 16-byte words
typedef SSB_LDS lslot lfp;
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
#define LP_DECL_T lv T_
#define LP_FOR(G) for (int role = g.role, once_ = 1; once_; once_ = 0)
#define LP_T T_
#define LP_SYNC() __syncthreads()
#define LP_FOR_ALL_CONSTS(i) for (int i = threadIdx.x; i < LP_NCODE_CONST; i += blockDim.x)
#else
#define LP_DECL_T lv T_[64]
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
SSB_INL lv lp_get(const lfp* p) {
  const SSB_LDS lp_u4* q = (const SSB_LDS lp_u4*)p;
  const lp_u4 a = q[0], b = q[1], c = q[2];
  const uint32_t d0 = p->w[12], d1 = p->w[13];
  lv r;
  r.l[0] = a.x; r.l[1] = a.y; r.l[2] = a.z; r.l[3] = a.w;
  r.l[4] = b.x; r.l[5] = b.y; r.l[6] = b.z; r.l[7] = b.w;
  r.l[8] = c.x; r.l[9] = c.y; r.l[10] = c.z; r.l[11] = c.w;
  r.l[12] = d0; r.l[13] = d1;
  return r;
}
SSB_INL void lp_put(lfp* p, const lv& v) {
  SSB_LDS lp_u4* q = (SSB_LDS lp_u4*)p;
  q[0] = lp_u4{v.l[0], v.l[1], v.l[2], v.l[3]};
  q[1] = lp_u4{v.l[4], v.l[5], v.l[6], v.l[7]};
  q[2] = lp_u4{v.l[8], v.l[9], v.l[10], v.l[11]};
  p->w[12] = v.l[12]; p->w[13] = v.l[13];
}
#else
SSB_INL lv lp_get(const lfp* p) { lv r; for (int i = 0; i < 14; ++i) r.l[i] = p->w[i]; return r; }
SSB_INL void lp_put(lfp* p, const lv& v) { for (int i = 0; i < 14; ++i) p->w[i] = v.l[i]; }
#endif

// ---- lane values ----
SSB_INL lv lv_zero() { lv r; for (int i = 0; i < 14; ++i) r.l[i] = 0u; return r; }
SSB_INL lv lv_one() { return r28::cst(r28::ONE28); }
// carry normalization of limbs up to 2^32 - 1: limbs 0..12 < 2^28, the rest in the top limb
SSB_INL void lv_norm(lv& x) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const uint32_t v = (x.l[i] & r28::M28) + c;
    c = (x.l[i] >> 28) + (v >> 28);
    x.l[i] = v & r28::M28;
  }
  x.l[13] += c;
}
// the engine's form a 2^384 (< p) -> a 2^392 (< 2p): the 12 x 32-bit limbs re-sliced 8 bits up, folded
SSB_INL lv lv_in(const fp& a) { lv r; r28::from_engine_shift(r, a); return r; }
// ... and back: x 2^-8 by one 8-bit Montgomery step ((x + m p) / 2^8, < 1.01 p), then canonical
SSB_INL fp lv_out(const lv& x) { fp r; r28::to_engine_shift(r, x); return r; }
SSB_INL bool lv_is_zero(const lv& x) { return r28::is_zero(x); }
// -x (< 2p)
SSB_INL void lv_neg(lv& x) {
  lv t; r28::neg_raw(t, x, r28::K4P); lv_norm(t); r28::fold(x, t);
}
SSB_INL void lp_put_in(lfp* p, const fp& v) { lp_put(p, lv_in(v)); }
SSB_INL fp lp_get_out(const lfp* p) { return lv_out(lp_get(p)); }
// a slot reached through a generic pointer (an LDS struct passed by reference) -> the engine's form
SSB_INL fp slot_out(const lslot& s) { lv v; for (int i = 0; i < 14; ++i) v.l[i] = s.w[i]; return lv_out(v); }

// ---- forms without modular reduction ----
SSB_INL void lp_add_raw(lv& x, const lv& v) {
#pragma unroll
  for (int i = 0; i < 14; ++i) x.l[i] += v.l[i];
}
SSB_INL void lp_pminus(lv& r, const lv& v) { r28::neg_raw(r, v, r28::K4P); }   // 4p - v (v < 2p: limbs >= 0)
SSB_INL void lp_sel(lv& r, const lv& a, const lv& b, uint32_t s) {  // r = s ? a : b
#pragma unroll
  for (int i = 0; i < 14; ++i) r.l[i] = s ? a.l[i] : b.l[i];
}

template <class GR> SSB_INL void lp_ld(lv& x, const GR& g, uint32_t c) { x = lp_get(lp_ptr(g, c)); }
template <class GR> SSB_INL void lp_ld_neg(lv& x, const GR& g, uint32_t c) { lp_pminus(x, lp_get(lp_ptr(g, c))); }
template <class GR> SSB_INL void lp_ld_sgn(lv& x, const GR& g, uint32_t c, uint32_t s) {
  const lv v = lp_get(lp_ptr(g, c));
  lv n; lp_pminus(n, v);
  lp_sel(x, n, v, s);
}
template <class GR> SSB_INL void lp_acc(lv& x, const GR& g, uint32_t c) { lp_add_raw(x, lp_get(lp_ptr(g, c))); }
template <class GR> SSB_INL void lp_acc_neg(lv& x, const GR& g, uint32_t c) {
  lv n; lp_pminus(n, lp_get(lp_ptr(g, c)));
  lp_add_raw(x, n);
}
template <class GR> SSB_INL void lp_acc_sgn(lv& x, const GR& g, uint32_t c, uint32_t s) {
  const lv v = lp_get(lp_ptr(g, c));
  lv n; lp_pminus(n, v);
  lv t; lp_sel(t, n, v, s);
  lp_add_raw(x, t);
}
template <class GR> SSB_INL void lp_st(const GR& g, uint32_t c, const lv& v) { lp_put(lp_ptr(g, c), v); }

// a materialised sum (<= 8 terms, < 32p) -> a slot value (< 2p, normalized)
SSB_INL void lp_reduce(lv& x) { lv_norm(x); r28::fold(x, x); }
// modular doubling / addition of slot values (the multiple-of-v forms; kept below 2p)
SSB_INL void lp_dbl_mod(lv& u) { lv t = u; lp_add_raw(u, t); lp_reduce(u); }
SSB_INL void lp_add_mod(lv& u, const lv& v) { lp_add_raw(u, v); lp_reduce(u); }
SSB_INL void lp_add_mod_sel(lv& u, const lv& v, uint32_t s) { lv t = u; lp_add_mod(t, v); lp_sel(u, t, u, s); }
// an operand whose limbs are too wide for the product's 64-bit columns
SSB_INL void lp_norm(lv& x) { lv_norm(x); }
// the product (< 2p, normalized)
SSB_INL void lp_mul(lv& r, const lv& x, const lv& y) { r28::mul(r, x, y); }

// ---- the accumulator engine for long / scaled forms ----------------------------------------
// value = sum_pos c v - sum_neg c v + 2K p (K = sum_neg c: v < 2p, so the value is >= 0), per 28-bit
// limb in one signed 64-bit accumulator (ONE v_mad_i64_i32 per limb and term, positive and negative
// coefficients alike), then a signed carry propagation; with `fold` the result is brought below 2p
// (a stored value, or an operand whose bound would break the product's), else it stays < 2p sum|c|.
struct lacc { int64_t a[14]; };
SSB_INL void la_zero(lacc& x) {
#pragma unroll
  for (int i = 0; i < 14; ++i) x.a[i] = 0;
}
SSB_INL void la_add(lacc& x, const lv& v, int32_t c) {
#pragma unroll
  for (int i = 0; i < 14; ++i) x.a[i] += (int64_t)(int32_t)v.l[i] * (int64_t)c;
}
SSB_INL void la_pos(lacc& x, const lv& v, uint32_t c) { la_add(x, v, (int32_t)c); }
SSB_INL void la_neg(lacc& x, const lv& v, uint32_t c) { la_add(x, v, -(int32_t)c); }
SSB_INL void la_mix(lacc& x, const lv& v, uint32_t cp, uint32_t cn) { la_add(x, v, (int32_t)cp - (int32_t)cn); }
template <class GR> SSB_INL void la_ld_pos(lacc& x, const GR& g, uint32_t code, uint32_t c) { la_pos(x, lp_get(lp_ptr(g, code)), c); }
template <class GR> SSB_INL void la_ld_neg(lacc& x, const GR& g, uint32_t code, uint32_t c) { la_neg(x, lp_get(lp_ptr(g, code)), c); }
template <class GR> SSB_INL void la_ld_mix(lacc& x, const GR& g, uint32_t code, uint32_t cp, uint32_t cn) {
  la_mix(x, lp_get(lp_ptr(g, code)), cp, cn);
}
SSB_INL void la_fin(lv& r, const lacc& x, uint32_t K, bool fold) {
  const int64_t k2 = 2 * (int64_t)K;
  int64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const int64_t t = x.a[i] + k2 * (int64_t)r28::P28[i] + carry;
    r.l[i] = (uint32_t)t & r28::M28;
    carry = t >> 28;   // (arithmetic)
  }
  r.l[13] = (uint32_t)(x.a[13] + k2 * (int64_t)r28::P28[13] + carry);
  if (fold) r28::fold(r, r);
}

template <class GR> SSB_INL void lp_chk(const GR& g, const lv& v, uint32_t bit) {
  if (bit < 31u && lv_is_zero(v)) {
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
