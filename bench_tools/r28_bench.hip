// Round 6: is a 14 x 28-bit product-scanning Montgomery product (carry-free 64-bit column
// accumulators: one v_mad_u64_u32 per limb product, R = 2^392, output < 2p left unreduced) faster than
// the engine's 12 x 32-bit FIPS product (one v_mad_u64_u32 + one v_addc per limb product) under a
// SUSTAINED all-MAD load (the subgroup kernel runs at ~1.7 GHz, power-limited)?  Dependent chains per
// lane, 4 waves per SIMD, each variant run for ~2 s (after a warm-up) so the clock settles.
// Output JSON: G products/s of each, instructions per product are read from the disassembly.
#include "../safestakeoperator_amd/csrc/ssb_field.h"
#include <chrono>
#include <cstdio>
using namespace ssb;

struct f28 { uint32_t l[14]; };
constexpr uint32_t M28 = (1u << 28) - 1;
__constant__ uint32_t P28[14];
__constant__ uint32_t P28_INV;   // -p^-1 mod 2^28

// r = a b / 2^392 mod p, r < 2p (limbs 0..12 < 2^28), for a, b < 2^386 with limbs < 2^30
__device__ __forceinline__ void mont28_fips(f28& r, const f28& a, const f28& b) {
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
      acc += (uint64_t)m[k] * P28[0];
    } else {
      r.l[k - 14] = (uint32_t)acc & M28;
    }
    acc >>= 28;
  }
  r.l[13] = (uint32_t)acc;
}

__global__ void __launch_bounds__(256) k_chain28(f28* io, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  f28 a = io[2 * i], b = io[2 * i + 1];
  for (int it = 0; it < iters; ++it) mont28_fips(a, a, b);
  io[2 * i] = a;
}
__global__ void __launch_bounds__(256) k_chain32(fp* io, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  fp a = io[2 * i], b = io[2 * i + 1];
  for (int it = 0; it < iters; ++it) mp_mont_mul_fips4<12>(a.l, a.l, b.l, P_LIMBS, P_INV32);
  io[2 * i] = a;
}

static void to28(uint32_t* o, const uint32_t* w12) {
  for (int k = 0; k < 14; ++k) {
    uint32_t v = 0;
    for (int b = 0; b < 28; ++b) {
      const int bit = 28 * k + b;
      if (bit < 384 && ((w12[bit >> 5] >> (bit & 31)) & 1u)) v |= 1u << b;
    }
    o[k] = v;
  }
}

int main() {
  const int nth = 256 * 4096;   // 4 waves per SIMD on 256 CUs
  uint32_t p28[14];
  to28(p28, P_LIMBS);
  uint32_t inv = 1;
  for (int k = 0; k < 5; ++k) inv *= 2u - p28[0] * inv;
  const uint32_t pinv = (0u - inv) & M28;
  hipMemcpyToSymbol(HIP_SYMBOL(P28), p28, sizeof(p28));
  hipMemcpyToSymbol(HIP_SYMBOL(P28_INV), &pinv, 4);
  f28* h = new f28[2 * nth];
  fp* h32 = new fp[2 * nth];
  uint64_t x = 88172645463325252ull;
  for (int i = 0; i < 2 * nth; ++i) {
    uint32_t w[12];
    for (int k = 0; k < 12; ++k) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; w[k] = (uint32_t)x; }
    w[11] &= 0x0fffffffu;
    to28(h[i].l, w);
    for (int k = 0; k < 12; ++k) h32[i].l[k] = w[k];
  }
  f28* d; fp* d32;
  hipMalloc(&d, sizeof(f28) * 2 * nth); hipMalloc(&d32, sizeof(fp) * 2 * nth);
  hipMemcpy(d, h, sizeof(f28) * 2 * nth, hipMemcpyHostToDevice);
  hipMemcpy(d32, h32, sizeof(fp) * 2 * nth, hipMemcpyHostToDevice);
  // correctness samples: 3 steps of the chain on threads 0..3
  hipLaunchKernelGGL(k_chain28, dim3(nth / 256), dim3(256), 0, 0, d, 3);
  f28* r = new f28[8];
  hipMemcpy(r, d, sizeof(f28) * 8, hipMemcpyDeviceToHost);
  auto hx = [](const f28& v) { static char buf[4][300]; static int q = 0; char* b = buf[q++ & 3]; char* s = b;
                               for (int k = 13; k >= 0; --k) s += sprintf(s, "%08x,", v.l[k]); return b; };
  printf("{\"samples\": [");
  for (int s = 0; s < 4; ++s) printf("%s[\"%s\", \"%s\", \"%s\"]", s ? ", " : "", hx(h[2 * s]), hx(h[2 * s + 1]), hx(r[2 * s]));
  printf("],\n");
  hipMemcpy(d, h, sizeof(f28) * 2 * nth, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](bool r28, int iters) {
    hipEventRecord(e0);
    if (r28) hipLaunchKernelGGL(k_chain28, dim3(nth / 256), dim3(256), 0, 0, d, iters);
    else hipLaunchKernelGGL(k_chain32, dim3(nth / 256), dim3(256), 0, 0, d32, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return (double)nth * iters / ms / 1e6;   // G products / s
  };
  run(false, 64); run(true, 64);
  // calibrate ~2 s per launch, then alternate 3 times
  const double g32 = run(false, 256), g28 = run(true, 256);
  const int it32 = (int)(g32 * 1e9 * 2.0 / nth), it28 = (int)(g28 * 1e9 * 2.0 / nth);
  printf(" \"short_Gmul_s\": {\"fips4_12x32\": %.2f, \"fips_14x28\": %.2f},\n \"sustained_2s\": [", g32, g28);
  for (int rep = 0; rep < 3; ++rep) {
    const double a = run(false, it32), b = run(true, it28);
    printf("%s{\"fips4_12x32\": %.2f, \"fips_14x28\": %.2f}", rep ? ", " : "", a, b);
  }
  printf("],\n \"threads\": %d}\n", nth);
  return 0;
}
