// Round 6: is the reduced-radix product (ssb_f28_field.h r28::mul: one 64-bit accumulator per column,
// each limb product one v_mad_u64_u32 into it -- a chain of up to 28 dependent MADs per column) limited
// by that chain's latency at the occupancies the kernels run (lane programs: one wave per SIMD; the
// per-share kernels: two)?  Variants: the product as shipped, and the column split into independent
// accumulators (products with even / odd j, the reduction's terms apart) summed at the column's end.
// Dependent chains of products per lane at 1, 2 and 4 waves per SIMD; G products/s of each.
#include "../safestakeoperator_amd/csrc/ssb_field.h"
#include <cstdio>
using namespace ssb;
using r28::f;

__device__ __forceinline__ void mul_split(f& r, const f& a, const f& b) {
  uint32_t m[14];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; ++k) {
    uint64_t s0 = 0, s1 = 0, t0 = 0, t1 = 0;
#pragma unroll
    for (int j = 0; j < 14; ++j)
      if (k - j >= 0 && k - j < 14) { if (j & 1) s1 += (uint64_t)a.l[j] * b.l[k - j]; else s0 += (uint64_t)a.l[j] * b.l[k - j]; }
#pragma unroll
    for (int j = 0; j < 14; ++j)
      if (j < k && k - j < 14) { if (j & 1) t1 += (uint64_t)m[j] * r28::P28[k - j]; else t0 += (uint64_t)m[j] * r28::P28[k - j]; }
    acc += (s0 + s1) + (t0 + t1);
    if (k < 14) {
      m[k] = ((uint32_t)acc * r28::P28_INV) & r28::M28;
      acc += (uint64_t)m[k] * r28::P28[0];
    } else {
      r.l[k - 14] = (uint32_t)acc & r28::M28;
    }
    acc >>= 28;
  }
  r.l[13] = (uint32_t)acc;
}

template <int V>
__global__ void __launch_bounds__(64) k_chain(f* io, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  f a = io[2 * i], b = io[2 * i + 1];
  for (int it = 0; it < iters; ++it) {
    if (V == 0) r28::mul(a, a, b); else mul_split(a, a, b);
  }
  io[2 * i] = a;
}

int main() {
  int ncu = 256;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int maxth = ncu * 4 * 4 * 64;
  f* h = new f[2 * maxth];
  uint64_t x = 88172645463325252ull;
  for (int i = 0; i < 2 * maxth; ++i) {
    for (int k = 0; k < 14; ++k) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i].l[k] = (uint32_t)x & r28::M28; }
    h[i].l[13] &= 0xffffu;   // < 2p
  }
  f* d;
  hipMalloc(&d, sizeof(f) * 2 * maxth);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  // the two forms agree (same residue, both < 2p: compared after one more product by 1 is not needed --
  // they are the same integer sums, so the same outputs)
  {
    hipMemcpy(d, h, sizeof(f) * 2 * 64, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), 0, 0, d, 5);
    f r0[2]; hipMemcpy(r0, d, sizeof(f) * 2, hipMemcpyDeviceToHost);
    hipMemcpy(d, h, sizeof(f) * 2 * 64, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, d, 5);
    f r1[2]; hipMemcpy(r1, d, sizeof(f) * 2, hipMemcpyDeviceToHost);
    bool same = true;
    for (int k = 0; k < 14; ++k) same = same && r0[0].l[k] == r1[0].l[k];
    printf("{\"same_outputs\": %s, \"runs\": [", same ? "true" : "false");
  }
  int first = 1;
  for (int w = 1; w <= 4; w *= 2) {
    const int nth = ncu * 4 * w * 64;
    for (int v = 0; v < 2; ++v) {
      hipMemcpy(d, h, sizeof(f) * 2 * nth, hipMemcpyHostToDevice);
      auto launch = [&](int iters) {
        if (v == 0) hipLaunchKernelGGL(k_chain<0>, dim3(nth / 64), dim3(64), 0, 0, d, iters);
        else hipLaunchKernelGGL(k_chain<1>, dim3(nth / 64), dim3(64), 0, 0, d, iters);
      };
      launch(16);
      hipEventRecord(e0); launch(2048); hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      printf("%s{\"waves_per_simd\": %d, \"variant\": \"%s\", \"G_products_s\": %.2f}", first ? "" : ", ", w,
             v ? "split" : "shipped", (double)nth * 2048 / ms / 1e6);
      first = 0;
    }
  }
  printf("]}\n");
  return 0;
}
