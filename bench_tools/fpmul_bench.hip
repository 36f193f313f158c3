// Fp-multiply variants on gfx950: bit-exactness, throughput (full chip), single-wave latency.
#include "../safestakeoperator_amd/csrc/ssb_field.h"
#include <cstdio>
using namespace ssb;

template <int V> __device__ __forceinline__ void mul(fp& r, const fp& a, const fp& b) {
  if (V == 0) mp_mont_mul_cios<12>(r.l, a.l, b.l, P_LIMBS, P_INV32);
  else if (V == 1) mp_mont_mul_fips<12>(r.l, a.l, b.l, P_LIMBS, P_INV32);
  else if (V == 2) mp_mont_mul_fips2<12>(r.l, a.l, b.l, P_LIMBS, P_INV32);
  else if (V == 3) mp_mont_mul_fips4<12>(r.l, a.l, b.l, P_LIMBS, P_INV32);
  else mp_mont_mul_fips4x2<12>(r.l, a.l, b.l, P_LIMBS, P_INV32);
}

template <int V> __global__ void __launch_bounds__(256) k_chain(fp* io, int iters, long long* cyc) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  fp a = io[2 * i], b = io[2 * i + 1];
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) mul<V>(a, a, b);
  long long t1 = clock64();
  io[2 * i] = a;
  if (cyc && threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
// two independent chains per thread (ILP 2)
template <int V> __global__ void __launch_bounds__(256) k_chain2(fp* io, int iters, long long* cyc) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  fp a = io[2 * i], b = io[2 * i + 1], c = b;
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) { mul<V>(a, a, b); mul<V>(c, c, a); }
  long long t1 = clock64();
  io[2 * i] = a; io[2 * i + 1] = c;
  if (cyc && threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int nth = 256 * 2048;
  fp* h = new fp[2 * nth];
  uint64_t x = 88172645463325252ull;
  for (int i = 0; i < 2 * nth; ++i) { for (int k = 0; k < 12; ++k) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i].l[k] = (uint32_t)x; } h[i].l[11] &= 0x0fffffffu; }
  fp *d0, *d1; long long* cyc;
  hipMalloc(&d0, sizeof(fp) * 2 * nth); hipMalloc(&d1, sizeof(fp) * 2 * nth); hipMalloc(&cyc, 8 * 4096);
  hipMemcpy(d0, h, sizeof(fp) * 2 * nth, hipMemcpyHostToDevice);
  hipMemcpy(d1, h, sizeof(fp) * 2 * nth, hipMemcpyHostToDevice);
  // exactness: 64 chained muls on every thread, both variants
  hipLaunchKernelGGL(k_chain<0>, dim3(nth / 256), dim3(256), 0, 0, d0, 64, (long long*)nullptr);
  hipLaunchKernelGGL(k_chain<1>, dim3(nth / 256), dim3(256), 0, 0, d1, 64, (long long*)nullptr);
  fp* d2; hipMalloc(&d2, sizeof(fp) * 2 * nth); hipMemcpy(d2, h, sizeof(fp) * 2 * nth, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_chain<4>, dim3(nth / 256), dim3(256), 0, 0, d2, 64, (long long*)nullptr);
  fp* r2 = new fp[2 * nth]; hipMemcpy(r2, d2, sizeof(fp) * 2 * nth, hipMemcpyDeviceToHost);
  fp* r0 = new fp[2 * nth]; fp* r1 = new fp[2 * nth];
  hipMemcpy(r0, d0, sizeof(fp) * 2 * nth, hipMemcpyDeviceToHost);
  hipMemcpy(r1, d1, sizeof(fp) * 2 * nth, hipMemcpyDeviceToHost);
  long bad = 0;
  for (int i = 0; i < 2 * nth; ++i) for (int k = 0; k < 12; ++k) bad += (r0[i].l[k] != r1[i].l[k]) + (r0[i].l[k] != r2[i].l[k]);
  printf("{\"mismatching_limbs\": %ld,\n", bad);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto thr = [&](const char* nm, void (*k)(fp*, int, long long*), int per) {
    int iters = 256;
    hipLaunchKernelGGL(k, dim3(nth / 256), dim3(256), 0, 0, d1, 8, (long long*)nullptr);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(nth / 256), dim3(256), 0, 0, d1, iters, (long long*)nullptr);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double muls = (double)nth * iters * per;
    printf(" \"%s_Gmul_per_s\": %.2f, \"%s_TMAD_per_s_at_300\": %.3f,\n", nm, muls / ms / 1e6, nm, muls * 300 / ms / 1e9);
  };
  thr("cios_thr", k_chain<0>, 1);
  thr("fips_thr", k_chain<1>, 1);
  thr("fips2_thr", k_chain<2>, 1);
  thr("fips4_thr", k_chain<3>, 1);
  thr("fips4_thr_ilp2", k_chain2<3>, 2);
  thr("fips4x2_thr", k_chain<4>, 1);
  thr("cios_thr_ilp2", k_chain2<0>, 2);
  thr("fips2_thr_ilp2", k_chain2<2>, 2);
  thr("fips_thr_ilp2", k_chain2<1>, 2);
  auto lat = [&](const char* nm, void (*k)(fp*, int, long long*), int per) {
    int iters = 2048;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d1, iters, cyc);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d1, iters, cyc);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf(" \"%s_1wave_ns_per_mul\": %.1f, \"%s_1wave_clk_per_mul\": %.1f,\n", nm, ms * 1e6 / (iters * per), nm, (double)c / (iters * per));
  };
  lat("cios", k_chain<0>, 1);
  lat("fips", k_chain<1>, 1);
  lat("fips2", k_chain<2>, 1);
  lat("fips4", k_chain<3>, 1);
  lat("fips4_ilp2", k_chain2<3>, 2);
  lat("fips4x2", k_chain<4>, 1);
  lat("fips2_ilp2", k_chain2<2>, 2);
  lat("cios_ilp2", k_chain2<0>, 2);
  lat("fips_ilp2", k_chain2<1>, 2);
  printf(" \"end\": 0}\n");
  return 0;
}
