// Fp inversion latency on one wave (64 lanes, distinct inputs): the engine's safegcd fp_inv against
// Fermat (fp_inv_fermat) and the earlier binary extended Euclid (fp_inv_bgcd), a chain of R per lane.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/inv_bench bench_tools/inv_bench.hip
#include "../safestakeoperator_amd/csrc/ssb_field.h"
#include <cstdio>
#include <vector>
using namespace ssb;

template <int V>
__global__ void __launch_bounds__(64) k_inv(int n, int reps, const fp* __restrict__ in, fp* __restrict__ out) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  fp a = in[s], one = fp_one();
  for (int r = 0; r < reps; ++r) {
    fp t;
    if (V == 0) fp_inv(t, a);
    else if (V == 1) fp_inv_fermat(t, a);
    else fp_inv_bgcd(t, a);
    fp_add(a, t, one);
  }
  out[s] = a;
}

int main() {
  const int N = 65536, R = 8;
  std::vector<fp> h(N);
  uint64_t z = 0x1234567;
  for (int i = 0; i < N; ++i)
    for (int k = 0; k < 12; ++k) { z = z * 6364136223846793005ull + 1442695040888963407ull; h[i].l[k] = (uint32_t)(z >> 33); }
  for (int i = 0; i < N; ++i) h[i].l[11] &= 0x0fffffffu;  // < p
  fp *d, *o0, *o1, *o2;
  hipMalloc(&d, N * sizeof(fp)); hipMalloc(&o0, N * sizeof(fp)); hipMalloc(&o1, N * sizeof(fp)); hipMalloc(&o2, N * sizeof(fp));
  hipMemcpy(d, h.data(), N * sizeof(fp), hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  printf("{");
  for (int n : {64, 16384, 65536}) {
    for (int v = 0; v < 3; ++v) {
      auto go = [&] {
        if (v == 0) hipLaunchKernelGGL(k_inv<0>, dim3(n / 64), dim3(64), 0, 0, n, R, d, o0);
        else if (v == 1) hipLaunchKernelGGL(k_inv<1>, dim3(n / 64), dim3(64), 0, 0, n, R, d, o1);
        else hipLaunchKernelGGL(k_inv<2>, dim3(n / 64), dim3(64), 0, 0, n, R, d, o2);
      };
      go(); hipDeviceSynchronize();
      float best = 1e9;
      for (int r = 0; r < 5; ++r) {
        hipEventRecord(e0); go(); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1); best = ms < best ? ms : best;
      }
      printf("%s\"%s_n%d_us_per_inv\": %.2f", (n == 64 && v == 0) ? "" : ", ", v == 0 ? "safegcd" : (v == 1 ? "fermat" : "bgcd"), n, best * 1000 / R);
    }
    std::vector<fp> a(n), b(n);
    hipMemcpy(a.data(), o0, n * sizeof(fp), hipMemcpyDeviceToHost); hipMemcpy(b.data(), o1, n * sizeof(fp), hipMemcpyDeviceToHost);
    int same = 0;
    for (int i = 0; i < n; ++i) same += fp_eq(a[i], b[i]);
    printf(", \"n%d_agree\": %d", n, same);
  }
  printf("}\n");
  return 0;
}
