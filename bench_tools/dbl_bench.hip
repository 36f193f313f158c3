// Single-lane G2 doubling / addition throughput and latency, built three ways (bench_tools/dbl_bench.sh):
// Montgomery products inlined into the point formulas (default), out of line by reference
// (-DSSB_FPMUL_CALL=1), out of line by value (-DSSB_FPMUL_CALL=2).
#include "../safestakeoperator_amd/csrc/ssb_curve.h"
#include <cstdio>
using namespace ssb;

template <int OP>
__global__ void __launch_bounds__(64) k_single(int iters, const fp* __restrict__ in, fp* __restrict__ out) {
  g2_jac p, q;
  const fp* s = in;
  p.x.c0 = s[0]; p.x.c1 = s[1]; p.y.c0 = s[2]; p.y.c1 = s[3]; p.z.c0 = s[4]; p.z.c1 = s[5];
  q.x.c0 = s[6]; q.x.c1 = s[7]; q.y.c0 = s[8]; q.y.c1 = s[9]; q.z.c0 = s[10]; q.z.c1 = s[11];
  p.x.c0.l[0] ^= threadIdx.x;
  for (int i = 0; i < iters; ++i) {
    if (OP == 0) jac_dbl(p, p);
    else jac_add(p, p, q);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) { out[0] = p.x.c0; }
}

int main() {
  fp* d_in; fp* d_out;
  hipMalloc(&d_in, 16 * sizeof(fp)); hipMalloc(&d_out, 16 * sizeof(fp));
  fp h[16];
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 12; ++k) h[i].l[k] = (k == 11) ? 0x0100u + i : 0x9e3779b9u * (i * 12 + k + 1);
  hipMemcpy(d_in, h, sizeof(h), hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const char* nm[] = {"dbl", "add"};
  printf("{");
  for (int op = 0; op < 2; ++op) {
    for (int wps : {1, 2, 4}) {
      const int grid = 1024 * wps, iters = 16;
      auto launch = [&](int it) {
        if (op == 0) hipLaunchKernelGGL(k_single<0>, dim3(grid), dim3(64), 0, 0, it, d_in, d_out);
        else hipLaunchKernelGGL(k_single<1>, dim3(grid), dim3(64), 0, 0, it, d_in, d_out);
      };
      launch(2); hipDeviceSynchronize();
      hipEventRecord(e0); launch(iters); hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double ops = (double)grid * 64 * iters;
      printf("%s\"%s_w%d\": {\"us_per_op_latency\": %.2f, \"Mops_per_s\": %.1f}", (op || wps > 1) ? ", " : "", nm[op], wps,
             ms * 1e3 / iters, ops / (ms * 1e-3) / 1e6);
    }
  }
  printf("}\n");
  return 0;
}
