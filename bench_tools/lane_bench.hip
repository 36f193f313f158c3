// Latency / throughput of the lane-group point programs against the single-lane formulas.
// One workgroup = one wave = 64/G groups; the grid decides how many waves share a SIMD.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I safestakeoperator_amd/csrc bench_tools/lane_bench.hip -o bench_tools/lane_bench
#include "../safestakeoperator_amd/csrc/ssb_lane_ops.h"
#include <cstdio>
using namespace ssb;
using namespace ssb::lane;

constexpr int GS = 40 + 16;  // scratch + A(6) + B(6) + spare

template <int OP>
__global__ void __launch_bounds__(64) k_lane(int iters, const fp* __restrict__ in, fp* __restrict__ out) {
  __shared__ fp lds[LP_NCODE_CONST + 8 * GS];
  __shared__ uint32_t flg[8];
  const int gi = threadIdx.x / 8, role = threadIdx.x % 8;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST + gi * GS, 0, 0, 0, (lu32*)&flg[gi], role};
  lp_init_consts(g);
  const int A = 40, B = 46;
  if (role < 6) { g.s[A + role] = in[role]; g.s[B + role] = in[6 + role]; }
  __syncthreads();
  uint32_t exc = 0;
  for (int i = 0; i < iters; ++i) {
    if (OP == 0) g2_dbl(g, A, A);
    else if (OP == 1) g2_add(g, A, B, A, exc);
    else g2_madd(g, A, B, A, exc);
  }
  if (role < 6 && blockIdx.x == 0 && gi == 0) out[role] = g.s[A + role];
  if (exc && role == 0 && blockIdx.x == 0) out[7].l[0] = exc;
}

template <int OP>
__global__ void __launch_bounds__(64) k_single(int iters, const fp* __restrict__ in, fp* __restrict__ out) {
  g2_jac p, q;
  const fp* s = in;
  p.x.c0 = s[0]; p.x.c1 = s[1]; p.y.c0 = s[2]; p.y.c1 = s[3]; p.z.c0 = s[4]; p.z.c1 = s[5];
  q.x.c0 = s[6]; q.x.c1 = s[7]; q.y.c0 = s[8]; q.y.c1 = s[9]; q.z.c0 = s[10]; q.z.c1 = s[11];
  p.x.c0.l[0] ^= threadIdx.x;  // distinct per lane
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
  const char* nm[] = {"dbl", "add", "madd"};
  printf("{");
  int first = 1;
  for (int op = 0; op < 3; ++op) {
    for (int wps : {1, 2, 4}) {  // waves per SIMD requested (grid = 1024 * wps WGs)
      const int grid = 1024 * wps, iters = 64;
      auto launch = [&](int it) {
        if (op == 0) hipLaunchKernelGGL(k_lane<0>, dim3(grid), dim3(64), 0, 0, it, d_in, d_out);
        else if (op == 1) hipLaunchKernelGGL(k_lane<1>, dim3(grid), dim3(64), 0, 0, it, d_in, d_out);
        else hipLaunchKernelGGL(k_lane<2>, dim3(grid), dim3(64), 0, 0, it, d_in, d_out);
      };
      launch(2); hipDeviceSynchronize();
      hipEventRecord(e0); launch(iters); hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double ops = (double)grid * 8 * iters;
      printf("%s\"lane_%s_w%d\": {\"us_per_op_latency\": %.2f, \"Mops_per_s\": %.1f}", first ? "" : ", ", nm[op], wps,
             ms * 1e3 / iters, ops / (ms * 1e-3) / 1e6);
      first = 0;
    }
  }
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
      printf(", \"single_%s_w%d\": {\"us_per_op_latency\": %.2f, \"Mops_per_s\": %.1f}", nm[op], wps,
             ms * 1e3 / iters, ops / (ms * 1e-3) / 1e6);
    }
  }
  printf("}\n");
  return 0;
}
