// Latency of one lane-program stage against the Fp product it is built around (one workgroup of
// one wave on an idle chip, in-kernel wall clock): where the final exponentiation's ~3.4 us per
// stage goes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I safestakeoperator_amd/csrc bench_tools/stage_bench.hip -o bench_tools/stage_bench
#include "../safestakeoperator_amd/csrc/ssb_lane_ops.h"
#include <cstdio>
using namespace ssb;
using namespace ssb::lane;

constexpr int S0 = FP12_CYC_SQR2_SCRATCH > FP12_MUL_SCRATCH ? FP12_CYC_SQR2_SCRATCH : FP12_MUL_SCRATCH;

// OP 0: cyclotomic squarings two at a time (3 stages); 1: Fp12 products (3 stages); 2: the exponentiation by x
template <int OP>
__global__ void __launch_bounds__(64) k_prog(int iters, const fp* __restrict__ in, fp* __restrict__ out,
                                             unsigned long long* __restrict__ t) {
  __shared__ fp lds[LP_NCODE_CONST + S0 + 24 + 84];
  __shared__ uint32_t flg;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST, 0, 0, 0, (lu32*)&flg, (int)threadIdx.x};
  lp_init_consts(g);
  const int A = S0, B = S0 + 12;
  if (threadIdx.x < 12) { g.s[A + threadIdx.x] = in[threadIdx.x]; g.s[B + threadIdx.x] = in[12 + threadIdx.x]; }
  __syncthreads();
  const unsigned long long t0 = wall_clock64();
  for (int i = 0; i < iters; ++i) {
    if (OP == 0) f12_cyc_sqr2(g, A, A);
    else if (OP == 1) f12_mul(g, A, B, A);
    else f12_cyc_exp_x(g, A, A);
  }
  __syncthreads();
  const unsigned long long t1 = wall_clock64();
  if (threadIdx.x < 12) out[threadIdx.x] = g.s[A + threadIdx.x];
  if (threadIdx.x == 0) t[0] = t1 - t0;
}

// a chain of Fp products on every lane (operands in registers)
__global__ void __launch_bounds__(64) k_mul(int iters, const fp* __restrict__ in, fp* __restrict__ out,
                                            unsigned long long* __restrict__ t) {
  fp a = in[0], b = in[1];
  a.l[0] ^= threadIdx.x;
  const unsigned long long t0 = wall_clock64();
  for (int i = 0; i < iters; ++i) fp_mul(a, a, b);
  const unsigned long long t1 = wall_clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) t[0] = t1 - t0;
}

// a chain of Fp products whose operands go through LDS with a barrier per product (a stage with
// no operand forms and no table lookups)
__global__ void __launch_bounds__(64) k_mul_lds(int iters, const fp* __restrict__ in, fp* __restrict__ out,
                                                unsigned long long* __restrict__ t) {
  __shared__ fp s[128];
  fp b = in[1];
  s[threadIdx.x] = in[0];
  s[64 + threadIdx.x] = b;
  __syncthreads();
  const unsigned long long t0 = wall_clock64();
  for (int i = 0; i < iters; ++i) {
    fp x = s[(threadIdx.x + 1) & 63], y = s[64 + threadIdx.x];
    fp r;
    fp_mul(r, x, y);
    __syncthreads();
    s[threadIdx.x] = r;
    __syncthreads();
  }
  const unsigned long long t1 = wall_clock64();
  out[threadIdx.x] = s[threadIdx.x];
  if (threadIdx.x == 0) t[0] = t1 - t0;
}

// point operations: lane programs (G lanes per operation) against the single-lane formulas
constexpr int PGS = 40 + 16;
template <int OP>   // 0 g2_dbl, 1 g2_add, 2 g1_dbl, 3 g1_add
__global__ void __launch_bounds__(64) k_pt_lane(int iters, const fp* __restrict__ in, fp* __restrict__ out,
                                                unsigned long long* __restrict__ t) {
  constexpr int G = OP < 2 ? 8 : 4;
  __shared__ fp lds[LP_NCODE_CONST + (64 / G) * PGS];
  __shared__ uint32_t flg[64 / G];
  const int gi = threadIdx.x / G, role = threadIdx.x % G;
  grp g{(lfp*)lds, (lfp*)lds + LP_NCODE_CONST + gi * PGS, 0, 0, 0, (lu32*)&flg[gi], role};
  lp_init_consts(g);
  const int A = 40, B = 46;
  if (role < 6) { g.s[A + role] = in[role]; g.s[B + role] = in[6 + role]; }
  __syncthreads();
  uint32_t exc = 0;
  const unsigned long long t0 = wall_clock64();
  for (int i = 0; i < iters; ++i) {
    if (OP == 0) g2_dbl(g, A, A);
    else if (OP == 1) g2_add(g, A, B, A, exc);
    else if (OP == 2) g1_dbl(g, A, A);
    else g1_add(g, A, B, A, exc);
  }
  __syncthreads();
  const unsigned long long t1 = wall_clock64();
  if (role < 6 && gi == 0) out[role] = g.s[A + role];
  if (threadIdx.x == 0) t[0] = t1 - t0;
  if (exc && threadIdx.x == 0) out[8].l[0] = exc;
}
template <int OP>
__global__ void __launch_bounds__(64) k_pt_single(int iters, const fp* __restrict__ in, fp* __restrict__ out,
                                                  unsigned long long* __restrict__ t) {
  g2_jac p, q;
  g1_jac p1, q1;
  const fp* s = in;
  p.x.c0 = s[0]; p.x.c1 = s[1]; p.y.c0 = s[2]; p.y.c1 = s[3]; p.z.c0 = s[4]; p.z.c1 = s[5];
  q.x.c0 = s[6]; q.x.c1 = s[7]; q.y.c0 = s[8]; q.y.c1 = s[9]; q.z.c0 = s[10]; q.z.c1 = s[11];
  p1.x = s[0]; p1.y = s[1]; p1.z = s[2]; q1.x = s[3]; q1.y = s[4]; q1.z = s[5];
  p.x.c0.l[0] ^= threadIdx.x;
  p1.x.l[0] ^= threadIdx.x;
  const unsigned long long t0 = wall_clock64();
  for (int i = 0; i < iters; ++i) {
    if (OP == 0) jac_dbl(p, p);
    else if (OP == 1) jac_add(p, p, q);
    else if (OP == 2) jac_dbl(p1, p1);
    else jac_add(p1, p1, q1);
  }
  const unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) { out[0] = p.x.c0; out[1] = p1.x; t[0] = t1 - t0; }
}

int main() {
  fp *d_in, *d_out;
  unsigned long long* d_t;
  hipMalloc(&d_in, 64 * sizeof(fp));
  hipMalloc(&d_out, 64 * sizeof(fp));
  hipMalloc(&d_t, 8);
  fp h[64];
  for (int i = 0; i < 64; ++i) for (int k = 0; k < 12; ++k) h[i].l[k] = (k == 11) ? 0x0100u + i : 0x9e3779b9u * (i * 12 + k + 1);
  hipMemcpy(d_in, h, sizeof(h), hipMemcpyHostToDevice);
  int rate_khz = 0;
  hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0);
  auto run = [&](const char* name, void (*k)(int, const fp*, fp*, unsigned long long*), int iters, double per) {
    unsigned long long t = 0;
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, iters, d_in, d_out, d_t);
      hipDeviceSynchronize();
    }
    hipMemcpy(&t, d_t, 8, hipMemcpyDeviceToHost);
    const double us = (double)t / (rate_khz * 1e-3);
    printf("%-22s iters %5d  total %9.1f us  per call %8.3f us  per %s\n", name, iters, us, us / iters,
           per > 0 ? "stage" : "item");
    if (per > 0) printf("%-22s   per stage %.3f us\n", "", us / iters / per);
  };
  printf("wall clock %d kHz\n", rate_khz);
  run("fp_mul chain", k_mul, 2000, 0);
  run("fp_mul via LDS", k_mul_lds, 2000, 0);
  run("fp12_cyc_sqr2", k_prog<0>, 200, 3);
  run("fp12_mul", k_prog<1>, 200, 3);
  run("fp12_cyc_exp_x", k_prog<2>, 10, 0);
  run("lane g2_dbl", k_pt_lane<0>, 200, 0);
  run("lane g2_add", k_pt_lane<1>, 200, 0);
  run("lane g1_dbl", k_pt_lane<2>, 200, 0);
  run("lane g1_add", k_pt_lane<3>, 200, 0);
  run("single g2_dbl", k_pt_single<0>, 200, 0);
  run("single g2_add", k_pt_single<1>, 200, 0);
  run("single g1_dbl", k_pt_single<2>, 200, 0);
  run("single g1_add", k_pt_single<3>, 200, 0);
  return 0;
}
