// Diagnostic (round 5): the ratio combine's device code in isolation.  64 registry-id jobs
// (3-of-3 shares over hash_to_G2 points), each phase in its own kernel with a progress word per lane
// in mapped host memory, polled by the host with a deadline -- which step does not finish, and are
// the results the host build's?
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 bench_tools/rc_test.hip -o bench_tools/rc_test
#include "../safestakeoperator_amd/csrc/ssb_units.h"
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>
using namespace ssb;

#ifndef RC_WAVES
#define RC_WAVES 2
#endif
#define LB __attribute__((amdgpu_flat_work_group_size(1, 64), amdgpu_waves_per_eu(RC_WAVES)))

constexpr int NJ = 64, T3 = 3;
struct job { g2_aff pts[T3]; uint32_t idx[T3]; int64_t c[T3]; uint64_t M; };

__device__ __forceinline__ void mark(volatile uint32_t* prog, uint32_t v) {
  prog[threadIdx.x] = v;
  __threadfence_system();
}

// the joint sum step by step, inline, with a mark after each stage
__global__ void LB k_steps(const job* __restrict__ J, uint8_t* __restrict__ tabs, g2_jac* __restrict__ Tout,
                           volatile uint32_t* prog) {
  const int j = threadIdx.x;
  const job& b = J[j];
  uint8_t* region = tabs + (size_t)j * RC_TAB_BYTES;
  g2_xy* xy = (g2_xy*)(region + RC_XY_OFF);
  fp2* zs = (fp2*)(region + RC_Z_OFF);
  fp2* pr = (fp2*)(region + RC_PR_OFF);
  mark(prog, 1);
  for (int q = 0; q < T3; ++q) rc_odd_multiples(xy + 8 * q, zs + 8 * q, (g2_jac*)pr, b.pts[q]);
  mark(prog, 2);
  rc_normalize(xy, zs, pr, 8 * T3);
  mark(prog, 3);
  int W = rc_windows(b.c, T3);
  for (int o = 32; o >= 1; o >>= 1) { const int x = __shfl_xor(W, o, 64); W = x > W ? x : W; }
  W = __builtin_amdgcn_readfirstlane(W);
  g2_jac acc;
  jac_set_inf(acc);
  for (int jj = W - 1; jj >= 0; --jj) {
    if (jj != W - 1)
      for (int q = 0; q < 4; ++q) jac_dbl_inl(acc, acc);
    for (int q = 0; q < T3; ++q) {
      const int64_t cb = b.c[q];
      const uint64_t m = (uint64_t)(cb < 0 ? -cb : cb) | 1ull;
      const int d = sw4_digit(m, jj, W);
      const int ad = d < 0 ? -d : d;
      jac_madd_xy(acc, xy + 8 * q + ((ad - 1) >> 1), (d < 0) != (cb < 0));
    }
    mark(prog, 100 + jj);
  }
  mark(prog, 4);
  Tout[j] = acc;
}
// phase T as the product runs it (out of line)
__global__ void LB k_phaseT(const job* __restrict__ J, uint8_t* __restrict__ tabs, g2_jac* __restrict__ Tout,
                            uint64_t* __restrict__ kk, volatile uint32_t* prog) {
  const int j = threadIdx.x;
  int64_t c[T3];
  for (int q = 0; q < T3; ++q) c[q] = J[j].c[q];
  int W = rc_windows(c, T3);
  for (int o = 32; o >= 1; o >>= 1) { const int x = __shfl_xor(W, o, 64); W = x > W ? x : W; }
  W = __builtin_amdgcn_readfirstlane(W);
  mark(prog, 1);
  unit_ratio_T(Tout + j, kk + 4 * j, J[j].pts, J[j].idx, c, T3, J[j].M, W, tabs + (size_t)j * RC_TAB_BYTES);
  mark(prog, 2);
}
__global__ void LB k_phaseK(const g2_jac* __restrict__ Tin, const uint64_t* __restrict__ kk, uint8_t* __restrict__ tabs,
                            uint8_t* __restrict__ out96, volatile uint32_t* prog) {
  const int j = threadIdx.x;
  mark(prog, 1);
  unit_ratio_K(out96 + 96 * j, Tin + j, kk + 4 * j, tabs + (size_t)j * RC_TAB_BYTES);
  mark(prog, 2);
}

static bool wait_for(volatile uint32_t* prog, uint32_t done, double sec, const char* name) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    bool all = true;
    for (int i = 0; i < NJ; ++i) all = all && prog[i] == done;
    if (all) { printf("%s: done in %.3f s\n", name, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count()); return true; }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > sec) {
      printf("%s: NOT done after %.0f s; lane progress:", name, sec);
      for (int i = 0; i < NJ; ++i) printf(" %u", prog[i]);
      printf("\n");
      fflush(stdout);
      return false;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

int main(int argc, char** argv) {
  const int which = argc > 1 ? atoi(argv[1]) : 0;   // 0: steps, 1: phase T, 2: phases T + K
  static const char* DST = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
  std::vector<job> jobs(NJ);
  std::vector<uint8_t> want(NJ * 96);
  uint64_t seed = 0x1234567;
  for (int j = 0; j < NJ; ++j) {
    uint64_t x[T3];
    for (int q = 0; q < T3; ++q) {
      uint8_t m[32] = {0}; m[0] = (uint8_t)j; m[1] = (uint8_t)q; m[2] = 0x77;
      hash_to_g2(jobs[j].pts[q], m, (const uint8_t*)DST, (int)strlen(DST));
      jobs[j].idx[q] = (uint32_t)q;
      seed = seed * 6364136223846793005ull + 1442695040888963407ull;
      x[q] = 1 + ((seed >> 33) % 65535) + (uint64_t)q * 7;   // distinct enough for the test
    }
    if (!unit_lagrange_ratio(jobs[j].c, &jobs[j].M, x, T3)) { printf("job %d not ratio-eligible\n", j); return 2; }
    std::vector<uint8_t> region(RC_TAB_BYTES);
    unit_combine_ratio_w4(&want[96 * j], jobs[j].pts, jobs[j].idx, jobs[j].c, T3, jobs[j].M,
                          rc_windows(jobs[j].c, T3), region.data());
  }
  job* dJ; uint8_t *dtabs, *dout; g2_jac* dT; uint64_t* dk; uint32_t* prog; uint32_t* dprog;
  hipMalloc(&dJ, sizeof(job) * NJ);
  hipMalloc(&dtabs, RC_TAB_BYTES * NJ);
  hipMalloc(&dout, 96 * NJ);
  hipMalloc(&dT, sizeof(g2_jac) * NJ);
  hipMalloc(&dk, 32 * NJ);
  hipHostMalloc((void**)&prog, 4 * NJ, hipHostMallocMapped);
  hipHostGetDevicePointer((void**)&dprog, prog, 0);
  hipMemcpy(dJ, jobs.data(), sizeof(job) * NJ, hipMemcpyHostToDevice);
  memset(prog, 0, 4 * NJ);
  if (which == 0) {
    hipLaunchKernelGGL(k_steps, dim3(1), dim3(64), 0, 0, dJ, dtabs, dT, dprog);
    if (!wait_for(prog, 4, 20, "k_steps")) return 3;
    hipDeviceSynchronize();
    return 0;
  }
  hipLaunchKernelGGL(k_phaseT, dim3(1), dim3(64), 0, 0, dJ, dtabs, dT, dk, dprog);
  if (!wait_for(prog, 2, 20, "k_phaseT")) return 3;
  hipDeviceSynchronize();
  if (which == 1) return 0;
  memset(prog, 0, 4 * NJ);
  hipLaunchKernelGGL(k_phaseK, dim3(1), dim3(64), 0, 0, dT, dk, dtabs, dout, dprog);
  if (!wait_for(prog, 2, 20, "k_phaseK")) return 3;
  hipDeviceSynchronize();
  std::vector<uint8_t> got(NJ * 96);
  hipMemcpy(got.data(), dout, 96 * NJ, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int j = 0; j < NJ; ++j) bad += memcmp(&got[96 * j], &want[96 * j], 96) != 0;
  printf("results: %d of %d differ from the host build\n", bad, NJ);
  return bad ? 4 : 0;
}
