// Per-operation latency of the wave-cooperative tower programs (one 64-lane workgroup).
#include "../safestakeoperator_amd/csrc/ssb_wave.h"
#include <cstdio>
using namespace ssb;

__global__ void __launch_bounds__(64) k(int which, int iters, fp* io, long long* cyc) {
  __shared__ fp slots[wave::S_USER + 64];
  wave::ws w{slots};
  const int lane = threadIdx.x;
  wave::init(w, lane, 64);
  const int U = wave::S_USER;
  for (int j = lane; j < 48; j += 64) slots[U + j] = io[j];
  __syncthreads();
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    if (which == 0) wave::run(w, wave::FP12_CYC_SQR, U, 0, U, lane, 64);
    else if (which == 1) wave::run(w, wave::FP12_MUL, U, U + 12, U, lane, 64);
    else if (which == 2) wave::run(w, wave::FP12_SQR, U, 0, U, lane, 64);
    else if (which == 3) wave::run(w, wave::FP12_MUL_014, U, U + 12, U, lane, 64);
    else if (which == 4) wave::run(w, wave::MILLER_DBL, U + 24, U + 36, U + 24, lane, 64);
    else wave::run(w, wave::FP12_CONJ, U, 0, U, lane, 64);
  }
  long long t1 = clock64();
  if (lane == 0) *cyc = t1 - t0;
  for (int j = lane; j < 48; j += 64) io[j] = slots[U + j];
}

int main() {
  fp* d; long long* c;
  hipMalloc(&d, 48 * sizeof(fp)); hipMalloc(&c, 8);
  fp h[48];
  for (int i = 0; i < 48; ++i) for (int k = 0; k < 12; ++k) h[i].l[k] = (k == 11) ? 0x0100u + i : 0x9e3779b9u * (i * 12 + k + 1);
  const char* nm[] = {"cyc_sqr", "fp12_mul", "fp12_sqr", "mul_014", "miller_dbl", "conj"};
  printf("{");
  for (int which = 0; which < 6; ++which) {
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    int iters = 200;
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, which, 4, d, c);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, which, iters, d, c);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long cy; hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
    printf("%s\"%s_us\": %.2f, \"%s_clk\": %.0f", which ? ", " : "", nm[which], ms * 1e3 / iters, nm[which], (double)cy / iters);
  }
  printf("}\n");
  return 0;
}
