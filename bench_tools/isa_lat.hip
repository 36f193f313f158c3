// Microbenchmarks for the Fp-multiply design on gfx950 (one wave per SIMD unless noted):
// dependent-chain latency of v_mad_u64_u32 (through the 64-bit addend), of the
// mad + v_addc carry-capture pair, and of v_add_co/v_addc chains; issue rate of independent mads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void lat_mad_chain(uint64_t* out, uint32_t a, uint32_t b, int iters, long long* cyc) {
  uint64_t acc = threadIdx.x;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 32; ++k) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b) : "s40", "s41");
  }
  long long t1 = clock64();
  out[threadIdx.x + blockIdx.x * blockDim.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void lat_mad_addc(uint64_t* out, uint32_t a, uint32_t b, int iters, long long* cyc) {
  uint64_t acc = threadIdx.x; uint32_t top = 0;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 32; ++k)
      asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %3, %0\n\tv_addc_co_u32_e64 %1, s[42:43], 0, %1, s[40:41]"
                   : "+v"(acc), "+v"(top) : "v"(a), "v"(b) : "s40", "s41", "s42", "s43");
  }
  long long t1 = clock64();
  out[threadIdx.x + blockIdx.x * blockDim.x] = acc + top;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void lat_addc_chain(uint64_t* out, uint32_t a, uint32_t b, int iters, long long* cyc) {
  uint32_t x = threadIdx.x, y = a;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      asm volatile("v_add_co_u32_e64 %0, s[40:41], %0, %2\n\tv_addc_co_u32_e64 %1, s[40:41], %1, %2, s[40:41]"
                   : "+v"(x), "+v"(y) : "v"(b) : "s40", "s41");
  }
  long long t1 = clock64();
  out[threadIdx.x + blockIdx.x * blockDim.x] = x + y;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void thr_mad_indep(uint64_t* out, uint32_t a, uint32_t b, int iters, long long* cyc) {
  uint64_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      asm volatile("v_mad_u64_u32 %0, s[40:41], %8, %9, %0\n\tv_mad_u64_u32 %1, s[40:41], %8, %9, %1\n\t"
                   "v_mad_u64_u32 %2, s[40:41], %8, %9, %2\n\tv_mad_u64_u32 %3, s[40:41], %8, %9, %3\n\t"
                   "v_mad_u64_u32 %4, s[40:41], %8, %9, %4\n\tv_mad_u64_u32 %5, s[40:41], %8, %9, %5\n\t"
                   "v_mad_u64_u32 %6, s[40:41], %8, %9, %6\n\tv_mad_u64_u32 %7, s[40:41], %8, %9, %7"
                   : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
                   : "v"(a), "v"(b) : "s40", "s41");
  }
  long long t1 = clock64();
  out[threadIdx.x + blockIdx.x * blockDim.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename K>
void run(const char* name, K k, int ops_per_iter, int blocks, int threads) {
  uint64_t* d; long long* c;
  hipMalloc(&d, (size_t)blocks * threads * 8); hipMalloc(&c, blocks * 8);
  int iters = 4096;
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 3u, 5u, iters, c);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 3u, 5u, iters, c);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  long long cy; hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
  double per = (double)cy / ((double)iters * ops_per_iter);
  printf("  \"%s_b%d_t%d\": {\"clock64_per_op\": %.2f, \"ns_per_op\": %.3f},\n", name, blocks, threads, per,
         ms * 1e6 / ((double)iters * ops_per_iter));
  hipFree(d); hipFree(c);
}

int main() {
  printf("{\n");
  run("dep_mad", lat_mad_chain, 32, 1, 64);
  run("dep_mad_addc_pair", lat_mad_addc, 32, 1, 64);
  run("dep_addc_pair", lat_addc_chain, 16, 1, 64);
  run("indep_mad", thr_mad_indep, 32, 1, 64);
  run("indep_mad", thr_mad_indep, 32, 1, 256);
  run("dep_mad", lat_mad_chain, 32, 1, 512);
  printf("  \"note\": \"clock64 = s_memtime ticks; ns from hipEvents\"\n}\n");
  return 0;
}
