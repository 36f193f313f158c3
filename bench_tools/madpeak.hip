// Microbenchmark: sustained v_mad_u64_u32 (32x32+64 -> 64) issue rate on gfx950.
// Each lane runs NCH independent multiply-add chains; the kernel reports MADs/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int NCH>
__global__ void __launch_bounds__(256) mad_chain(uint64_t* out, uint32_t seed, int iters) {
  uint32_t b = seed ^ (threadIdx.x * 2654435761u);
  uint64_t acc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c] = (uint64_t)(b + c) << 7;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        // acc = lo(acc) * b + acc   (one v_mad_u64_u32)
        acc[c] = (uint64_t)(uint32_t)acc[c] * b + acc[c];
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// v_mul_lo_u32 + v_mul_hi_u32 pair for comparison
template <int NCH>
__global__ void __launch_bounds__(256) mulhilo_chain(uint64_t* out, uint32_t seed, int iters) {
  uint32_t b = seed ^ (threadIdx.x * 2654435761u);
  uint32_t lo[NCH], hi[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) { lo[c] = b + c; hi[c] = b ^ c; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        uint32_t l, h;
        asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(l) : "v"(lo[c]), "v"(b));
        asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(h) : "v"(hi[c]), "v"(b));
        lo[c] = l; hi[c] = h;
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s ^= ((uint64_t)hi[c] << 32) | lo[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// plain 32-bit add for the VALU issue reference
template <int NCH>
__global__ void __launch_bounds__(256) add_chain(uint64_t* out, uint32_t seed, int iters) {
  uint32_t b = seed ^ (threadIdx.x * 2654435761u);
  uint32_t a[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) a[c] = b + c;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        uint32_t r;
        asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(a[c]), "v"(b));
        a[c] = r;
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
double run(K kern, int blocks, int iters, int ops_per_iter_per_lane, uint64_t* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 1u, iters);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 2u, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double ops = (double)blocks * 256 * iters * ops_per_iter_per_lane;
  return ops / (ms * 1e-3);
}

int main() {
  int blocks = 256 * 16;
  uint64_t* d; hipMalloc(&d, (size_t)blocks * 256 * 8);
  int iters = 2000;
  printf("{\"mad_u64_u32_per_s\": {\n");
  printf("  \"nch4\": %.4e,\n", run(mad_chain<4>, blocks, iters, 16 * 4, d));
  printf("  \"nch8\": %.4e,\n", run(mad_chain<8>, blocks, iters, 16 * 8, d));
  printf("  \"nch16\": %.4e,\n", run(mad_chain<16>, blocks, iters, 16 * 16, d));
  printf("  \"nch8_1wave_per_simd\": %.4e\n", run(mad_chain<8>, 256, iters, 16 * 8, d));
  printf("},\n\"mul_lo_plus_hi_pairs_per_s\": {\n");
  printf("  \"nch8\": %.4e\n", run(mulhilo_chain<8>, blocks, iters, 16 * 8, d));
  printf("},\n\"add_u32_per_s\": {\n");
  printf("  \"nch8\": %.4e\n", run(add_chain<8>, blocks, iters, 16 * 8, d));
  printf("}}\n");
  hipFree(d);
  return 0;
}
