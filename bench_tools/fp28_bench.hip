// Reduced-radix Montgomery multiplication on gfx950: 14 limbs of 28 bits, 64-bit column
// accumulators fed by v_mad_u64_u32 with no carry handling inside the product (each 56-bit partial
// product leaves 8 bits of headroom: 28 products per column < 2^61), R = 2^392.  Compared with
// the library's 12 x 32-bit FIPS product (every MAD needs a carry-propagating add).
// Output: JSON with throughput (full chip), single-wave latency, and sample (a, b, r) triples
// for a host check (bench_tools/fp28_check.py: r == a b 2^-392 mod p).
#include "../safestakeoperator_amd/csrc/ssb_field.h"
#include <cstdio>
using namespace ssb;

struct f28 { uint32_t l[14]; };
constexpr uint32_t M28 = (1u << 28) - 1;

__constant__ uint32_t P28[14];
__constant__ uint32_t P28_INV;  // -p^-1 mod 2^28

__device__ __forceinline__ void mont28(f28& r, const f28& a, const f28& b) {
  uint64_t t[15];
#pragma unroll
  for (int j = 0; j < 15; ++j) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) {
#pragma unroll
    for (int j = 0; j < 14; ++j) t[j] += (uint64_t)a.l[i] * b.l[j];
    const uint32_t m = ((uint32_t)t[0] * P28_INV) & M28;
#pragma unroll
    for (int j = 0; j < 14; ++j) t[j] += (uint64_t)m * P28[j];
    const uint64_t c = t[0] >> 28;          // low 28 bits are zero now
#pragma unroll
    for (int j = 0; j < 14; ++j) t[j] = t[j + 1];
    t[0] += c;
    t[14] = 0;
  }
  // normalise to 28-bit limbs (value < 2p), then one conditional subtraction of p
  uint32_t n[14];
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < 14; ++j) { const uint64_t v = t[j] + c; n[j] = (uint32_t)v & M28; c = v >> 28; }
  uint32_t s[14];
  int32_t br = 0;
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    const int32_t v = (int32_t)n[j] - (int32_t)P28[j] + br;
    s[j] = (uint32_t)v & M28;
    br = v >> 28;                            // 0 or -1
  }
  const bool keep = br != 0;
#pragma unroll
  for (int j = 0; j < 14; ++j) r.l[j] = keep ? n[j] : s[j];
}

__global__ void __launch_bounds__(256) k_chain28(f28* io, int iters, long long* cyc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  f28 a = io[2 * i], b = io[2 * i + 1];
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) mont28(a, a, b);
  const long long t1 = clock64();
  io[2 * i] = a;
  if (cyc && threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(256) k_chain32(fp* io, int iters, long long* cyc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  fp a = io[2 * i], b = io[2 * i + 1];
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) mp_mont_mul_fips4<12>(a.l, a.l, b.l, P_LIMBS, P_INV32);
  const long long t1 = clock64();
  io[2 * i] = a;
  if (cyc && threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

static void to28(uint32_t* o, const uint32_t* w12) {  // 12 x 32 -> 14 x 28 (value < 2^392)
  for (int k = 0; k < 14; ++k) {
    uint32_t v = 0;
    for (int b = 0; b < 28; ++b) {
      const int bit = 28 * k + b;
      if (bit < 384 && ((w12[bit >> 5] >> (bit & 31)) & 1u)) v |= 1u << b;
    }
    o[k] = v;
  }
}

int main() {
  const int nth = 256 * 2048;
  uint32_t p28[14];
  to28(p28, P_LIMBS);
  // -p^-1 mod 2^28 by Newton iteration
  uint32_t inv = 1;
  for (int k = 0; k < 5; ++k) inv *= 2u - p28[0] * inv;
  const uint32_t pinv = (0u - inv) & M28;
  hipMemcpyToSymbol(HIP_SYMBOL(P28), p28, sizeof(p28));
  hipMemcpyToSymbol(HIP_SYMBOL(P28_INV), &pinv, 4);
  f28* h = new f28[2 * nth];
  fp* h32 = new fp[2 * nth];
  uint64_t x = 88172645463325252ull;
  for (int i = 0; i < 2 * nth; ++i) {
    uint32_t w[12];
    for (int k = 0; k < 12; ++k) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; w[k] = (uint32_t)x; }
    w[11] &= 0x0fffffffu;                   // < p
    to28(h[i].l, w);
    for (int k = 0; k < 12; ++k) h32[i].l[k] = w[k];
  }
  f28* d; fp* d32; long long* cyc;
  hipMalloc(&d, sizeof(f28) * 2 * nth); hipMalloc(&d32, sizeof(fp) * 2 * nth); hipMalloc(&cyc, 8 * 4096);
  hipMemcpy(d, h, sizeof(f28) * 2 * nth, hipMemcpyHostToDevice);
  hipMemcpy(d32, h32, sizeof(fp) * 2 * nth, hipMemcpyHostToDevice);
  // samples: one multiplication on the first 4 threads
  hipLaunchKernelGGL(k_chain28, dim3(nth / 256), dim3(256), 0, 0, d, 1, (long long*)nullptr);
  f28* r = new f28[8];
  hipMemcpy(r, d, sizeof(f28) * 8, hipMemcpyDeviceToHost);
  printf("{\"p_inv28\": %u,\n \"samples\": [", pinv);
  for (int s = 0; s < 4; ++s) {
    auto hx = [](const f28& v) { static char buf[200]; char* q = buf; for (int k = 13; k >= 0; --k) q += sprintf(q, "%07x", v.l[k]); return buf; };
    printf("%s[\"%s\",", s ? ", " : "", hx(h[2 * s]));
    printf("\"%s\",", hx(h[2 * s + 1]));
    printf("\"%s\"]", hx(r[2 * s]));
  }
  printf("],\n");
  hipMemcpy(d, h, sizeof(f28) * 2 * nth, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](const char* nm, bool r28) {
    const int iters = 256;
    for (int pass = 0; pass < 2; ++pass) {
      hipEventRecord(e0);
      if (r28) hipLaunchKernelGGL(k_chain28, dim3(nth / 256), dim3(256), 0, 0, d, pass ? iters : 8, (long long*)nullptr);
      else hipLaunchKernelGGL(k_chain32, dim3(nth / 256), dim3(256), 0, 0, d32, pass ? iters : 8, (long long*)nullptr);
      hipEventRecord(e1); hipEventSynchronize(e1);
    }
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double muls = (double)nth * iters;
    printf(" \"%s_Gmul_per_s\": %.2f,\n", nm, muls / ms / 1e6);
    const int li = 2048;
    if (r28) hipLaunchKernelGGL(k_chain28, dim3(1), dim3(64), 0, 0, d, li, cyc);
    else hipLaunchKernelGGL(k_chain32, dim3(1), dim3(64), 0, 0, d32, li, cyc);
    hipDeviceSynchronize();
    long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf(" \"%s_1wave_clk_per_mul\": %.1f,\n", nm, (double)c / li);
  };
  run("fips4_12x32", false);
  run("mont_14x28", true);
  printf(" \"end\": 0}\n");
  return 0;
}
