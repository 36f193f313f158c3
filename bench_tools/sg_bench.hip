// Subgroup-check kernel variants (psi(P) == [x]P on G2), single lane per point: time per launch at
// C2 size (16,384 points = 256 waves) and at full chip (65,536), and agreement of the verdicts.
//   V0: the engine's g2_in_subgroup (out-of-line additions)     V1: everything inlined
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o bench_tools/sg_bench bench_tools/sg_bench.hip
#include "../safestakeoperator_amd/csrc/ssb_units.h"
#include <cstdio>
#include <vector>
using namespace ssb;

template <class F> SSB_INL void mul_x_abs_aff_inl(jac<F>& r, const aff<F>& p) {
  jac<F> acc; jac_from_aff(acc, p);
  for (int i = 62; i >= 0; --i) {
    jac_dbl_inl(acc, acc);
    if ((BLS_X_ABS >> i) & 1ull) jac_add_aff_inl(acc, acc, p);
  }
  r = acc;
}
SSB_INL bool in_subgroup_inl(const g2_aff& p) {
  if (p.inf) return true;
  g2_jac xp; mul_x_abs_aff_inl(xp, p); jac_neg(xp, xp);
  g2_aff ps; g2_psi_aff(ps, p);
  return jac_eq_aff(xp, ps);
}

template <int V>
__global__ void SSB_LB(64) k_sg(int n, const g2_aff* __restrict__ pts, uint32_t* __restrict__ out) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const g2_aff p = pts[s];
  bool r;
  if (V == 0) r = g2_in_subgroup(p);
  else r = in_subgroup_inl(p);
  out[s] = r ? 1u : 0u;
}
// V2 / V3: the same bodies capped at 256 registers (VGPR + AGPR): two waves per SIMD
template <int V>
__global__ void __attribute__((amdgpu_flat_work_group_size(1, 64), amdgpu_waves_per_eu(2)))
k_sg2(int n, const g2_aff* __restrict__ pts, uint32_t* __restrict__ out) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const g2_aff p = pts[s];
  bool r;
  if (V == 0) r = g2_in_subgroup(p);
  else r = in_subgroup_inl(p);
  out[s] = r ? 1u : 0u;
}

int main() {
  const int NMAX = 262144;
  // points: multiples of the hash of a fixed root (in G2) and raw isogeny images (not in G2)
  std::vector<g2_aff> h(NMAX);
  uint8_t m[32] = {0};
  const char* dst = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
  g2_aff base; hash_to_g2(base, m, (const uint8_t*)dst, 43);
  g2_jac acc; jac_from_aff(acc, base);
  for (int i = 0; i < 64; ++i) { jac_to_aff(h[i], acc); jac_add_aff(acc, acc, base); }
  for (int i = 64; i < NMAX; ++i) h[i] = h[i % 64];
  { uint8_t uni[256]; expand_message_xmd_256(uni, m, (const uint8_t*)dst, 43);
    fp2 u; fp_from_be64_mod(u.c0, uni); fp_from_be64_mod(u.c1, uni + 64);
    fp2 x, y; map_to_curve_sswu(x, y, u); g2_aff raw; iso3_map(raw, x, y);
    for (int i = 5; i < NMAX; i += 97) h[i] = raw; }
  g2_aff* d; uint32_t *o0, *o1, *ov;
  hipMalloc(&d, NMAX * sizeof(g2_aff)); hipMalloc(&o0, NMAX * 4); hipMalloc(&o1, NMAX * 4); hipMalloc(&ov, NMAX * 4);
  hipMemcpy(d, h.data(), NMAX * sizeof(g2_aff), hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  printf("{");
  bool first = true;
  for (int n : {16384, 65536, 131072, 262144}) {
    for (int v = 0; v < 4; ++v) {
      auto go = [&] {
        if (v == 0) hipLaunchKernelGGL(k_sg<0>, dim3(n / 64), dim3(64), 0, 0, n, d, o0);
        else if (v == 1) hipLaunchKernelGGL(k_sg<1>, dim3(n / 64), dim3(64), 0, 0, n, d, o1);
        else if (v == 2) hipLaunchKernelGGL(k_sg2<1>, dim3(n / 64), dim3(64), 0, 0, n, d, ov);
        else hipLaunchKernelGGL(k_sg2<0>, dim3(n / 64), dim3(64), 0, 0, n, d, ov);
      };
      go(); hipDeviceSynchronize();
      float best = 1e9;
      for (int r = 0; r < 5; ++r) {
        hipEventRecord(e0); go(); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1); best = ms < best ? ms : best;
      }
      printf("%s\"V%d_n%d_ms\": %.4f", first ? "" : ", ", v, n, best);
      first = false;
    }
    std::vector<uint32_t> a(n), b(n);
    hipMemcpy(a.data(), o0, n * 4, hipMemcpyDeviceToHost); hipMemcpy(b.data(), o1, n * 4, hipMemcpyDeviceToHost);
    int same = 0, ones = 0;
    for (int i = 0; i < n; ++i) { same += a[i] == b[i]; ones += a[i]; }
    printf(", \"n%d_agree\": %d, \"n%d_in_group\": %d", n, same, n, ones);
  }
  // cross-stream concurrency: K streams, each a chain of R launches of 16,384 points (one C2
  // batch's subgroup checks); ideal = the time of one K*R*16384-point launch
  {
    const int n = 16384, R = 8;
    hipStream_t ss[24];
    for (int k = 0; k < 24; ++k) hipStreamCreateWithFlags(&ss[k], hipStreamNonBlocking);
    for (int K : {1, 2, 4, 8, 12, 14, 16, 20}) {
      float best = 1e9;
      for (int rep = 0; rep < 3; ++rep) {
        hipDeviceSynchronize();
        hipEventRecord(e0, 0);
        for (int k = 0; k < K; ++k) hipStreamWaitEvent(ss[k], e0, 0);
        for (int r = 0; r < R; ++r)
          for (int k = 0; k < K; ++k)
            hipLaunchKernelGGL(k_sg2<1>, dim3(n / 64), dim3(64), 0, ss[k], n, d + (size_t)(k % 16) * n, ov + (size_t)(k % 16) * n);
        for (int k = 0; k < K; ++k) { hipEvent_t e; hipEventCreate(&e); hipEventRecord(e, ss[k]); hipStreamWaitEvent(0, e, 0); }
        hipEventRecord(e1, 0); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1); best = ms < best ? ms : best;
      }
      printf(", \"streams%d_ms\": %.3f, \"streams%d_ms_per_launch\": %.4f", K, best, K, best / (K * R));
    }
  }
  printf("}\n");
  return 0;
}
