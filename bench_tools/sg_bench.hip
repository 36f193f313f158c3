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

// V4: P re-read from global memory at each of the 5 additions (pointer laundered through an empty
// asm so the loads are not hoisted into 48 live registers): fewer spills at two waves per SIMD
template <class F> SSB_INL void mul_x_abs_gmem(jac<F>& r, const aff<F>* gp) {
  jac<F> acc; jac_from_aff(acc, *gp);
  for (int i = 62; i >= 0; --i) {
    jac_dbl_inl(acc, acc);
    if ((BLS_X_ABS >> i) & 1ull) {
      const aff<F>* q = gp;
      asm volatile("" : "+v"(q));
      const aff<F> pq = *q;
      jac_add_aff_inl(acc, acc, pq);
    }
  }
  r = acc;
}
// V5: low-pressure mixed addition whose exceptional case (acc == +-P: P has order dividing a
// 64-bit prefix of |x| +- 1, so P is not in G2) answers "not in the subgroup" at once instead of
// carrying an inlined doubling: 61 VGPR spills at two waves per SIMD instead of 146
SSB_INL bool add_aff_sg(g2_jac& r, const g2_jac& p, const g2_aff& q) {
  if (jac_is_inf(p)) { jac_from_aff(r, q); return true; }
  fp2 Z1Z1, H, rr, HH, z3, t;
  fp2_sqr(Z1Z1, p.z);
  fp2_mul(H, q.x, Z1Z1); fp2_sub(H, H, p.x);
  fp2_mul(t, q.y, p.z); fp2_mul(t, t, Z1Z1); fp2_sub(rr, t, p.y);
  if (fp2_is_zero(H)) return false;
  fp2_dbl(rr, rr);
  fp2_sqr(HH, H);
  fp2_add(z3, p.z, H); fp2_sqr(z3, z3); fp2_sub(z3, z3, Z1Z1); fp2_sub(z3, z3, HH);
  fp2 I, J, V;
  fp2_dbl(I, HH); fp2_dbl(I, I);
  fp2_mul(J, H, I);
  fp2_mul(V, p.x, I);
  fp2 x3, y3;
  fp2_sqr(x3, rr); fp2_sub(x3, x3, J); fp2_dbl(t, V); fp2_sub(x3, x3, t);
  fp2_sub(t, V, x3); fp2_mul(y3, rr, t); fp2_mul(t, p.y, J); fp2_dbl(t, t); fp2_sub(y3, y3, t);
  r.x = x3; r.y = y3; r.z = z3;
  return true;
}
__global__ void __attribute__((amdgpu_flat_work_group_size(1, 64), amdgpu_waves_per_eu(2)))
k_sg5(int n, const g2_aff* __restrict__ pts, uint32_t* __restrict__ out) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const g2_aff p = pts[s];
  uint32_t res = 1;
  if (!p.inf) {
    g2_jac acc; jac_from_aff(acc, p);
    for (int i = 62; i >= 0 && res; --i) {
      jac_dbl_inl(acc, acc);
      if ((BLS_X_ABS >> i) & 1ull) res = add_aff_sg(acc, acc, p) ? 1u : 0u;
    }
    if (res) { jac_neg(acc, acc); g2_aff ps; g2_psi_aff(ps, p); res = jac_eq_aff(acc, ps) ? 1u : 0u; }
  }
  out[s] = res;
}
SSB_INL bool in_subgroup_gmem(const g2_aff* gp) {
  if (gp->inf) return true;
  g2_jac xp; mul_x_abs_gmem(xp, gp); jac_neg(xp, xp);
  const g2_aff* q = gp;
  asm volatile("" : "+v"(q));
  g2_aff ps; g2_psi_aff(ps, *q);
  return jac_eq_aff(xp, ps);
}
__global__ void __attribute__((amdgpu_flat_work_group_size(1, 64), amdgpu_waves_per_eu(2)))
k_sg4(int n, const g2_aff* __restrict__ pts, uint32_t* __restrict__ out) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  out[s] = in_subgroup_gmem(pts + s) ? 1u : 0u;
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
    for (int v = 0; v < 6; ++v) {
      auto go = [&] {
        if (v == 0) hipLaunchKernelGGL(k_sg<0>, dim3(n / 64), dim3(64), 0, 0, n, d, o0);
        else if (v == 1) hipLaunchKernelGGL(k_sg<1>, dim3(n / 64), dim3(64), 0, 0, n, d, o1);
        else if (v == 2) hipLaunchKernelGGL(k_sg2<1>, dim3(n / 64), dim3(64), 0, 0, n, d, ov);
        else if (v == 3) hipLaunchKernelGGL(k_sg2<0>, dim3(n / 64), dim3(64), 0, 0, n, d, ov);
        else if (v == 4) hipLaunchKernelGGL(k_sg4, dim3(n / 64), dim3(64), 0, 0, n, d, ov);
        else hipLaunchKernelGGL(k_sg5, dim3(n / 64), dim3(64), 0, 0, n, d, ov);
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
    std::vector<uint32_t> c(n);
    hipMemcpy(c.data(), ov, n * 4, hipMemcpyDeviceToHost);   // last writer: V5
    int same = 0, ones = 0, same5 = 0;
    for (int i = 0; i < n; ++i) { same += a[i] == b[i]; ones += a[i]; same5 += a[i] == c[i]; }
    printf(", \"n%d_agree\": %d, \"n%d_v5_agree\": %d, \"n%d_in_group\": %d", n, same, n, same5, n, ones);
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
