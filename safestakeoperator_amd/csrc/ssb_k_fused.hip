// ssb_k_fused.hip -- kernels (gfx950) of the one-stream slot path that carry independent stages of
// a batch in one launch (ssb_blocks.h): the counting sort of the MSM entries rides along the
// decode and the subgroup checks instead of standing between them as ten small launches.
// Launched from ssbls.hip (declarations in ssb_kernels.h).
#include "ssb_kernels.h"
#include "ssb_blocks.h"

namespace ssb {
namespace k {

// blocks [0, nz): zero the sort's counts (and the order bins); then one lane per root: the hash's
// expand_message_xmd + the two field elements (k_h2c_u)
__global__ void SSB_LB(64) k_prep_fused(uint32_t nz, uint32_t K, uint32_t* __restrict__ cnt, uint32_t* __restrict__ tickets,
                                        uint32_t ntk, int n_roots, const uint8_t* __restrict__ roots, dst_arg dst,
                                        fp2* __restrict__ u) {
  if (blockIdx.x == 0) for (uint32_t i = threadIdx.x; i < ntk; i += 64) tickets[i] = 0u;
  if (blockIdx.x < nz) {
    for (uint32_t x = blockIdx.x * 64 * 16 + threadIdx.x; x < (blockIdx.x + 1) * 64 * 16 && x < K; x += 64) cnt[x] = 0u;
    return;
  }
  const int i = (blockIdx.x - nz) * 64 + threadIdx.x;
  if (i >= n_roots) return;
  uint8_t m[32];
  for (int k = 0; k < 32; ++k) m[k] = roots[32 * i + k];
  fp2 u0, u1;
  h2c_field(u0, u1, m, dst.b, dst.len, 32);
  u[2 * i] = u0;
  u[2 * i + 1] = u1;
}

// One wave: start[] = cur[] = exclusive scan of cnt[0..K), then the bucket order (within each MSM's
// key range, by count, largest first -- the k_order_* kernels' order).  sh: 64 + 512 words of LDS.
SSB_INL void sort_scan_wave(uint32_t K, uint32_t K2, uint32_t* __restrict__ cnt, uint32_t* __restrict__ start,
                            uint32_t* __restrict__ cur, uint32_t* __restrict__ order, uint32_t* sh) {
  uint32_t* bins = sh + 64;
  const int t = threadIdx.x;
  const uint32_t per = (K + 63) / 64, k0 = t * per, k1 = k0 + per < K ? k0 + per : K;
  for (int b = t; b < 512; b += 64) bins[b] = 0u;
  uint32_t sum = 0;
  for (uint32_t k = k0; k < k1; ++k) sum += cnt[k];
  sh[t] = sum;
  __syncthreads();
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = t >= off ? sh[t - off] : 0u;
    __syncthreads();
    sh[t] += o;
    __syncthreads();
  }
  uint32_t run = sh[t] - sum;
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t c = cnt[k];
    start[k] = run; cur[k] = run; run += c;
    atomicAdd(&bins[(k >= K2 ? 256u : 0u) + 255u - (c < 255u ? c : 255u)], 1u);
  }
  __syncthreads();
  // exclusive scan of the 512 bins, eight per lane
  uint32_t v[8], tot = 0;
  for (int q = 0; q < 8; ++q) { v[q] = bins[8 * t + q]; tot += v[q]; }
  __syncthreads();
  sh[t] = tot;
  __syncthreads();
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = t >= off ? sh[t - off] : 0u;
    __syncthreads();
    sh[t] += o;
    __syncthreads();
  }
  uint32_t base = sh[t] - tot;
  for (int q = 0; q < 8; ++q) { bins[8 * t + q] = base; base += v[q]; }
  __syncthreads();
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t c = cnt[k];
    order[atomicAdd(&bins[(k >= K2 ? 256u : 0u) + 255u - (c < 255u ? c : 255u)], 1u)] = k;
    cnt[k] = 0u;   // dead from here (the buckets read the cursors): clean for the slot's next batch
  }
}

// blocks [0, nbd): signature decode; [nbd, 2 nbd): public keys (gathered from the cache, or
// decoded); [2 nbd, 3 nbd): the sort's count pass
#ifndef SSB_DC_WAVES   // experiment knob: waves per SIMD the decode launch is built for
#define SSB_DC_WAVES 2
#endif
// (the attribute's minimum alone lets the compiler trade registers for a third wave: 142 VGPRs and a
// spilling sqrt table; SSB_DC_WAVES_MAX caps the waves so the registers stay)
#ifdef SSB_DC_WAVES_MAX
#define SSB_DC_ATTR amdgpu_waves_per_eu(SSB_DC_WAVES, SSB_DC_WAVES_MAX)
#else
#define SSB_DC_ATTR amdgpu_waves_per_eu(SSB_DC_WAVES)
#endif
// (blocks [3 nbd, 3 nbd + nbu): the hash's first stage, one lane per root, when the slot's counts
// and tickets are already clean -- then no prep launch stands in front of the decode)
// the roles out of line: each gets its own register allocation (inlined, the hash's and the decode's
// demands were merged into one allocation for every lane of the launch, and all of them spilled)
// a record of B bytes (a multiple of 16) into b: 16-byte loads when the array is 16-byte aligned (the
// device buffers and workspaces are), else bytes -- one dwordx4 load per 16 bytes instead of 16
// byte loads (round 5: the decode launch's instruction count and reported traffic)
template <int B>
SSB_INL void load_record(uint8_t* __restrict__ b, const uint8_t* __restrict__ rec, const uint8_t* __restrict__ base) {
  if (((uintptr_t)base & 15u) == 0) {
    const uint4* q = (const uint4*)rec;
#pragma unroll
    for (int k = 0; k < B / 16; ++k) ((uint4*)b)[k] = q[k];
  } else {
    for (int k = 0; k < B; ++k) b[k] = rec[k];
  }
}
// (out of line, the DST by value: inlined, the kernel copied the 256-byte kernel argument into its
// private frame at entry for the role's pointer -- in every wave of every role, 256 B of scratch
// writes per share: most of the launch's HBM writes, round 5 PMC)
SSB_FN void dc_hash_role(int i, const uint8_t* __restrict__ roots, const dst_arg dst, fp2* __restrict__ u) {
  uint8_t m[32];
  for (int k = 0; k < 32; ++k) m[k] = roots[32 * i + k];
  fp2 u0, u1;
  h2c_field(u0, u1, m, dst.b, dst.len, 32);
  u[2 * i] = u0;
  u[2 * i + 1] = u1;
}
SSB_ROLE void dc_count_role(int s, const job_map& jm, const uint32_t* __restrict__ share_root, const rlc_key& key,
                          const msm_cfg& c2, const msm_cfg& c1, uint32_t* __restrict__ cnt) {
  uint32_t g;
  if (jm.n_jobs) { uint32_t j; share_lookup((uint32_t)s, jm, j, g); }   // (the decode blocks store it)
  else g = share_root[s];
  msm_sort_lane_root<false>(s, g, key, c2, c1, cnt, (uint32_t*)nullptr);
}
SSB_ROLE void dc_sig_role(int s, const uint8_t* __restrict__ sig96, g2_aff* __restrict__ sig_aff, uint32_t* __restrict__ sflags,
                        const job_map& jm) {
  if (jm.n_jobs) {   // share -> (job, root) for the later launches (k_share_map's work)
    uint32_t j, r;
    share_lookup((uint32_t)s, jm, j, r);
    jm.share_job[s] = j;
    jm.share_root[s] = r;
  }
  uint8_t b[96];
  load_record<96>(b, sig96 + 96 * (size_t)s, sig96);
  g2_aff sig;
  sflags[s] = unit_decode_sig(sig, b);
  sig_aff[s] = sig;
}
SSB_ROLE void dc_pk_role(int s, const uint8_t* __restrict__ pk48, g1_aff* __restrict__ pk_aff, uint32_t* __restrict__ pflags) {
  uint8_t b[48];
  load_record<48>(b, pk48 + 48 * (size_t)s, pk48);
  g1_aff pk;
  pflags[s] = unit_decode_pk(pk, b);
  pk_aff[s] = pk;
}
template <bool CACHED>
__global__ void __attribute__((amdgpu_flat_work_group_size(1, 64), SSB_DC_ATTR)) k_decode_count(int n, uint32_t nbd, const uint8_t* __restrict__ sig96,
                                           const uint8_t* __restrict__ pk48, const uint32_t* __restrict__ pk_index,
                                           uint32_t n_cache, const g1_aff* __restrict__ cache_aff,
                                           const uint32_t* __restrict__ cache_flags, g2_aff* __restrict__ sig_aff,
                                           g1_aff* __restrict__ pk_aff, uint32_t* __restrict__ sflags,
                                           uint32_t* __restrict__ pflags, rlc_key key, const uint32_t* __restrict__ share_root,
                                           msm_cfg c2, msm_cfg c1, uint32_t* __restrict__ cnt, uint32_t K,
                                           uint32_t* __restrict__ start, uint32_t* __restrict__ cur,
                                           uint32_t* __restrict__ order, uint32_t* __restrict__ tickets,
                                           int n_roots, const uint8_t* __restrict__ roots, dst_arg dst,
                                           fp2* __restrict__ u, job_map jm) {
  const uint32_t part = blockIdx.x / nbd;
  if (part >= 3) {
    const int i = (int)(blockIdx.x - 3 * nbd) * 64 + threadIdx.x;
    if (i < n_roots) dc_hash_role(i, roots, dst, u);
    return;
  }
  const int s = (blockIdx.x - part * nbd) * 64 + threadIdx.x;
  if (part == 2) {   // count pass; the last count block to finish runs the scans
    __shared__ uint32_t sh[64 + 512];
    __shared__ uint32_t last;
    if (s < n) dc_count_role(s, jm, share_root, key, c2, c1, cnt);
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      last = atomicAdd(&tickets[0], 1u) == nbd - 1 ? 1u : 0u;
    }
    __syncthreads();
    if (last) {
      __threadfence();
      sort_scan_wave(K, c1.base, cnt, start, cur, order, sh);
      if (threadIdx.x == 0) tickets[0] = 0u;   // every count block has passed: clean for the next batch
    }
    return;
  }
  if (s >= n) return;
  if (part == 0) {
    dc_sig_role(s, sig96, sig_aff, sflags, jm);
  } else if (part == 1) {
    if (CACHED) {
      const uint32_t i = pk_index[s];
      if (i < n_cache) { pk_aff[s] = cache_aff[i]; pflags[s] = cache_flags[i]; }
      else pflags[s] = 0u;   // out-of-range index: the share cannot verify
    } else {
      dc_pk_role(s, pk48, pk_aff, pflags);
    }
  }
}

}  // namespace k

namespace launch {
using namespace ssb::k;

void prep_fused(hipStream_t st, const fused_sort& fs, int n_roots, const uint8_t* roots, const dst_arg& dst, const h2c_ws& hw) {
  const uint32_t nz = (fs.K + 64 * 16 - 1) / (64 * 16), nu = (uint32_t)(n_roots + 63) / 64;
  hipLaunchKernelGGL(k_prep_fused, dim3(nz + nu), dim3(64), 0, st, nz, fs.K, fs.cnt, fs.tickets, fs.ntk, n_roots, roots, dst,
                     hw.u);
}

void decode_count(hipStream_t st, int n, const uint8_t* sig96, const uint8_t* pk48, const uint32_t* pk_index,
                  uint32_t n_cache, const g1_aff* cache_aff, const uint32_t* cache_flags, g2_aff* sig_aff, g1_aff* pk_aff,
                  uint32_t* sflags, uint32_t* pflags, const fused_sort& fs, int n_roots, const uint8_t* roots,
                  const dst_arg* dst, const h2c_ws* hw) {
  if (n <= 0) return;
  const uint32_t nbd = (uint32_t)(n + 63) / 64;
  const bool u = dst && hw && n_roots > 0;
  const uint32_t nbu = u ? (uint32_t)(n_roots + 63) / 64 : 0u;
  const dst_arg d = u ? *dst : dst_arg{};
  fp2* uo = u ? hw->u : nullptr;
  if (pk_index)
    hipLaunchKernelGGL(k_decode_count<true>, dim3(3 * nbd + nbu), dim3(64), 0, st, n, nbd, sig96, pk48, pk_index, n_cache,
                       cache_aff, cache_flags, sig_aff, pk_aff, sflags, pflags, fs.key, fs.share_root, fs.c2, fs.c1, fs.cnt,
                       fs.K, fs.start, fs.cur, fs.order, fs.tickets, u ? n_roots : 0, roots, d, uo, fs.jm);
  else
    hipLaunchKernelGGL(k_decode_count<false>, dim3(3 * nbd + nbu), dim3(64), 0, st, n, nbd, sig96, pk48, pk_index, n_cache,
                       cache_aff, cache_flags, sig_aff, pk_aff, sflags, pflags, fs.key, fs.share_root, fs.c2, fs.c1, fs.cnt,
                       fs.K, fs.start, fs.cur, fs.order, fs.tickets, u ? n_roots : 0, roots, d, uo, fs.jm);
}


}  // namespace launch
}  // namespace ssb
