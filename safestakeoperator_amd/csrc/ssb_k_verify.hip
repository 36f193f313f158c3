// ssb_k_verify.hip -- kernels (gfx950): share map, decompression, flags, verdicts, per-root segment sums.
// Launched from ssbls.hip (declarations in ssb_kernels.h); one TU per kernel family so the
// library compiles in parallel.
#include "ssb_kernels.h"
#include "ssb_blocks.h"

namespace ssb {
namespace k {

// share -> job and share -> root, one thread per share (share_lookup, ssb_blocks.h); the fused
// one-stream path does the same lookups inside k_decode_count instead of a launch of its own
__global__ void k_share_map(int n_jobs, uint32_t n_shares, const uint32_t* __restrict__ off, const uint32_t* __restrict__ tt,
                            const uint32_t* __restrict__ job_root, uint32_t* __restrict__ share_job,
                            uint32_t* __restrict__ share_root) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_shares) return;
  const job_map jm{n_jobs, n_shares, off, tt, job_root, share_job, share_root};
  uint32_t j, r;
  share_lookup(s, jm, j, r);
  share_job[s] = j;
  if (share_root) share_root[s] = r;
}
__global__ void SSB_LB(64) k_decode(int n, const uint8_t* __restrict__ sig96,
                                               const uint8_t* __restrict__ pk48, int group_check,
                                               g2_aff* __restrict__ sig_aff, g1_aff* __restrict__ pk_aff,
                                               uint32_t* __restrict__ flags) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  uint8_t b[96], c[48];
  for (int k = 0; k < 96; ++k) b[k] = sig96[96 * (size_t)s + k];
  if (pk48) for (int k = 0; k < 48; ++k) c[k] = pk48[48 * (size_t)s + k];
  g2_aff sig; g1_aff pk;
  const uint32_t fl = unit_decode(sig, pk, b, pk48 ? c : nullptr, group_check);
  sig_aff[s] = sig;
  if (pk48) pk_aff[s] = pk;
  flags[s] = fl;
}
__global__ void SSB_LB2(64) k_decode2(int n, const uint8_t* __restrict__ sig96, const uint8_t* __restrict__ pk48,
                                                g2_aff* __restrict__ sig_aff, g1_aff* __restrict__ pk_aff,
                                                uint32_t* __restrict__ sflags, uint32_t* __restrict__ pflags) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n) {
    uint8_t b[96];
    for (int k = 0; k < 96; ++k) b[k] = sig96[96 * (size_t)g + k];
    g2_aff sig;
    sflags[g] = unit_decode_sig(sig, b);
    sig_aff[g] = sig;
  } else if (g < 2 * n) {
    const int s = g - n;
    uint8_t b[48];
    for (int k = 0; k < 48; ++k) b[k] = pk48[48 * (size_t)s + k];
    g1_aff pk;
    pflags[s] = unit_decode_pk(pk, b);
    pk_aff[s] = pk;
  }
}
// decoded-public-key path (ssb_pk_cache_set): n lanes decode the signatures, the public keys are
// gathered from the context's table of points decompressed once (lighthouse's PublicKey holds the
// decompressed point too: the reference never decompresses a key per verification)
__global__ void SSB_LB2(64) k_decode_sig(int n, const uint8_t* __restrict__ sig96, g2_aff* __restrict__ sig_aff,
                                                   uint32_t* __restrict__ sflags) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  uint8_t b[96];
  for (int k = 0; k < 96; ++k) b[k] = sig96[96 * (size_t)g + k];
  g2_aff sig;
  sflags[g] = unit_decode_sig(sig, b);
  sig_aff[g] = sig;
}
__global__ void SSB_LB(256) k_pk_gather(int n, const uint32_t* __restrict__ pk_index, uint32_t n_cache,
                                                   const g1_aff* __restrict__ cache_aff, const uint32_t* __restrict__ cache_flags,
                                                   g1_aff* __restrict__ pk_aff, uint32_t* __restrict__ pflags) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const uint32_t i = pk_index[s];
  if (i < n_cache) { pk_aff[s] = cache_aff[i]; pflags[s] = cache_flags[i]; }
  else pflags[s] = 0u;  // out-of-range index: the share cannot verify
}
__global__ void SSB_LB2(64) k_decode_pk(int n, const uint8_t* __restrict__ pk48, g1_aff* __restrict__ pk_aff,
                                                  uint32_t* __restrict__ pflags) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  uint8_t b[48];
  for (int k = 0; k < 48; ++k) b[k] = pk48[48 * (size_t)s + k];
  g1_aff pk;
  pflags[s] = unit_decode_pk(pk, b);
  pk_aff[s] = pk;
}
// the key cache's precomputed bases for the merged G1 MSM: pow[PKPOW_W s + w] = [2^(4 w)] pk_s (keys that
// did not decode to a usable point are never read: their shares are no candidates)
__global__ void SSB_LB2(64) k_pk_pow(int n, const g1_aff* __restrict__ pk_aff, const uint32_t* __restrict__ pflags,
                                     g1_aff* __restrict__ pow) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  g1_aff* o = pow + (size_t)s * PKPOW_W;
  const g1_aff a = pk_aff[s];
  o[0] = a;
  const uint32_t f = pflags[s];
  if (!(f & DEC_OK) || (f & DEC_INF)) {
    for (uint32_t w = 1; w < PKPOW_W; ++w) o[w] = a;
    return;
  }
  g1_jac p;
  jac_from_aff(p, a);
  for (uint32_t w = 1; w < PKPOW_W; ++w) {
    for (int q = 0; q < 4; ++q) jac_dbl(p, p);
    g1_aff t;
    jac_to_aff(t, p);
    o[w] = t;
  }
}
__global__ void k_flags(int n, const uint32_t* __restrict__ sflags, const uint32_t* __restrict__ pflags,
                        const uint32_t* __restrict__ gflags, const uint32_t* __restrict__ share_root, uint32_t n_roots,
                        uint32_t* __restrict__ flags) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  uint32_t f = combine_flags(sflags[s], pflags[s], gflags[s]);
  if (share_root[s] >= n_roots) f &= ~FLAG_CANDIDATE;  // no H(root): the share cannot verify
  flags[s] = f;
}

// ---- per-root RLC sums: counting sort of the shares by root, then one block per (root, group) ----
__global__ void k_root_hist(int n, int n_roots, const uint32_t* __restrict__ share_root, uint32_t* __restrict__ cnt) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < n && share_root[s] < (uint32_t)n_roots) atomicAdd(&cnt[share_root[s]], 1u);
}
__global__ void k_root_scan(int n_roots, const uint32_t* __restrict__ cnt, uint32_t* __restrict__ start,
                            uint32_t* __restrict__ cursor) {
  if (threadIdx.x != 0) return;
  uint32_t acc = 0;
  for (int r = 0; r < n_roots; ++r) { start[r] = acc; cursor[r] = acc; acc += cnt[r]; }
}
__global__ void k_root_scatter(int n, int n_roots, const uint32_t* __restrict__ share_root, uint32_t* __restrict__ cursor,
                               uint32_t* __restrict__ perm) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < n && share_root[s] < (uint32_t)n_roots) perm[atomicAdd(&cursor[share_root[s]], 1u)] = (uint32_t)s;
}
// blocks [0, n_roots): S_r = sum r_i pk_i over the candidate shares of root r (G1);
// blocks [n_roots, 2 n_roots): T_r = sum r_i sig_i (G2).  Affine outputs (infinity if none).
// The summation order inside a segment is whatever the scatter produced: the affine sum is the
// same group element either way, and jac_add is exact for every input.
__global__ void SSB_LB(SEG_THREADS) k_sum_seg(int n_roots, const uint32_t* __restrict__ start,
                                                         const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ perm,
                                                         const uint32_t* __restrict__ flags, const g1_jac* __restrict__ rpk,
                                                         const g2_jac* __restrict__ rsig, g1_aff* __restrict__ s1,
                                                         g2_aff* __restrict__ s2) {
  __shared__ g2_jac sh2[SEG_THREADS];
  g1_jac* sh1 = (g1_jac*)sh2;
  const bool g1 = (int)blockIdx.x < n_roots;
  const int r = g1 ? blockIdx.x : blockIdx.x - n_roots;
  const uint32_t b = start[r], e = b + cnt[r];
  if (g1) {
    g1_jac acc; jac_set_inf(acc);
    for (uint32_t k = b + threadIdx.x; k < e; k += SEG_THREADS) {
      const uint32_t s = perm[k];
      if (flags[s] & FLAG_CANDIDATE) jac_add(acc, acc, rpk[s]);
    }
    sh1[threadIdx.x] = acc;
    __syncthreads();
    for (int w = SEG_THREADS / 2; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) { g1_jac o = sh1[threadIdx.x + w]; jac_add(acc, acc, o); sh1[threadIdx.x] = acc; }
      __syncthreads();
    }
    if (threadIdx.x == 0) { g1_aff a; jac_to_aff(a, acc); s1[r] = a; }
  } else {
    g2_jac acc; jac_set_inf(acc);
    for (uint32_t k = b + threadIdx.x; k < e; k += SEG_THREADS) {
      const uint32_t s = perm[k];
      if (flags[s] & FLAG_CANDIDATE) jac_add(acc, acc, rsig[s]);
    }
    sh2[threadIdx.x] = acc;
    __syncthreads();
    for (int w = SEG_THREADS / 2; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) { g2_jac o = sh2[threadIdx.x + w]; jac_add(acc, acc, o); sh2[threadIdx.x] = acc; }
      __syncthreads();
    }
    if (threadIdx.x == 0) { g2_aff a; jac_to_aff(a, acc); s2[r] = a; }
  }
}

}  // namespace k
}  // namespace ssb
