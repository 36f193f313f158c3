// ssb_k_wire.hip -- kernels (gfx950): wire-format decode of partial signatures.
//
// Operators exchange partial signatures as bincode(bls::Signature) (src/node/dvfcore.rs:245-251,
// src/validation/operator.rs:108): lighthouse serialises a Signature through serde as the string
// "0x" + 192 lowercase hex digits of the 96-byte compressed point, and bincode (1.x, fixint,
// little endian) writes a string as its u64 length followed by the bytes -- 202 bytes a record:
//     [194, 0, 0, 0, 0, 0, 0, 0] "0x" h0 h1 ... h191
// k_wire_sig turns a batch of such records (record i at wire + i * stride) into the 96-byte
// compressed form the verify/combine pipeline consumes, one thread per record; HBM-bound byte
// work (202 B in, 96 B + 4 B out per record).  The G2 decompression stays in k_decode_sig.
// status[i]: 0 ok, 1 length field is not 194, 2 no "0x" prefix, 3 a non-hex digit (hex digits of
// either case decode, as hex::decode accepts them).
#include "ssb_kernels.h"

namespace ssb {
namespace k {

__device__ __forceinline__ int hexval(uint32_t c) {
  if (c >= '0' && c <= '9') return (int)(c - '0');
  c |= 0x20u;                                   // fold case
  if (c >= 'a' && c <= 'f') return (int)(c - 'a' + 10);
  return -1;
}

__global__ void SSB_LB(64) k_wire_sig(int n, const uint8_t* __restrict__ wire, size_t stride, uint8_t* __restrict__ out96,
                           int32_t* __restrict__ status, int check_point) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* r = wire + (size_t)i * stride;
  uint64_t len = 0;
  for (int k = 0; k < 8; ++k) len |= (uint64_t)r[k] << (8 * k);
  int32_t st = 0;
  if (len != 194) st = 1;
  else if (r[8] != '0' || r[9] != 'x') st = 2;
  uint8_t* o = out96 + (size_t)i * 96;
  for (int b = 0; b < 96; ++b) {
    const int hi = st ? 0 : hexval(r[10 + 2 * b]), lo = st ? 0 : hexval(r[11 + 2 * b]);
    if ((hi | lo) < 0) st = st ? st : 3;
    o[b] = (uint8_t)(((hi & 15) << 4) | (lo & 15));
  }
  if (st)   // a record that did not parse leaves zeros (no compression flag: never decodes downstream)
    for (int b = 0; b < 96; ++b) o[b] = 0;
  // bincode::deserialize::<Signature> also decompresses the point (blst uncompress: flags, x < p,
  // on the curve; infinity is a valid Signature) -- a record that fails is dropped by the reference
  // (operator.rs:108-113), so it is reported here instead of failing later as an invalid share
  if (!st && check_point) {
    uint8_t b[96];
    for (int k = 0; k < 96; ++k) b[k] = o[k];
    g2_aff pt;
    if (!(g2_decompress(pt, b) & DEC_OK)) st = 4;
  }
  status[i] = st;
}

}  // namespace k

namespace launch {
void wire_sig(hipStream_t st, int n, const uint8_t* wire, size_t stride, uint8_t* out96, int32_t* status, int check_point) {
  if (n > 0) hipLaunchKernelGGL(k::k_wire_sig, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, n, wire, stride, out96, status,
                                check_point);
}
}  // namespace launch
}  // namespace ssb
