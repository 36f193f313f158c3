/* capi_golden.c -- a plain C caller of the drop-in boundary: compiled with gcc against
 * include/ssbls.h only, linked to libssbls.so (no C++, no torch, no Python), the way the Rust shim
 * (rust/src/crypto/impls/hip.rs) or any other FFI binds it.  tests/test_capi.py builds it and the
 * GPU test feeds it the golden threshold cases.
 *
 * stdin (text):  n_jobs n_roots
 *                n_roots lines: root (64 hex)
 *                per job: t n_shares root_index, then n_shares lines: sig (192 hex) pk (96 hex) id
 * stdout:        per job: "job <j> <status> <err0> <err1> <combined sig hex or ->"
 *                then "verdicts <0/1 per share>", and "verify <0/1 per share>" from ssb_verify_batch
 * exit status:   0, or 2 when an entry point fails (the message on stderr). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ssbls.h"

static const char DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";

static int hexval(int c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}
static int read_hex(uint8_t* out, size_t n) {
  char buf[512];
  if (n * 2 >= sizeof buf || scanf("%511s", buf) != 1 || strlen(buf) != 2 * n) return -1;
  for (size_t i = 0; i < n; ++i) {
    const int a = hexval(buf[2 * i]), b = hexval(buf[2 * i + 1]);
    if (a < 0 || b < 0) return -1;
    out[i] = (uint8_t)(a * 16 + b);
  }
  return 0;
}

int main(void) {
  size_t n_jobs = 0, n_roots = 0;
  if (scanf("%zu %zu", &n_jobs, &n_roots) != 2 || !n_jobs || !n_roots) { fprintf(stderr, "bad header\n"); return 1; }
  uint8_t* roots = malloc(32 * n_roots);
  uint32_t *off = malloc(4 * (n_jobs + 1)), *t = malloc(4 * n_jobs), *jr = malloc(4 * n_jobs);
  for (size_t r = 0; r < n_roots; ++r)
    if (read_hex(roots + 32 * r, 32)) { fprintf(stderr, "bad root\n"); return 1; }
  size_t cap = 64, n = 0;
  uint8_t *sig = malloc(96 * cap), *pk = malloc(48 * cap);
  uint64_t* ids = malloc(8 * cap);
  off[0] = 0;
  for (size_t j = 0; j < n_jobs; ++j) {
    unsigned tj, nj, rj;
    if (scanf("%u %u %u", &tj, &nj, &rj) != 3) { fprintf(stderr, "bad job\n"); return 1; }
    t[j] = tj; jr[j] = rj;
    for (unsigned i = 0; i < nj; ++i, ++n) {
      if (n == cap) {
        cap *= 2;
        sig = realloc(sig, 96 * cap); pk = realloc(pk, 48 * cap); ids = realloc(ids, 8 * cap);
      }
      unsigned long long id;
      if (read_hex(sig + 96 * n, 96) || read_hex(pk + 48 * n, 48) || scanf("%llu", &id) != 1) {
        fprintf(stderr, "bad share\n");
        return 1;
      }
      ids[n] = id;
    }
    off[j + 1] = (uint32_t)n;
  }
  ssb_ctx* ctx = NULL;
  int rc = ssb_create(&ctx, 0);
  if (rc != SSB_OK) { fprintf(stderr, "ssb_create: %d\n", rc); return 2; }
  uint8_t* out = calloc(n_jobs, 96);
  int32_t* st = calloc(n_jobs, 4);
  uint64_t* err = calloc(n_jobs, 16);
  uint8_t* ver = calloc(n ? n : 1, 1);
  rc = ssb_threshold_aggregate_batch(ctx, n_jobs, off, t, sig, pk, ids, jr, n_roots, roots, (const uint8_t*)DST,
                                     strlen(DST), 0x5AFE57A4Eull, out, st, err, ver);
  if (rc != SSB_OK) { fprintf(stderr, "ssb_threshold_aggregate_batch: %d %s\n", rc, ssb_last_error(ctx)); return 2; }
  for (size_t j = 0; j < n_jobs; ++j) {
    printf("job %zu %d %llu %llu ", j, st[j], (unsigned long long)err[2 * j], (unsigned long long)err[2 * j + 1]);
    if (st[j] == SSB_DVF_OK) for (int k = 0; k < 96; ++k) printf("%02x", out[96 * j + k]);
    else printf("-");
    printf("\n");
  }
  printf("verdicts ");
  for (size_t i = 0; i < n; ++i) printf("%d", ver[i] ? 1 : 0);
  printf("\n");
  /* the same shares through the per-share verify entry point (Signature::verify) */
  uint32_t* ri = malloc(4 * (n ? n : 1));
  for (size_t j = 0; j < n_jobs; ++j)
    for (uint32_t s = off[j]; s < off[j + 1]; ++s) ri[s] = jr[j];
  uint8_t* v2 = calloc(n ? n : 1, 1);
  rc = ssb_verify_batch(ctx, n, pk, sig, ri, n_roots, roots, (const uint8_t*)DST, strlen(DST), 7, v2);
  if (rc != SSB_OK) { fprintf(stderr, "ssb_verify_batch: %d %s\n", rc, ssb_last_error(ctx)); return 2; }
  printf("verify ");
  for (size_t i = 0; i < n; ++i) printf("%d", v2[i] ? 1 : 0);
  printf("\n");
  ssb_destroy(ctx);
  free(roots); free(off); free(t); free(jr); free(sig); free(pk); free(ids); free(out); free(st); free(err);
  free(ver); free(ri); free(v2);
  return 0;
}
