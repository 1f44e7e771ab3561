/*
 * abi_host.c — TEST DRIVER: a plain C host program on the C-ABI (what the cgo binding in
 * go/gpdecode does), with no Python or PyTorch in the process, so libgpd.so runs on
 * /opt/rocm's HIP runtime exactly as it would under Go.
 *
 *   abi_host BATCH_FILE
 *
 * BATCH_FILE: u64 data_len, u64 n, u32 decoders, u32 options, data[data_len], u32 offset[n],
 * u32 caplen[n].  The batch is decoded three ways and every output word is compared:
 *   1. gpd_decode on device buffers (hipMalloc + hipMemcpy, the caller's own stream),
 *   2. gpd_decode_host (host arrays, pinned double-buffered staging inside the library),
 *   3. the CPU oracle (oracle/libgpd_oracle.so, test infrastructure) as the checker.
 * Prints "abi_host ok N" and exits 0 when all three agree bit for bit.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "../../include/gpd.h"
#include "../../oracle/gpd_oracle.h"

#define CHECK(x)                                                                    \
  do {                                                                              \
    int rc_ = (x);                                                                  \
    if (rc_ != 0) {                                                                 \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_,         \
              gpd_last_error_string());                                             \
      exit(2);                                                                      \
    }                                                                               \
  } while (0)
#define HCHECK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                      \
    }                                                                               \
  } while (0)

typedef struct {
  uint32_t *status, *csum, *hdr_off;
  uint64_t *layers, *net_hash, *tp_hash;
} res_t;

static res_t res_alloc(uint64_t n) {
  res_t r;
  r.status = calloc(n, 4);
  r.csum = calloc(n, 4);
  r.hdr_off = calloc(n, 4);
  r.layers = calloc(n, 8);
  r.net_hash = calloc(n, 8);
  r.tp_hash = calloc(n, 8);
  return r;
}

static int res_cmp(const char *what, const res_t *a, const res_t *b, uint64_t n) {
  for (uint64_t i = 0; i < n; i++) {
    if (a->status[i] != b->status[i] || a->layers[i] != b->layers[i] ||
        a->net_hash[i] != b->net_hash[i] || a->tp_hash[i] != b->tp_hash[i] ||
        a->csum[i] != b->csum[i] || a->hdr_off[i] != b->hdr_off[i]) {
      fprintf(stderr,
              "%s: packet %llu differs: status %08x/%08x layers %016llx/%016llx net %016llx/%016llx "
              "tp %016llx/%016llx csum %08x/%08x\n",
              what, (unsigned long long)i, a->status[i], b->status[i],
              (unsigned long long)a->layers[i], (unsigned long long)b->layers[i],
              (unsigned long long)a->net_hash[i], (unsigned long long)b->net_hash[i],
              (unsigned long long)a->tp_hash[i], (unsigned long long)b->tp_hash[i], a->csum[i],
              b->csum[i]);
      return 1;
    }
  }
  return 0;
}

int main(int argc, char **argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: %s BATCH_FILE\n", argv[0]);
    return 2;
  }
  FILE *f = fopen(argv[1], "rb");
  if (!f) { perror(argv[1]); return 2; }
  uint64_t hdr[2];
  uint32_t cfgw[2];
  if (fread(hdr, 8, 2, f) != 2 || fread(cfgw, 4, 2, f) != 2) return 2;
  const uint64_t data_len = hdr[0], n = hdr[1];
  const uint64_t alloc = ((data_len + 15) & ~15ull) + 64;  /* gpd.h: readable to round_up + pad */
  uint8_t *data = aligned_alloc(16, alloc);
  uint32_t *off = malloc(4 * n + 4), *cap = malloc(4 * n + 4);
  memset(data, 0, alloc);
  if (fread(data, 1, data_len, f) != data_len || fread(off, 4, n, f) != n ||
      fread(cap, 4, n, f) != n) {
    fprintf(stderr, "short batch file\n");
    return 2;
  }
  fclose(f);

  gpd_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.first_layer = GPD_LT_ETHERNET;
  cfg.decoders = cfgw[0];
  cfg.options = cfgw[1];
  gpd_ctx *ctx = NULL;
  CHECK(gpd_ctx_create(0, &cfg, &ctx));

  /* 1. device-resident batch on the caller's stream */
  res_t dv = res_alloc(n);
  void *d_data, *d_off, *d_cap, *d_st, *d_ly, *d_nh, *d_th, *d_cs, *d_ho;
  hipStream_t s;
  HCHECK(hipStreamCreate(&s));
  HCHECK(hipMalloc(&d_data, alloc));
  HCHECK(hipMalloc(&d_off, 4 * n + 4));
  HCHECK(hipMalloc(&d_cap, 4 * n + 4));
  HCHECK(hipMalloc(&d_st, 4 * n + 4));
  HCHECK(hipMalloc(&d_ly, 8 * n + 8));
  HCHECK(hipMalloc(&d_nh, 8 * n + 8));
  HCHECK(hipMalloc(&d_th, 8 * n + 8));
  HCHECK(hipMalloc(&d_cs, 4 * n + 4));
  HCHECK(hipMalloc(&d_ho, 4 * n + 4));
  HCHECK(hipMemcpy(d_data, data, alloc, hipMemcpyHostToDevice));
  HCHECK(hipMemcpy(d_off, off, 4 * n, hipMemcpyHostToDevice));
  HCHECK(hipMemcpy(d_cap, cap, 4 * n, hipMemcpyHostToDevice));
  gpd_batch db = {(const uint8_t *)d_data, data_len, (const uint32_t *)d_off,
                  (const uint32_t *)d_cap, n};
  gpd_result dr = {(uint32_t *)d_st, (uint64_t *)d_ly, (uint64_t *)d_nh, (uint64_t *)d_th,
                   (uint32_t *)d_cs, NULL, (uint32_t *)d_ho};
  CHECK(gpd_decode(ctx, &db, &dr, s));
  CHECK(gpd_sync(ctx, s));
  HCHECK(hipMemcpy(dv.status, d_st, 4 * n, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(dv.layers, d_ly, 8 * n, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(dv.net_hash, d_nh, 8 * n, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(dv.tp_hash, d_th, 8 * n, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(dv.csum, d_cs, 4 * n, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(dv.hdr_off, d_ho, 4 * n, hipMemcpyDeviceToHost));

  /* 2. host batch through the library's pinned pipeline */
  res_t hv = res_alloc(n);
  gpd_batch hb = {data, data_len, off, cap, n};
  gpd_result hr = {hv.status, hv.layers, hv.net_hash, hv.tp_hash, hv.csum, NULL, hv.hdr_off};
  CHECK(gpd_decode_host(ctx, &hb, &hr));

  /* 3. the oracle */
  res_t ov = res_alloc(n);
  uint16_t *et = malloc(65536 * 2), *ip = malloc(256 * 2), *tp = malloc(65536 * 2),
           *up = malloc(65536 * 2);
  gpd_default_tables(et, ip, tp, up);
  gpo_tables t = {et, ip, tp, up};
  gpo_decode_batch(data, off, cap, n, GPD_LT_ETHERNET, cfg.decoders, cfg.options, &t, ov.status,
                   ov.layers, ov.net_hash, ov.tp_hash, ov.csum, ov.hdr_off, NULL, 8);

  int bad = res_cmp("gpd_decode vs oracle", &dv, &ov, n) | res_cmp("gpd_decode_host vs oracle", &hv, &ov, n);
  CHECK(gpd_ctx_destroy(ctx));
  HCHECK(hipStreamDestroy(s));
  if (bad) return 1;
  printf("abi_host ok %llu\n", (unsigned long long)n);
  return 0;
}
