/*
 * capi_roundtrip.c — GPU test driver for the C-ABI (include/fory_rowfmt.h),
 * called the way a JNI / cgo / ctypes shim would call it: plain C, HIP runtime
 * C API for device memory, no Python, no torch.
 *
 * Schema (Java order: names sorted): {a: int32, b: Long (nullable int64),
 * c: double, d: String (nullable utf8), e: List<Long> (list<int64>)}.
 * For N records: device encode (raw rows and frame stream) must equal the CPU
 * oracle's bytes (tests infrastructure: oracle/_build/liboracle.so), and
 * decode must return the input columns. Then the host path
 * (fory_rowfmt_host_*) on a fixed-width schema {a, b, c} against the oracle.
 * Exit status 0 = pass.
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fory_rowfmt.h"

/* oracle (test infrastructure, oracle/rowfmt_oracle.c) */
int64_t oracle_encode(const fory_field_desc* d, int n_desc, const fory_column* cols, int64_t nrows,
                      int frame_mode, uint8_t* out, int64_t cap, int64_t* row_offsets);

#define CHECK(x)                                                                  \
  do {                                                                            \
    int rc_ = (x);                                                                \
    if (rc_) {                                                                    \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_,       \
              fory_rowfmt_last_error());                                          \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)
#define HIPCHECK(x)                                                               \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next(void) {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return rng;
}

static void* dev_copy(const void* h, size_t n) {
  void* d = NULL;
  HIPCHECK(hipMalloc(&d, n ? n : 16));
  if (n) HIPCHECK(hipMemcpy(d, h, n, hipMemcpyHostToDevice));
  return d;
}

static int varlen_roundtrip(int64_t n, int frame) {
  const fory_field_desc desc[] = {
      {FORY_TYPE_INT32, 0, 0, 0}, {FORY_TYPE_INT64, 1, 0, 0}, {FORY_TYPE_DOUBLE, 0, 0, 0},
      {FORY_TYPE_STRING, 1, 0, 0}, {FORY_TYPE_LIST, 1, 1, 0}, {FORY_TYPE_INT64, 1, 0, 0}};
  const int nd = 6;
  /* host columns */
  int32_t* a = malloc(n * 4);
  int64_t* b = malloc(n * 8);
  double* c = malloc(n * 8);
  int32_t* doff = malloc((n + 1) * 4);
  int32_t* eoff = malloc((n + 1) * 4);
  uint8_t* bval = calloc((n + 31) / 8 + 4, 1);
  uint8_t* dval = calloc((n + 31) / 8 + 4, 1);
  uint8_t* evalid = calloc((n + 31) / 8 + 4, 1);
  char* dbytes = malloc(n * 24 + 16);
  int64_t* items = malloc(n * 20 * 8 + 8);
  uint8_t* ivalid = calloc((n * 20 + 31) / 8 + 4, 1);
  int64_t nb = 0, ni = 0;
  doff[0] = eoff[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    a[i] = (int32_t)next();
    b[i] = (int64_t)next();
    c[i] = (double)(int64_t)next() / 3.0;
    if (next() % 5) bval[i >> 3] |= 1u << (i & 7);
    if (next() % 4) {
      dval[i >> 3] |= 1u << (i & 7);
      int len = (int)(next() % 24);
      for (int k = 0; k < len; ++k) dbytes[nb++] = (char)('a' + next() % 26);
    }
    doff[i + 1] = (int32_t)nb;
    if (next() % 6) {
      evalid[i >> 3] |= 1u << (i & 7);
      int len = (int)(next() % 20);
      for (int k = 0; k < len; ++k) {
        items[ni] = (int64_t)next();
        if (next() % 7) ivalid[ni >> 3] |= 1u << (ni & 7);
        ++ni;
      }
    }
    eoff[i + 1] = (int32_t)ni;
  }
  fory_column hc[6] = {
      {a, NULL, NULL, n, 0}, {b, NULL, bval, n, 0}, {c, NULL, NULL, n, 0},
      {dbytes, doff, dval, n, 0}, {NULL, eoff, evalid, n, 0}, {items, NULL, ivalid, ni, 0}};
  /* expected bytes */
  int64_t* eoffs = malloc((n + 1) * 8);
  int64_t total = oracle_encode(desc, nd, hc, n, frame, NULL, 0, eoffs);
  uint8_t* expect = malloc(total + 16);
  if (oracle_encode(desc, nd, hc, n, frame, expect, total, eoffs) != total) return 1;

  /* device columns */
  fory_column dc[6];
  for (int k = 0; k < 6; ++k) dc[k] = hc[k];
  dc[0].values = dev_copy(a, n * 4);
  dc[1].values = dev_copy(b, n * 8);
  dc[1].validity = dev_copy(bval, (n + 31) / 8 + 4);
  dc[2].values = dev_copy(c, n * 8);
  dc[3].values = dev_copy(dbytes, nb + 8);
  dc[3].offsets = dev_copy(doff, (n + 1) * 4);
  dc[3].validity = dev_copy(dval, (n + 31) / 8 + 4);
  dc[4].offsets = dev_copy(eoff, (n + 1) * 4);
  dc[4].validity = dev_copy(evalid, (n + 31) / 8 + 4);
  dc[5].values = dev_copy(items, ni * 8 + 8);
  dc[5].validity = dev_copy(ivalid, (ni + 31) / 8 + 4);

  fory_plan* plan = NULL;
  CHECK(fory_rowfmt_plan_create(desc, nd, &plan));
  fory_plan_info info;
  CHECK(fory_rowfmt_plan_info(plan, &info));
  const int64_t wsb = fory_rowfmt_workspace_bytes(plan, n);
  void* ws = NULL;
  HIPCHECK(hipMalloc(&ws, wsb));
  int64_t* d_offs = NULL;
  HIPCHECK(hipMalloc((void**)&d_offs, (n + 1) * 8));
  int32_t* d_status = NULL;
  HIPCHECK(hipMalloc((void**)&d_status, 4));
  HIPCHECK(hipMemset(d_status, 0, 4));
  CHECK(fory_rowfmt_encoded_size(plan, dc, n, frame, d_offs, ws, wsb, NULL));
  int64_t got_total = 0;
  HIPCHECK(hipMemcpy(&got_total, d_offs + n, 8, hipMemcpyDeviceToHost));
  if (got_total != total) {
    fprintf(stderr, "encoded_size %lld != oracle %lld\n", (long long)got_total, (long long)total);
    return 1;
  }
  uint8_t* d_out = NULL;
  HIPCHECK(hipMalloc((void**)&d_out, total + 16));
  CHECK(fory_rowfmt_encode(plan, dc, n, frame, d_offs, d_out, total, d_status, ws, wsb, NULL));
  CHECK(fory_rowfmt_read_status(d_status, NULL));
  uint8_t* got = malloc(total + 16);
  HIPCHECK(hipMemcpy(got, d_out, total, hipMemcpyDeviceToHost));
  if (memcmp(got, expect, total) != 0) {
    fprintf(stderr, "encode bytes differ from the oracle (n=%lld frame=%d)\n", (long long)n, frame);
    return 1;
  }
  /* decode: offsets first (decode_sizes), then values */
  fory_column oc[6];
  memset(oc, 0, sizeof(oc));
  HIPCHECK(hipMalloc(&oc[0].values, n * 4 + 4));
  HIPCHECK(hipMalloc(&oc[1].values, n * 8 + 8));
  HIPCHECK(hipMalloc((void**)&oc[1].validity, (n + 31) / 8 + 4));
  HIPCHECK(hipMalloc(&oc[2].values, n * 8 + 8));
  HIPCHECK(hipMalloc((void**)&oc[3].offsets, (n + 1) * 4));
  HIPCHECK(hipMalloc((void**)&oc[3].validity, (n + 31) / 8 + 4));
  HIPCHECK(hipMalloc((void**)&oc[4].offsets, (n + 1) * 4));
  HIPCHECK(hipMalloc((void**)&oc[4].validity, (n + 31) / 8 + 4));
  for (int k = 0; k < 5; ++k) oc[k].length = n;
  CHECK(fory_rowfmt_decode_sizes(plan, d_out, d_offs, n, frame, oc, d_status, ws, wsb, NULL));
  int32_t tb = 0, ti = 0;
  HIPCHECK(hipMemcpy(&tb, oc[3].offsets + n, 4, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(&ti, oc[4].offsets + n, 4, hipMemcpyDeviceToHost));
  if (tb != nb || ti != ni) {
    fprintf(stderr, "decode_sizes totals %d/%d != %lld/%lld\n", tb, ti, (long long)nb, (long long)ni);
    return 1;
  }
  HIPCHECK(hipMalloc(&oc[3].values, nb + 8));
  oc[3].capacity = nb + 8;
  HIPCHECK(hipMalloc(&oc[5].values, ni * 8 + 8));
  HIPCHECK(hipMalloc((void**)&oc[5].validity, (ni + 31) / 8 + 4));
  oc[5].length = ni;
  CHECK(fory_rowfmt_decode(plan, d_out, d_offs, n, frame, oc, d_status, ws, wsb, NULL));
  CHECK(fory_rowfmt_read_status(d_status, NULL));
  /* compare valid values */
  int32_t* a2 = malloc(n * 4);
  int64_t* b2 = malloc(n * 8);
  int32_t* doff2 = malloc((n + 1) * 4);
  char* dbytes2 = malloc(nb + 8);
  int32_t* eoff2 = malloc((n + 1) * 4);
  int64_t* items2 = malloc(ni * 8 + 8);
  uint8_t* ivalid2 = malloc((ni + 31) / 8 + 4);
  HIPCHECK(hipMemcpy(a2, oc[0].values, n * 4, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(b2, oc[1].values, n * 8, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(doff2, oc[3].offsets, (n + 1) * 4, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(dbytes2, oc[3].values, nb, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(eoff2, oc[4].offsets, (n + 1) * 4, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(items2, oc[5].values, ni * 8, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(ivalid2, oc[5].validity, (ni + 7) / 8, hipMemcpyDeviceToHost));
  for (int64_t i = 0; i < n; ++i) {
    int bv = (bval[i >> 3] >> (i & 7)) & 1;
    if (a2[i] != a[i] || (bv && b2[i] != b[i]) || doff2[i + 1] != doff[i + 1] || eoff2[i + 1] != eoff[i + 1]) {
      fprintf(stderr, "decode mismatch at record %lld\n", (long long)i);
      return 1;
    }
  }
  if (memcmp(dbytes2, dbytes, nb) != 0) return fprintf(stderr, "string bytes differ\n"), 1;
  for (int64_t q = 0; q < ni; ++q) {
    int v = (ivalid[q >> 3] >> (q & 7)) & 1, v2 = (ivalid2[q >> 3] >> (q & 7)) & 1;
    if (v != v2 || (v && items2[q] != items[q])) return fprintf(stderr, "list item %lld differs\n", (long long)q), 1;
  }
  fory_rowfmt_plan_destroy(plan);
  printf("varlen n=%lld frame=%d: %lld bytes == oracle, decode == input\n", (long long)n, frame, (long long)total);
  return 0;
}

static int host_path(int64_t n, int frame) {
  const fory_field_desc desc[] = {{FORY_TYPE_INT32, 0, 0, 0}, {FORY_TYPE_INT64, 1, 0, 0}, {FORY_TYPE_DOUBLE, 0, 0, 0}};
  int32_t* a = malloc(n * 4);
  int64_t* b = malloc(n * 8);
  double* c = malloc(n * 8);
  uint8_t* bval = calloc((n + 31) / 8 + 4, 1);
  for (int64_t i = 0; i < n; ++i) {
    a[i] = (int32_t)next();
    b[i] = (int64_t)next();
    c[i] = (double)(int64_t)next();
    if (next() % 3) bval[i >> 3] |= 1u << (i & 7);
  }
  fory_column hc[3] = {{a, NULL, NULL, n, 0}, {b, NULL, bval, n, 0}, {c, NULL, NULL, n, 0}};
  int64_t total = oracle_encode(desc, 3, hc, n, frame, NULL, 0, NULL);
  uint8_t* expect = malloc(total + 16);
  oracle_encode(desc, 3, hc, n, frame, expect, total, NULL);
  fory_plan* plan = NULL;
  CHECK(fory_rowfmt_plan_create(desc, 3, &plan));
  fory_host_ctx* ctx = NULL;
  CHECK(fory_rowfmt_host_ctx_create(plan, 0, 4096, &ctx));
  uint8_t* out = malloc(total + 16);
  CHECK(fory_rowfmt_host_register(out, total));
  CHECK(fory_rowfmt_host_encode(ctx, hc, n, frame, out, total));
  if (memcmp(out, expect, total) != 0) return fprintf(stderr, "host encode differs\n"), 1;
  int32_t* a2 = malloc(n * 4);
  int64_t* b2 = malloc(n * 8);
  double* c2 = malloc(n * 8);
  uint8_t* bval2 = calloc((n + 31) / 8 + 4, 1);
  fory_column oc[3] = {{a2, NULL, NULL, n, n * 4}, {b2, NULL, bval2, n, n * 8}, {c2, NULL, NULL, n, n * 8}};
  CHECK(fory_rowfmt_host_decode(ctx, out, total, n, frame, oc));
  for (int64_t i = 0; i < n; ++i) {
    int v = (bval[i >> 3] >> (i & 7)) & 1, v2 = (bval2[i >> 3] >> (i & 7)) & 1;
    if (a2[i] != a[i] || v != v2 || (v && b2[i] != b[i]) || memcmp(&c2[i], &c[i], 8))
      return fprintf(stderr, "host decode mismatch at %lld\n", (long long)i), 1;
  }
  CHECK(fory_rowfmt_host_unregister(out));
  fory_rowfmt_host_ctx_destroy(ctx);
  fory_rowfmt_plan_destroy(plan);
  printf("host path n=%lld frame=%d: %lld bytes == oracle, decode == input\n", (long long)n, frame, (long long)total);
  return 0;
}

int main(void) {
  if (fory_rowfmt_abi_version() != FORY_ROWFMT_ABI_VERSION) return 1;
  const int64_t sizes[] = {1, 63, 64, 1000, 20011};
  for (int f = 0; f < 2; ++f)
    for (int k = 0; k < 5; ++k)
      if (varlen_roundtrip(sizes[k], f) || host_path(sizes[k] * 3, f)) return 1;
  printf("capi_roundtrip: all ok\n");
  return 0;
}
