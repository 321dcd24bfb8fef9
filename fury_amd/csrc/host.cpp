// host.cpp — host-memory path of the C-ABI (include/fory_rowfmt.h, "host path").
//
// The reference path starts and ends in host memory: Encoder.encode(MemoryBuffer, T)
// appends frames to an off-heap MemoryBuffer on its way to an RPC socket and
// Encoder.decode(MemoryBuffer) reads them back (java/fory-format/.../encoder/
// Encoders.java:177-225; off-heap addresses: java/fory-core/.../memory/
// MemoryBuffer.java:287-297). A fory_host_ctx moves such host batches through
// the device kernels with a three-stream chunk pipeline: H2D of chunk k+1 ||
// kernel of chunk k || D2H of chunk k-1, double-buffered device chunks
// allocated once per context. It is a client of the device entry points in
// capi.cpp (plan_info / workspace_bytes / encode / decode / read_status).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/fory_rowfmt.h"

namespace {


constexpr int64_t kAlign = 256;
int64_t align_up(int64_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

struct Slice {  // one column's device chunk buffers
  uint8_t* values = nullptr;
  uint8_t* validity = nullptr;
};

}  // namespace

struct fory_host_ctx {
  const fory_plan* plan = nullptr;
  fory_plan_info info{};
  int device = 0;
  int64_t chunk = 0;
  std::vector<int32_t> width;       // per top-level column (fixed-width plans: one column per field)
  std::vector<int32_t> nullable;
  uint8_t* arena = nullptr;         // both buffers, carved
  struct Buf {
    std::vector<Slice> cols;
    uint8_t* rows = nullptr;
    void* ws = nullptr;
    int32_t* status = nullptr;
  } buf[2];
  int64_t ws_bytes = 0;
  hipStream_t s_in = nullptr, s_k = nullptr, s_out = nullptr;
  hipEvent_t ev_in[2] = {}, ev_k[2] = {}, ev_out[2] = {};
};

namespace {

int fail_host(int code, const std::string& msg);

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return FORY_OK;
  return fail_host(FORY_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

// Library-internal helpers of capi.cpp (not in the public header): last_error
// is thread-local there; column widths/nullability of a fixed-width plan.
extern "C" int fory_rowfmt_internal_set_error(int code, const char* msg);
extern "C" int fory_rowfmt_internal_column_layout(const fory_plan* plan, int32_t* width, int32_t* nullable);

namespace {

int fail_host(int code, const std::string& msg) { return fory_rowfmt_internal_set_error(code, msg.c_str()); }

int64_t validity_bytes(int64_t rows) { return ((rows + 7) / 8 + 3) / 4 * 4; }

// Chunk k's row range.
void chunk_range(const fory_host_ctx* c, int64_t n, int64_t k, int64_t* a, int64_t* rows) {
  *a = k * c->chunk;
  *rows = n - *a < c->chunk ? n - *a : c->chunk;
}

}  // namespace

extern "C" {

int fory_rowfmt_host_ctx_create(const fory_plan* plan, int32_t device, int64_t chunk_rows,
                                fory_host_ctx** out) {
  if (!out) return fail_host(FORY_ERR_INVALID_ARGUMENT, "out is null");
  *out = nullptr;
  if (!plan) return fail_host(FORY_ERR_INVALID_ARGUMENT, "plan is null");
  fory_plan_info info{};
  int rc = fory_rowfmt_plan_info(plan, &info);
  if (rc) return rc;
  if (!info.fixed_width)
    return fail_host(FORY_ERR_UNSUPPORTED, "host path: fixed-width plans only (ABI 1); varlen plans use the device "
                                           "entry points with caller-staged buffers");
  if (chunk_rows <= 0) chunk_rows = 1 << 20;
  chunk_rows = (chunk_rows + 63) / 64 * 64;  // whole 64-record tiles: validity slices are byte aligned
  fory_host_ctx* c = new fory_host_ctx();
  c->plan = plan;
  c->info = info;
  c->device = device;
  c->chunk = chunk_rows;
  rc = hip_check(hipSetDevice(device), "hipSetDevice");
  if (rc) {
    delete c;
    return rc;
  }
  c->width.resize(info.num_columns);
  c->nullable.resize(info.num_columns);
  fory_rowfmt_internal_column_layout(plan, c->width.data(), c->nullable.data());  // pre-order = schema order
  const int64_t stride = info.fixed_size + 12;  // room for frames too
  c->ws_bytes = fory_rowfmt_workspace_bytes(plan, chunk_rows);
  int64_t per = 0;
  for (int i = 0; i < info.num_columns; ++i)
    per += align_up(c->width[i] * chunk_rows) + (c->nullable[i] ? align_up(validity_bytes(chunk_rows)) : 0);
  per += align_up(stride * chunk_rows) + align_up(c->ws_bytes) + kAlign;
  rc = hip_check(hipMalloc(&c->arena, (size_t)(2 * per)), "hipMalloc(host ctx chunk buffers)");
  if (rc) {
    delete c;
    return rc;
  }
  for (int b = 0; b < 2; ++b) {
    uint8_t* p = c->arena + b * per;
    c->buf[b].cols.resize(info.num_columns);
    for (int i = 0; i < info.num_columns; ++i) {
      c->buf[b].cols[i].values = p;
      p += align_up(c->width[i] * chunk_rows);
      if (c->nullable[i]) {
        c->buf[b].cols[i].validity = p;
        p += align_up(validity_bytes(chunk_rows));
      }
    }
    c->buf[b].rows = p;
    p += align_up(stride * chunk_rows);
    c->buf[b].ws = p;
    p += align_up(c->ws_bytes);
    c->buf[b].status = reinterpret_cast<int32_t*>(p);
  }
  rc = hip_check(hipMemset(c->arena, 0, (size_t)(2 * per)), "hipMemset");
  for (hipStream_t* s : {&c->s_in, &c->s_k, &c->s_out})
    if (!rc) rc = hip_check(hipStreamCreateWithFlags(s, hipStreamNonBlocking), "hipStreamCreate");
  for (int b = 0; b < 2 && !rc; ++b)
    for (hipEvent_t* e : {&c->ev_in[b], &c->ev_k[b], &c->ev_out[b]})
      if (!rc) rc = hip_check(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate");
  if (rc) {
    fory_rowfmt_host_ctx_destroy(c);
    return rc;
  }
  *out = c;
  return FORY_OK;
}

void fory_rowfmt_host_ctx_destroy(fory_host_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->s_in) (void)hipStreamSynchronize(c->s_in);
  if (c->s_k) (void)hipStreamSynchronize(c->s_k);
  if (c->s_out) (void)hipStreamSynchronize(c->s_out);
  for (int b = 0; b < 2; ++b)
    for (hipEvent_t e : {c->ev_in[b], c->ev_k[b], c->ev_out[b]})
      if (e) (void)hipEventDestroy(e);
  for (hipStream_t s : {c->s_in, c->s_k, c->s_out})
    if (s) (void)hipStreamDestroy(s);
  if (c->arena) (void)hipFree(c->arena);
  delete c;
}

int fory_rowfmt_host_register(void* host_ptr, int64_t bytes) {
  if (!host_ptr || bytes <= 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "null pointer or empty range");
  return hip_check(hipHostRegister(host_ptr, (size_t)bytes, hipHostRegisterDefault), "hipHostRegister");
}

int fory_rowfmt_host_unregister(void* host_ptr) {
  if (!host_ptr) return fail_host(FORY_ERR_INVALID_ARGUMENT, "null pointer");
  return hip_check(hipHostUnregister(host_ptr), "hipHostUnregister");
}

int fory_rowfmt_host_encode(fory_host_ctx* c, const fory_column* host_cols, int64_t n, int32_t frame,
                            void* host_out, int64_t out_capacity) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  if (frame != FORY_FRAME_RAW && frame != FORY_FRAME_STREAM)
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "frame_mode must be 0 (raw) or 1 (stream)");
  if (n < 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "num_rows < 0");
  if (n == 0) return FORY_OK;
  if (!host_cols || !host_out) return fail_host(FORY_ERR_INVALID_ARGUMENT, "host columns or output is null");
  const int64_t stride = c->info.fixed_size + (frame ? 12 : 0);
  if (n * stride > out_capacity)  // MemoryBuffer bounds check (MemoryBuffer.java:303-309)
    return fail_host(FORY_ERR_CAPACITY, "output capacity " + std::to_string(out_capacity) + " < " +
                                            std::to_string(n * stride) + " bytes");
  for (int i = 0; i < c->info.num_columns; ++i)
    if (!host_cols[i].values || host_cols[i].length < n)
      return fail_host(FORY_ERR_INVALID_ARGUMENT, "column " + std::to_string(i) + " missing or shorter than num_rows");
  int rc = hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  for (int b = 0; b < 2 && !rc; ++b)
    rc = hip_check(hipMemsetAsync(c->buf[b].status, 0, 4, c->s_k), "hipMemsetAsync");
  const int64_t chunks = (n + c->chunk - 1) / c->chunk;
  std::vector<fory_column> dcols(c->info.num_columns);
  uint8_t* out = static_cast<uint8_t*>(host_out);
  for (int64_t k = 0; k < chunks && !rc; ++k) {
    const int b = (int)(k & 1);
    int64_t a, rows;
    chunk_range(c, n, k, &a, &rows);
    fory_host_ctx::Buf& B = c->buf[b];
    // H2D: column slices (+ validity bytes) into buffer b once chunk k-2's kernel is done with it
    if (k >= 2) rc = hip_check(hipStreamWaitEvent(c->s_in, c->ev_k[b], 0), "hipStreamWaitEvent");
    for (int i = 0; i < c->info.num_columns && !rc; ++i) {
      const fory_column& h = host_cols[i];
      rc = hip_check(hipMemcpyAsync(B.cols[i].values, static_cast<const uint8_t*>(h.values) + a * c->width[i],
                                    (size_t)(rows * c->width[i]), hipMemcpyHostToDevice, c->s_in), "H2D");
      if (!rc && c->nullable[i] && h.validity)
        rc = hip_check(hipMemcpyAsync(B.cols[i].validity, h.validity + a / 8, (size_t)((rows + 7) / 8),
                                      hipMemcpyHostToDevice, c->s_in), "H2D validity");
      dcols[i] = fory_column{B.cols[i].values, nullptr, (c->nullable[i] && h.validity) ? B.cols[i].validity : nullptr,
                             rows, rows * c->width[i]};
    }
    if (!rc) rc = hip_check(hipEventRecord(c->ev_in[b], c->s_in), "hipEventRecord");
    // kernel: after the chunk landed and chunk k-2's rows left buffer b
    if (!rc) rc = hip_check(hipStreamWaitEvent(c->s_k, c->ev_in[b], 0), "hipStreamWaitEvent");
    if (!rc && k >= 2) rc = hip_check(hipStreamWaitEvent(c->s_k, c->ev_out[b], 0), "hipStreamWaitEvent");
    if (!rc)
      rc = fory_rowfmt_encode(c->plan, dcols.data(), rows, frame, nullptr, B.rows, rows * stride, B.status, B.ws,
                              c->ws_bytes, c->s_k);
    if (!rc) rc = hip_check(hipEventRecord(c->ev_k[b], c->s_k), "hipEventRecord");
    // D2H: the chunk's rows, contiguous in the output (row/frame i at i * stride)
    if (!rc) rc = hip_check(hipStreamWaitEvent(c->s_out, c->ev_k[b], 0), "hipStreamWaitEvent");
    if (!rc)
      rc = hip_check(hipMemcpyAsync(out + a * stride, B.rows, (size_t)(rows * stride), hipMemcpyDeviceToHost,
                                    c->s_out), "D2H");
    if (!rc) rc = hip_check(hipEventRecord(c->ev_out[b], c->s_out), "hipEventRecord");
  }
  const int rc_sync = hip_check(hipStreamSynchronize(c->s_out), "hipStreamSynchronize");
  (void)hipStreamSynchronize(c->s_k);
  (void)hipStreamSynchronize(c->s_in);
  if (rc) return rc;
  if (rc_sync) return rc_sync;
  for (int b = 0; b < 2; ++b) {
    rc = fory_rowfmt_read_status(c->buf[b].status, c->s_k);
    if (rc) return rc;
  }
  return FORY_OK;
}

int fory_rowfmt_host_decode(fory_host_ctx* c, const void* host_rows, int64_t rows_bytes, int64_t n, int32_t frame,
                            const fory_column* host_out_cols) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  if (frame != FORY_FRAME_RAW && frame != FORY_FRAME_STREAM)
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "frame_mode must be 0 (raw) or 1 (stream)");
  if (n < 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "num_rows < 0");
  if (n == 0) return FORY_OK;
  if (!host_rows || !host_out_cols) return fail_host(FORY_ERR_INVALID_ARGUMENT, "host rows or output columns null");
  const int64_t stride = c->info.fixed_size + (frame ? 12 : 0);
  if (n * stride > rows_bytes)
    return fail_host(FORY_ERR_CORRUPT, "row buffer holds " + std::to_string(rows_bytes) + " bytes < " +
                                           std::to_string(n) + " rows x " + std::to_string(stride));
  for (int i = 0; i < c->info.num_columns; ++i) {
    const fory_column& h = host_out_cols[i];
    if (!h.values || (h.capacity > 0 && h.capacity < n * c->width[i]))
      return fail_host(FORY_ERR_CAPACITY, "output column " + std::to_string(i) + " missing or too small");
  }
  int rc = hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  for (int b = 0; b < 2 && !rc; ++b)
    rc = hip_check(hipMemsetAsync(c->buf[b].status, 0, 4, c->s_k), "hipMemsetAsync");
  const int64_t chunks = (n + c->chunk - 1) / c->chunk;
  std::vector<fory_column> dcols(c->info.num_columns);
  const uint8_t* in = static_cast<const uint8_t*>(host_rows);
  for (int64_t k = 0; k < chunks && !rc; ++k) {
    const int b = (int)(k & 1);
    int64_t a, rows;
    chunk_range(c, n, k, &a, &rows);
    fory_host_ctx::Buf& B = c->buf[b];
    if (k >= 2) rc = hip_check(hipStreamWaitEvent(c->s_in, c->ev_k[b], 0), "hipStreamWaitEvent");
    if (!rc)
      rc = hip_check(hipMemcpyAsync(B.rows, in + a * stride, (size_t)(rows * stride), hipMemcpyHostToDevice, c->s_in),
                     "H2D");
    if (!rc) rc = hip_check(hipEventRecord(c->ev_in[b], c->s_in), "hipEventRecord");
    if (!rc) rc = hip_check(hipStreamWaitEvent(c->s_k, c->ev_in[b], 0), "hipStreamWaitEvent");
    if (!rc && k >= 2) rc = hip_check(hipStreamWaitEvent(c->s_k, c->ev_out[b], 0), "hipStreamWaitEvent");
    for (int i = 0; i < c->info.num_columns; ++i)
      dcols[i] = fory_column{B.cols[i].values, nullptr,
                             (c->nullable[i] && host_out_cols[i].validity) ? B.cols[i].validity : nullptr, rows,
                             rows * c->width[i]};
    if (!rc) rc = fory_rowfmt_decode(c->plan, B.rows, nullptr, rows, frame, dcols.data(), B.status, B.ws, c->ws_bytes,
                                     c->s_k);
    if (!rc) rc = hip_check(hipEventRecord(c->ev_k[b], c->s_k), "hipEventRecord");
    if (!rc) rc = hip_check(hipStreamWaitEvent(c->s_out, c->ev_k[b], 0), "hipStreamWaitEvent");
    for (int i = 0; i < c->info.num_columns && !rc; ++i) {
      const fory_column& h = host_out_cols[i];
      rc = hip_check(hipMemcpyAsync(static_cast<uint8_t*>(h.values) + a * c->width[i], B.cols[i].values,
                                    (size_t)(rows * c->width[i]), hipMemcpyDeviceToHost, c->s_out), "D2H");
      if (!rc && dcols[i].validity)
        rc = hip_check(hipMemcpyAsync(h.validity + a / 8, B.cols[i].validity, (size_t)((rows + 7) / 8),
                                      hipMemcpyDeviceToHost, c->s_out), "D2H validity");
    }
    if (!rc) rc = hip_check(hipEventRecord(c->ev_out[b], c->s_out), "hipEventRecord");
  }
  const int rc_sync = hip_check(hipStreamSynchronize(c->s_out), "hipStreamSynchronize");
  (void)hipStreamSynchronize(c->s_k);
  (void)hipStreamSynchronize(c->s_in);
  if (rc) return rc;
  if (rc_sync) return rc_sync;
  for (int b = 0; b < 2; ++b) {
    rc = fory_rowfmt_read_status(c->buf[b].status, c->s_k);
    if (rc) return rc;
  }
  return FORY_OK;
}

}  // extern "C"
