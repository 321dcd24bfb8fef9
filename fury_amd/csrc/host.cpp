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

#include <algorithm>
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
  // varlen plans (whole batch per call; device buffers kept and grown)
  bool varlen = false;
  std::vector<int32_t> kind, parent;
  uint8_t* dbuf = nullptr;   // columns, row offsets, workspace, status
  int64_t dbuf_bytes = 0;
  uint8_t* drows = nullptr;  // rows / frames
  int64_t drows_bytes = 0;
  uint8_t* dout = nullptr;   // decode: output columns
  int64_t dout_bytes = 0;
  // decode state between host_decode_var_sizes and host_decode_var
  int64_t dec_n = -1;
  int32_t dec_frame = 0;
  std::vector<int64_t> dec_count, dec_bytes;
  std::vector<fory_column> dec_cols;
  int64_t* dec_offs = nullptr;
  void* dec_ws = nullptr;
  int32_t* dec_status = nullptr;
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
extern "C" int fory_rowfmt_internal_node_layout(const fory_plan* plan, int32_t* kind, int32_t* width,
                                                int32_t* nullable, int32_t* parent);

namespace {

int fail_host(int code, const std::string& msg) { return fory_rowfmt_internal_set_error(code, msg.c_str()); }

int64_t validity_bytes(int64_t rows) { return ((rows + 7) / 8 + 3) / 4 * 4; }

// Caller host memory is copied asynchronously only when it is pinned (registered
// with fory_rowfmt_host_register / hipHostRegister, or hipHostMalloc): the chunk
// pipeline orders those copies with events. Pageable memory is copied with a
// blocking hipMemcpy once the stream's earlier work (and the events it waits on) is
// done: the async pageable path was seen to leave a chunk kernel reading columns
// whose H2D had not landed (tests/test_gpu_host.py, intermittent, first rows zero).
bool host_pinned(const void* p) {
  hipPointerAttribute_t a{};
  if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type != hipMemoryTypeUnregistered;
}

int hcopy(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s, const char* what) {
  if (bytes == 0) return FORY_OK;
  if (host_pinned(kind == hipMemcpyHostToDevice ? src : dst))
    return hip_check(hipMemcpyAsync(dst, src, bytes, kind, s), what);
  int rc = hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
  if (!rc) rc = hip_check(hipMemcpy(dst, src, bytes, kind), what);
  return rc;
}

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
  if (!info.fixed_width) {  // varlen: fory_rowfmt_host_encode_var / host_decode_var_sizes / host_decode_var
    fory_host_ctx* c = new fory_host_ctx();
    c->plan = plan;
    c->info = info;
    c->device = device;
    c->varlen = true;
    c->kind.resize(info.num_columns);
    c->parent.resize(info.num_columns);
    c->width.resize(info.num_columns);
    c->nullable.resize(info.num_columns);
    fory_rowfmt_internal_node_layout(plan, c->kind.data(), c->width.data(), c->nullable.data(), c->parent.data());
    rc = hip_check(hipSetDevice(device), "hipSetDevice");
    if (!rc) rc = hip_check(hipStreamCreateWithFlags(&c->s_k, hipStreamNonBlocking), "hipStreamCreate");
    if (rc) {
      fory_rowfmt_host_ctx_destroy(c);
      return rc;
    }
    *out = c;
    return FORY_OK;
  }
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
  for (uint8_t* b : {c->dbuf, c->drows, c->dout})
    if (b) (void)hipFree(b);
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

}  // extern "C"

namespace {

// Host output windows: window w receives rows [first[w], first[w+1]) of the batch
// (whole rows/frames only), at most cap[w] bytes. One window of the caller's
// capacity is the contiguous MemoryBuffer of host_encode / host_encode_var.
struct OutWindows {
  std::vector<uint8_t*> ptr;
  std::vector<int64_t> cap;
  std::vector<int64_t> first;  // size() + 1 entries once split
};

// Greedy split (a MemoryBuffer is int-sized, MemoryBuffer.java:87: the JNI side
// fills one buffer with whole frames, then the next): window w takes rows while
// they fit its capacity. Offsets from `offs` (n+1, host) or i * stride. A window too
// small for the next row stays empty; running out of windows is FORY_ERR_CAPACITY.
int split_rows(const int64_t* offs, int64_t stride, int64_t n, OutWindows* W) {
  const int64_t nw = (int64_t)W->cap.size();
  W->first.assign((size_t)nw + 1, n);
  auto at = [&](int64_t i) { return offs ? offs[i] : i * stride; };
  int64_t start = 0;
  for (int64_t w = 0; w < nw; ++w) {
    W->first[(size_t)w] = start;
    if (start >= n) continue;
    const int64_t limit = at(start) + W->cap[(size_t)w];
    int64_t lo = start, hi = n;  // largest e in [start, n] with at(e) <= limit
    while (lo < hi) {
      const int64_t mid = hi - (hi - lo) / 2;
      if (at(mid) <= limit) lo = mid;
      else hi = mid - 1;
    }
    start = lo;
  }
  W->first[(size_t)nw] = start;
  if (start < n)
    return fail_host(FORY_ERR_CAPACITY, "output windows hold " + std::to_string(start) + " of " + std::to_string(n) +
                                            " rows (" + std::to_string(at(n) - at(start)) + " more bytes needed)");
  return FORY_OK;
}

// Queues the D2H of rows [a, a + rows) (contiguous at `src`, row i at (i - a) * stride)
// into the windows they belong to.
int d2h_rows_windows(const OutWindows& W, const uint8_t* src, int64_t a, int64_t rows, int64_t stride, hipStream_t s) {
  int rc = FORY_OK;
  for (size_t w = 0; w + 1 < W.first.size() && !rc; ++w) {
    const int64_t lo = std::max(a, W.first[w]), hi = std::min(a + rows, W.first[w + 1]);
    if (lo >= hi) continue;
    rc = hcopy(W.ptr[w] + (lo - W.first[w]) * stride, src + (lo - a) * stride, (size_t)((hi - lo) * stride), hipMemcpyDeviceToHost, s, "D2H");
  }
  return rc;
}

int host_encode_fixed(fory_host_ctx* c, const fory_column* host_cols, int64_t n, int32_t frame, OutWindows* W) {
  if (c->varlen) return fail_host(FORY_ERR_INVALID_ARGUMENT, "varlen plan: use fory_rowfmt_host_encode_var");
  if (frame != FORY_FRAME_RAW && frame != FORY_FRAME_STREAM && frame != FORY_FRAME_HASHED)
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "frame_mode must be 0 (raw), 1 (stream) or 3 (hashed)");
  if (n < 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "num_rows < 0");
  const int64_t stride = c->info.fixed_size + (frame == FORY_FRAME_STREAM ? 12 : frame == FORY_FRAME_HASHED ? 8 : 0);
  int rc = split_rows(nullptr, stride, n, W);  // MemoryBuffer bounds check (MemoryBuffer.java:303-309)
  if (rc || n == 0) return rc;
  if (!host_cols) return fail_host(FORY_ERR_INVALID_ARGUMENT, "host columns are null");
  for (size_t w = 0; w + 1 < W->first.size(); ++w)
    if (W->first[w + 1] > W->first[w] && !W->ptr[w]) return fail_host(FORY_ERR_INVALID_ARGUMENT, "output is null");
  for (int i = 0; i < c->info.num_columns; ++i)
    if (!host_cols[i].values || host_cols[i].length < n)
      return fail_host(FORY_ERR_INVALID_ARGUMENT, "column " + std::to_string(i) + " missing or shorter than num_rows");
  rc = hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  for (int b = 0; b < 2 && !rc; ++b)
    rc = hip_check(hipMemsetAsync(c->buf[b].status, 0, 4, c->s_k), "hipMemsetAsync");
  const int64_t chunks = (n + c->chunk - 1) / c->chunk;
  std::vector<fory_column> dcols(c->info.num_columns);
  for (int64_t k = 0; k < chunks && !rc; ++k) {
    const int b = (int)(k & 1);
    int64_t a, rows;
    chunk_range(c, n, k, &a, &rows);
    fory_host_ctx::Buf& B = c->buf[b];
    // H2D: column slices (+ validity bytes) into buffer b once chunk k-2's kernel is done with it
    if (k >= 2) rc = hip_check(hipStreamWaitEvent(c->s_in, c->ev_k[b], 0), "hipStreamWaitEvent");
    for (int i = 0; i < c->info.num_columns && !rc; ++i) {
      const fory_column& h = host_cols[i];
      rc = hcopy(B.cols[i].values, static_cast<const uint8_t*>(h.values) + a * c->width[i], (size_t)(rows * c->width[i]), hipMemcpyHostToDevice, c->s_in, "H2D");
      if (!rc && c->nullable[i] && h.validity)
        rc = hcopy(B.cols[i].validity, h.validity + a / 8, (size_t)((rows + 7) / 8), hipMemcpyHostToDevice, c->s_in, "H2D validity");
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
    // D2H: the chunk's rows into the window(s) holding them
    if (!rc) rc = hip_check(hipStreamWaitEvent(c->s_out, c->ev_k[b], 0), "hipStreamWaitEvent");
    if (!rc) rc = d2h_rows_windows(*W, B.rows, a, rows, stride, c->s_out);
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

}  // namespace

extern "C" {

int fory_rowfmt_host_encode(fory_host_ctx* c, const fory_column* host_cols, int64_t n, int32_t frame,
                            void* host_out, int64_t out_capacity) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  if (n > 0 && !host_out) return fail_host(FORY_ERR_INVALID_ARGUMENT, "output is null");
  OutWindows W;
  W.ptr = {static_cast<uint8_t*>(host_out)};
  W.cap = {out_capacity};
  return host_encode_fixed(c, host_cols, n, frame, &W);
}

int fory_rowfmt_host_decode(fory_host_ctx* c, const void* host_rows, int64_t rows_bytes, int64_t n, int32_t frame,
                            const fory_column* host_out_cols) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  if (c->varlen) return fail_host(FORY_ERR_INVALID_ARGUMENT, "varlen plan: use fory_rowfmt_host_decode_var");
  if (frame != FORY_FRAME_RAW && frame != FORY_FRAME_STREAM && frame != FORY_FRAME_HASHED)
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "frame_mode must be 0 (raw), 1 (stream) or 3 (hashed)");
  if (n < 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "num_rows < 0");
  if (n == 0) return FORY_OK;
  if (!host_rows || !host_out_cols) return fail_host(FORY_ERR_INVALID_ARGUMENT, "host rows or output columns null");
  const int64_t stride = c->info.fixed_size + (frame == FORY_FRAME_STREAM ? 12 : frame == FORY_FRAME_HASHED ? 8 : 0);
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
      rc = hcopy(B.rows, in + a * stride, (size_t)(rows * stride), hipMemcpyHostToDevice, c->s_in, "H2D");
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
      rc = hcopy(static_cast<uint8_t*>(h.values) + a * c->width[i], B.cols[i].values, (size_t)(rows * c->width[i]), hipMemcpyDeviceToHost, c->s_out, "D2H");
      if (!rc && dcols[i].validity)
        rc = hcopy(h.validity + a / 8, B.cols[i].validity, (size_t)((rows + 7) / 8), hipMemcpyDeviceToHost, c->s_out, "D2H validity");
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


// ---------------------------------------------------------------------------
// Varlen plans (strings, lists, maps, nested structs, collection frames): the
// whole batch per call. Row sizes are data-dependent, so the chunk pipeline's
// fixed strides do not apply; device buffers live in the context and grow.
// ---------------------------------------------------------------------------

}  // extern "C"

namespace {

constexpr int32_t kKindFixed = 0, kKindBool = 1, kKindBytes = 2, kKindStruct = 3, kKindList = 4, kKindMap = 5;

bool has_offsets(int32_t k) { return k == kKindBytes || k == kKindList || k == kKindMap; }

// Grows a context-owned device buffer (synchronising the context's stream first).
// Regrowing dbuf or drows frees what a staged decode (host_decode_var_sizes ->
// host_decode_var) points into, so it also drops that staged state.
int ensure(fory_host_ctx* c, uint8_t** buf, int64_t* have, int64_t need) {
  if (need <= *have) return FORY_OK;
  if (buf == &c->dbuf || buf == &c->drows) c->dec_n = -1;
  int rc = hip_check(hipStreamSynchronize(c->s_k), "hipStreamSynchronize");
  if (rc) return rc;
  if (*buf) (void)hipFree(*buf);
  *buf = nullptr;
  *have = 0;
  const int64_t sz = align_up(need + need / 4);
  rc = hip_check(hipMalloc(buf, (size_t)sz), "hipMalloc(host ctx varlen buffers)");
  if (!rc) *have = sz;
  return rc;
}

// Carves per-column device regions (values, offsets, validity) for the element
// counts / value bytes given, then row offsets (n+1 int64), the workspace and the
// status word; returns the bytes needed when base is null.
int64_t carve(fory_host_ctx* c, uint8_t* base, const std::vector<int64_t>& cnt, const std::vector<int64_t>& vbytes,
              const std::vector<char>& want_validity, int64_t n, std::vector<fory_column>* cols, int64_t** d_offs,
              void** ws, int64_t ws_bytes, int32_t** status) {
  int64_t at = 0;
  const int N = (int)cnt.size();
  if (cols) cols->assign(N, fory_column{});
  for (int i = 0; i < N; ++i) {
    fory_column d{};
    d.length = cnt[i];
    if (vbytes[i] > 0 || c->kind[i] == kKindFixed || c->kind[i] == kKindBool || c->kind[i] == kKindBytes) {
      d.values = base ? base + at : nullptr;
      d.capacity = vbytes[i];
      at += align_up(vbytes[i] > 0 ? vbytes[i] : 1);
    }
    if (has_offsets(c->kind[i]) && cnt[i] >= 0) {
      d.offsets = base ? reinterpret_cast<int32_t*>(base + at) : nullptr;
      at += align_up((cnt[i] + 1) * 4);
    }
    if (want_validity[i]) {
      d.validity = base ? base + at : nullptr;
      at += align_up(validity_bytes(cnt[i] > 0 ? cnt[i] : 1));
    }
    if (cols) (*cols)[i] = d;
  }
  if (d_offs) *d_offs = base ? reinterpret_cast<int64_t*>(base + at) : nullptr;
  at += align_up((n + 1) * 8);
  if (ws) *ws = base ? base + at : nullptr;
  at += align_up(ws_bytes);
  if (status) *status = base ? reinterpret_cast<int32_t*>(base + at) : nullptr;
  at += kAlign;
  return at;
}

}  // namespace

namespace {

int host_encode_var(fory_host_ctx* c, const fory_column* host_cols, int64_t n, int32_t frame, OutWindows* W,
                    int64_t* host_row_offsets, int64_t* out_bytes) {
  if (!c->varlen) return fail_host(FORY_ERR_INVALID_ARGUMENT, "fixed-width plan: use fory_rowfmt_host_encode");
  if (n < 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "num_rows < 0");
  if (out_bytes) *out_bytes = 0;
  if (n == 0) {
    if (host_row_offsets) host_row_offsets[0] = 0;
    return FORY_OK;
  }
  if (!host_cols) return fail_host(FORY_ERR_INVALID_ARGUMENT, "host columns are null");
  // the encode reuses the device buffers a staged decode lives in: a later
  // host_decode_var must be preceded by a fresh host_decode_var_sizes
  c->dec_n = -1;
  const int N = c->info.num_columns;
  // element count and value bytes of every column, from the host offsets
  std::vector<int64_t> cnt(N, 0), vbytes(N, 0);
  std::vector<char> want_validity(N, 0);
  for (int i = 0; i < N; ++i) {
    const int p = c->parent[i];
    if (p < 0) cnt[i] = n;
    else if (c->kind[p] == kKindStruct) cnt[i] = cnt[p];
    else cnt[i] = cnt[p] > 0 ? host_cols[p].offsets[cnt[p]] : 0;  // list items / map entries
    const fory_column& h = host_cols[i];
    if (has_offsets(c->kind[i]) && !h.offsets)
      return fail_host(FORY_ERR_INVALID_ARGUMENT, "column " + std::to_string(i) + " needs offsets");
    if (c->kind[i] == kKindFixed || c->kind[i] == kKindBool) vbytes[i] = cnt[i] * c->width[i];
    else if (c->kind[i] == kKindBytes) vbytes[i] = cnt[i] > 0 ? h.offsets[cnt[i]] : 0;
    if (vbytes[i] > 0 && !h.values)
      return fail_host(FORY_ERR_INVALID_ARGUMENT, "column " + std::to_string(i) + " has no values");
    want_validity[i] = c->nullable[i] && h.validity;
  }
  int rc = hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  const int64_t ws_bytes = fory_rowfmt_workspace_bytes(c->plan, n);
  rc = ensure(c, &c->dbuf, &c->dbuf_bytes, carve(c, nullptr, cnt, vbytes, want_validity, n, nullptr, nullptr,
                                                 nullptr, ws_bytes, nullptr));
  if (rc) return rc;
  std::vector<fory_column> d;
  int64_t* d_offs = nullptr;
  void* ws = nullptr;
  int32_t* status = nullptr;
  carve(c, c->dbuf, cnt, vbytes, want_validity, n, &d, &d_offs, &ws, ws_bytes, &status);
  for (int i = 0; i < N && !rc; ++i) {  // H2D of every column
    const fory_column& h = host_cols[i];
    if (d[i].values && vbytes[i] > 0)
      rc = hcopy(d[i].values, h.values, (size_t)vbytes[i], hipMemcpyHostToDevice, c->s_k, "H2D");
    if (!rc && d[i].offsets)
      rc = hcopy(d[i].offsets, h.offsets, (size_t)(cnt[i] + 1) * 4, hipMemcpyHostToDevice, c->s_k, "H2D offsets");
    if (!rc && d[i].validity)
      rc = hcopy(d[i].validity, h.validity, (size_t)((cnt[i] + 7) / 8), hipMemcpyHostToDevice, c->s_k, "H2D validity");
  }
  if (!rc) rc = hip_check(hipMemsetAsync(status, 0, 4, c->s_k), "hipMemsetAsync");
  if (!rc) rc = fory_rowfmt_encoded_size(c->plan, d.data(), n, frame, d_offs, ws, ws_bytes, c->s_k);
  // row/frame offsets to the host: the split into the caller's windows needs them
  std::vector<int64_t> tmp;
  int64_t* ho = host_row_offsets;
  if (!ho) {
    tmp.resize((size_t)n + 1);
    ho = tmp.data();
  }
  if (!rc) rc = hcopy(ho, d_offs, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, c->s_k, "D2H offsets");
  if (!rc) rc = hip_check(hipStreamSynchronize(c->s_k), "hipStreamSynchronize");
  if (rc) return rc;
  const int64_t total = ho[n];
  if (out_bytes) *out_bytes = total;
  rc = split_rows(ho, 0, n, W);  // MemoryBuffer bounds check (MemoryBuffer.java:303-309)
  if (rc) return rc;
  for (size_t w = 0; w + 1 < W->first.size(); ++w)
    if (W->first[w + 1] > W->first[w] && !W->ptr[w]) return fail_host(FORY_ERR_INVALID_ARGUMENT, "output is null");
  rc = ensure(c, &c->drows, &c->drows_bytes, total + 16);
  if (!rc) rc = fory_rowfmt_encode(c->plan, d.data(), n, frame, d_offs, c->drows, total, status, ws, ws_bytes, c->s_k);
  for (size_t w = 0; w + 1 < W->first.size() && !rc; ++w) {  // each window: its rows' contiguous bytes
    const int64_t lo = ho[W->first[w]], hi = ho[W->first[w + 1]];
    if (hi > lo)
      rc = hcopy(W->ptr[w], c->drows + lo, (size_t)(hi - lo), hipMemcpyDeviceToHost, c->s_k, "D2H rows");
  }
  if (!rc) rc = fory_rowfmt_read_status(status, c->s_k);  // synchronises the stream
  return rc;
}

}  // namespace

extern "C" {

int fory_rowfmt_host_encode_var(fory_host_ctx* c, const fory_column* host_cols, int64_t n, int32_t frame,
                                void* host_out, int64_t out_capacity, int64_t* host_row_offsets,
                                int64_t* out_bytes) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  OutWindows W;
  W.ptr = {static_cast<uint8_t*>(host_out)};
  W.cap = {out_capacity};
  return host_encode_var(c, host_cols, n, frame, &W, host_row_offsets, out_bytes);
}

int fory_rowfmt_host_encode_windows(fory_host_ctx* c, const fory_column* host_cols, int64_t n, int32_t frame,
                                    void* const* windows, const int64_t* window_caps, int32_t num_windows,
                                    int64_t* window_rows, int64_t* window_bytes) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  if (num_windows <= 0 || !windows || !window_caps)
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "windows / window_caps null or num_windows <= 0");
  OutWindows W;
  for (int32_t w = 0; w < num_windows; ++w) {
    if (window_caps[w] < 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "window capacity < 0");
    W.ptr.push_back(static_cast<uint8_t*>(windows[w]));
    W.cap.push_back(window_caps[w]);
  }
  int rc;
  int64_t stride = 0;
  std::vector<int64_t> offs;
  if (c->varlen) {
    offs.resize((size_t)(n > 0 ? n : 0) + 1, 0);
    rc = host_encode_var(c, host_cols, n, frame, &W, offs.data(), nullptr);
  } else {
    stride = c->info.fixed_size + (frame == FORY_FRAME_STREAM ? 12 : frame == FORY_FRAME_HASHED ? 8 : 0);
    rc = host_encode_fixed(c, host_cols, n, frame, &W);
  }
  if (rc) return rc;
  if (W.first.size() != (size_t)num_windows + 1) W.first.assign((size_t)num_windows + 1, 0);
  for (int32_t w = 0; w < num_windows; ++w) {
    const int64_t f0 = W.first[(size_t)w], f1 = W.first[(size_t)w + 1];
    if (window_rows) window_rows[w] = f1 - f0;
    if (window_bytes) window_bytes[w] = c->varlen ? offs[(size_t)f1] - offs[(size_t)f0] : (f1 - f0) * stride;
  }
  return FORY_OK;
}

}  // extern "C"

namespace {

// Stages a decode batch on the device: rows (host_row_offsets given: the run
// [offs[0], offs[n]) with offsets rebased to it; else the first rows_bytes bytes of
// a frame stream, indexed on the device by fory_rowfmt_index_frames) and sizes
// every output column (fory_rowfmt_decode_sizes, repeated while list/map element
// counts become known). The staged state serves the next host_decode_var.
int decode_var_stage(fory_host_ctx* c, const void* host_rows, const int64_t* host_row_offsets, int64_t rows_bytes,
                     int64_t n, int32_t frame, int64_t* host_counts, int64_t* host_bytes, int64_t* consumed) {
  const int N = c->info.num_columns;
  c->dec_n = -1;
  int64_t r0 = 0, r1 = rows_bytes;
  if (host_row_offsets) {
    r0 = host_row_offsets[0];
    r1 = host_row_offsets[n];
    if (r1 < r0 || r0 < 0) return fail_host(FORY_ERR_CORRUPT, "row offsets decrease");
  }
  int rc = hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  // device run: [rows (16-byte aligned start)][row offsets n+1][index status][index workspace]
  const int64_t rows_sz = align_up((r1 - r0) + 16), offs_sz = align_up((n + 1) * 8);
  const int64_t iws = host_row_offsets ? 0 : fory_rowfmt_index_workspace_bytes(c->plan, n, r1 - r0);
  rc = ensure(c, &c->drows, &c->drows_bytes, rows_sz + offs_sz + kAlign + iws);
  if (rc) return rc;
  uint8_t* drow0 = c->drows;
  int64_t* d_offs = reinterpret_cast<int64_t*>(c->drows + rows_sz);
  int32_t* istatus = reinterpret_cast<int32_t*>(c->drows + rows_sz + offs_sz);
  if (r1 > r0)
    rc = hcopy(drow0, static_cast<const uint8_t*>(host_rows) + r0, (size_t)(r1 - r0), hipMemcpyHostToDevice, c->s_k, "H2D rows");
  if (host_row_offsets) {  // row offsets relative to the staged run
    std::vector<int64_t> rel_offs((size_t)n + 1);
    for (int64_t k = 0; k <= n; ++k) rel_offs[(size_t)k] = host_row_offsets[k] - r0;
    if (!rc)
      rc = hcopy(d_offs, rel_offs.data(), (size_t)(n + 1) * 8, hipMemcpyHostToDevice, c->s_k, "H2D row offsets");
    if (!rc) rc = hip_check(hipStreamSynchronize(c->s_k), "hipStreamSynchronize");  // rel_offs is pageable
    if (consumed) *consumed = r1;
  } else {  // Encoder.decode(MemoryBuffer) x n over the stream alone
    if (!rc) rc = hip_check(hipMemsetAsync(istatus, 0, 4, c->s_k), "hipMemsetAsync");
    if (!rc)
      rc = fory_rowfmt_index_frames(c->plan, drow0, r1 - r0, n, frame, d_offs, istatus,
                                    c->drows + rows_sz + offs_sz + kAlign, iws, c->s_k);
    int64_t end = 0;
    if (!rc) rc = hcopy(&end, d_offs + n, 8, hipMemcpyDeviceToHost, c->s_k, "D2H frame end");
    if (!rc) rc = fory_rowfmt_read_status(istatus, c->s_k);  // synchronises the stream
    if (rc) return rc;
    if (consumed) *consumed = end;
  }
  if (rc) return rc;
  // element counts: top level n; struct fields as their struct; list/map elements
  // from the container totals (pass 1), string/binary elements' bytes (pass 2)
  std::vector<int64_t> cnt(N, -1), vbytes(N, 0);
  std::vector<char> want_validity(N, 0);
  for (int i = 0; i < N; ++i) want_validity[i] = c->nullable[i] != 0;
  auto resolve = [&]() {
    for (int i = 0; i < N; ++i) {
      const int p = c->parent[i];
      if (cnt[i] >= 0) continue;
      if (p < 0) cnt[i] = n;
      else if (cnt[p] >= 0 && c->kind[p] == kKindStruct) cnt[i] = cnt[p];
    }
  };
  resolve();
  const int64_t ws_bytes = fory_rowfmt_workspace_bytes(c->plan, n);
  std::vector<fory_column> d;
  void* ws = nullptr;
  int32_t* status = nullptr;
  for (int pass = 0; pass < 20 && !rc; ++pass) {  // one level of list/map nesting per pass (<= 17)
    // layout for the counts known so far (unknown: no buffers, length 0)
    std::vector<int64_t> kc(N);
    for (int i = 0; i < N; ++i) kc[i] = cnt[i] < 0 ? -1 : cnt[i];
    std::vector<int64_t> vb0(N, 0);
    std::vector<char> wv(N, 0);
    rc = ensure(c, &c->dbuf, &c->dbuf_bytes, carve(c, nullptr, kc, vb0, wv, n, nullptr, nullptr, nullptr, ws_bytes,
                                                   nullptr));
    if (rc) break;
    carve(c, c->dbuf, kc, vb0, wv, n, &d, nullptr, &ws, ws_bytes, &status);
    for (int i = 0; i < N; ++i) {
      d[i].values = nullptr;
      d[i].capacity = 0;
      if (kc[i] < 0) d[i] = fory_column{};
    }
    rc = hip_check(hipMemsetAsync(status, 0, 4, c->s_k), "hipMemsetAsync");
    if (!rc)
      rc = fory_rowfmt_decode_sizes(c->plan, drow0, d_offs, n, frame, d.data(), status, ws, ws_bytes, c->s_k);
    std::vector<int32_t> tot(N, 0);
    for (int i = 0; i < N && !rc; ++i)
      if (d[i].offsets && kc[i] >= 0)
        rc = hcopy(&tot[i], d[i].offsets + kc[i], 4, hipMemcpyDeviceToHost, c->s_k, "D2H totals");
    if (!rc) rc = fory_rowfmt_read_status(status, c->s_k);
    if (rc) break;
    bool changed = false;
    for (int i = 0; i < N; ++i) {
      if (!has_offsets(c->kind[i]) || kc[i] < 0) continue;
      if (c->kind[i] == kKindBytes) vbytes[i] = tot[i];
      else
        for (int j = 0; j < N; ++j)  // direct children of a list/map: its element total
          if (c->parent[j] == i && cnt[j] < 0) cnt[j] = tot[i], changed = true;
    }
    resolve();
    if (!changed) break;
  }
  if (rc) return rc;
  for (int i = 0; i < N; ++i) {
    if (cnt[i] < 0) cnt[i] = 0;
    if (c->kind[i] == kKindFixed || c->kind[i] == kKindBool) vbytes[i] = cnt[i] * c->width[i];
    host_counts[i] = cnt[i];
    host_bytes[i] = vbytes[i];
  }
  c->dec_n = n;
  c->dec_frame = frame;
  c->dec_count = cnt;
  c->dec_bytes = vbytes;
  c->dec_cols = d;  // the last pass's device offsets (tile bases / totals for decode)
  c->dec_offs = d_offs;  // in the drows run
  c->dec_ws = ws;
  c->dec_status = status;
  return FORY_OK;
}

}  // namespace

extern "C" {

int fory_rowfmt_host_decode_var_sizes(fory_host_ctx* c, const void* host_rows, const int64_t* host_row_offsets,
                                      int64_t n, int32_t frame, int64_t* host_counts, int64_t* host_bytes) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  if (!c->varlen) return fail_host(FORY_ERR_INVALID_ARGUMENT, "fixed-width plan: use fory_rowfmt_host_decode");
  if (n < 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "num_rows < 0");
  if (!host_row_offsets || !host_counts || !host_bytes || (n > 0 && !host_rows))
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "host rows, row offsets or size outputs null");
  return decode_var_stage(c, host_rows, host_row_offsets, 0, n, frame, host_counts, host_bytes, nullptr);
}

int fory_rowfmt_host_decode_stream_sizes(fory_host_ctx* c, const void* host_rows, int64_t rows_bytes, int64_t n,
                                         int64_t* host_counts, int64_t* host_bytes, int64_t* consumed_bytes) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  if (!c->varlen) return fail_host(FORY_ERR_INVALID_ARGUMENT, "fixed-width plan: use fory_rowfmt_host_decode");
  if (n < 0 || rows_bytes < 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "num_rows or rows_bytes < 0");
  if (!host_counts || !host_bytes || (n > 0 && !host_rows))
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "host rows or size outputs null");
  return decode_var_stage(c, host_rows, nullptr, rows_bytes, n, FORY_FRAME_STREAM, host_counts, host_bytes,
                          consumed_bytes);
}

int fory_rowfmt_host_decode_var(fory_host_ctx* c, const fory_column* host_out_cols) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  if (!c->varlen || c->dec_n < 0)
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "call fory_rowfmt_host_decode_var_sizes first");
  const int N = c->info.num_columns;
  const int64_t n = c->dec_n;
  if (n > 0 && !host_out_cols) return fail_host(FORY_ERR_INVALID_ARGUMENT, "host output columns null");
  for (int i = 0; i < N && n > 0; ++i) {
    const fory_column& h = host_out_cols[i];
    if (c->dec_bytes[i] > 0 && (!h.values || (h.capacity > 0 && h.capacity < c->dec_bytes[i])))
      return fail_host(FORY_ERR_CAPACITY, "output column " + std::to_string(i) + " values missing or too small");
    if (has_offsets(c->kind[i]) && !h.offsets)
      return fail_host(FORY_ERR_INVALID_ARGUMENT, "output column " + std::to_string(i) + " needs offsets");
  }
  if (n == 0) {
    for (int i = 0; i < N; ++i)
      if (host_out_cols && host_out_cols[i].offsets) host_out_cols[i].offsets[0] = 0;
    return FORY_OK;
  }
  int rc = hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  std::vector<char> wv(N, 0);
  for (int i = 0; i < N; ++i) wv[i] = c->nullable[i] && host_out_cols[i].validity;
  const int64_t ws_bytes = fory_rowfmt_workspace_bytes(c->plan, n);
  // output columns in their own buffer (the row offsets / workspace stay in dbuf)
  rc = ensure(c, &c->dout, &c->dout_bytes, carve(c, nullptr, c->dec_count, c->dec_bytes, wv, 0, nullptr, nullptr,
                                                 nullptr, 0, nullptr));
  if (rc) return rc;
  std::vector<fory_column> d;
  carve(c, c->dout, c->dec_count, c->dec_bytes, wv, 0, &d, nullptr, nullptr, 0, nullptr);
  const std::vector<int64_t>& kc = c->dec_count;
  const std::vector<fory_column>& dsz = c->dec_cols;
  int64_t* d_offs = c->dec_offs;
  void* ws = c->dec_ws;
  int32_t* status = c->dec_status;
  // the sizes pass wrote the offsets into dbuf's column regions: copy them over
  for (int i = 0; i < N && !rc; ++i) {
    if (d[i].offsets && dsz[i].offsets)
      rc = hip_check(hipMemcpyAsync(d[i].offsets, dsz[i].offsets, (size_t)(kc[i] + 1) * 4, hipMemcpyDeviceToDevice,
                                    c->s_k), "D2D offsets");
    if (!rc && d[i].validity)
      rc = hip_check(hipMemsetAsync(d[i].validity, 0, (size_t)validity_bytes(kc[i] > 0 ? kc[i] : 1), c->s_k),
                     "hipMemsetAsync");
  }
  if (!rc) rc = hip_check(hipMemsetAsync(status, 0, 4, c->s_k), "hipMemsetAsync");
  if (!rc)
    rc = fory_rowfmt_decode(c->plan, c->drows, d_offs, n, c->dec_frame, d.data(), status, ws, ws_bytes, c->s_k);
  for (int i = 0; i < N && !rc; ++i) {  // D2H of every column
    const fory_column& h = host_out_cols[i];
    if (d[i].values && c->dec_bytes[i] > 0)
      rc = hcopy(h.values, d[i].values, (size_t)c->dec_bytes[i], hipMemcpyDeviceToHost, c->s_k, "D2H values");
    if (!rc && d[i].offsets)
      rc = hcopy(h.offsets, d[i].offsets, (size_t)(kc[i] + 1) * 4, hipMemcpyDeviceToHost, c->s_k, "D2H offsets");
    if (!rc && d[i].validity)
      rc = hcopy(h.validity, d[i].validity, (size_t)((kc[i] + 7) / 8), hipMemcpyDeviceToHost, c->s_k, "D2H validity");
  }
  if (!rc) rc = fory_rowfmt_read_status(status, c->s_k);
  return rc;
}

}  // extern "C"
