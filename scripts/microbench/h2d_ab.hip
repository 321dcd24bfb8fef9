// H2D of a Struct104 chunk's columns (104 x 8 B x 1M rows, registered host memory)
// while the previous chunk's rows go D2H, the host path's duplex pattern:
//   A: one hipMemcpyAsync per column (today's host_encode)
//   B: one copy of the same bytes (upper bound of batching)
//   C: a gather kernel reading the mapped host columns over PCIe (zero-copy)
// Usage: h2d_ab [rows] [reg]  (prints GB/s of the H2D leg and of the concurrent D2H;
// reg: host buffers are malloc'd and hipHostRegister'd, as a caller's heap arrays are,
// instead of hipHostMalloc'd)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

struct Cols {
  const uint4* src[104];
};

__global__ void gather_kernel(Cols c, uint4* dst, int64_t words_per_col) {
  const int col = blockIdx.y;
  const uint4* s = c.src[col];
  uint4* d = dst + col * words_per_col;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words_per_col; i += (int64_t)gridDim.x * blockDim.x)
    d[i] = s[i];
}

int main(int argc, char** argv) {
  const int64_t rows = argc > 1 ? atoll(argv[1]) : (1 << 20);
  const int ncol = 104;
  const size_t col_bytes = rows * 8, total = col_bytes * ncol;
  const bool reg = argc > 2 && !strcmp(argv[2], "reg");
  auto host_alloc = [&](void** p, size_t n) {
    if (!reg) {
      CK(hipHostMalloc(p, n, hipHostMallocDefault));
      return;
    }
    *p = aligned_alloc(4096, (n + 4095) / 4096 * 4096);
    memset(*p, 0, n);
    CK(hipHostRegister(*p, n, hipHostRegisterMapped));
  };
  std::vector<void*> h(ncol);
  for (int i = 0; i < ncol; ++i) {
    host_alloc(&h[i], col_bytes);
    memset(h[i], i, col_bytes);
  }
  void* hrows = nullptr;
  host_alloc(&hrows, total + 16 * rows);
  void *dcols = nullptr, *drows = nullptr;
  CK(hipMalloc(&dcols, total));
  CK(hipMalloc(&drows, total + 16 * rows));
  hipStream_t s_in, s_out;
  CK(hipStreamCreateWithFlags(&s_in, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s_out, hipStreamNonBlocking));
  Cols c;
  for (int i = 0; i < ncol; ++i) {
    void* dp = nullptr;
    CK(hipHostGetDevicePointer(&dp, h[i], 0));
    c.src[i] = static_cast<const uint4*>(dp);
  }
  hipEvent_t a0, a1, b0, b1;
  CK(hipEventCreate(&a0));
  CK(hipEventCreate(&a1));
  CK(hipEventCreate(&b0));
  CK(hipEventCreate(&b1));
  const size_t out_bytes = total + 16 * rows;
  for (int mode = 0; mode < 3; ++mode) {
    for (int duplex = 0; duplex < 2; ++duplex) {
      float best_in = 1e9, best_out = 1e9;
      for (int it = 0; it < 4; ++it) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a0, s_in));
        if (duplex) {
          CK(hipEventRecord(b0, s_out));
          CK(hipMemcpyAsync(hrows, drows, out_bytes, hipMemcpyDeviceToHost, s_out));
          CK(hipEventRecord(b1, s_out));
        }
        if (mode == 0) {
          for (int i = 0; i < ncol; ++i)
            CK(hipMemcpyAsync(static_cast<uint8_t*>(dcols) + i * col_bytes, h[i], col_bytes, hipMemcpyHostToDevice, s_in));
        } else if (mode == 1) {
          CK(hipMemcpyAsync(static_cast<uint8_t*>(dcols), hrows, total, hipMemcpyHostToDevice, s_in));
        } else {
          hipLaunchKernelGGL(gather_kernel, dim3(16, ncol), dim3(256), 0, s_in, c, static_cast<uint4*>(dcols),
                             (int64_t)(col_bytes / 16));
        }
        CK(hipEventRecord(a1, s_in));
        CK(hipDeviceSynchronize());
        float t_in = 0, t_out = 0;
        CK(hipEventElapsedTime(&t_in, a0, a1));
        if (duplex) CK(hipEventElapsedTime(&t_out, b0, b1));
        if (t_in < best_in) best_in = t_in;
        if (duplex && t_out < best_out) best_out = t_out;
      }
      printf("{\"host\": \"%s\", \"mode\": \"%s\", \"duplex\": %d, \"h2d_ms\": %.3f, \"h2d_GBps\": %.1f, \"d2h_GBps\": %.1f}\n",
             reg ? "registered" : "hipHostMalloc", mode == 0 ? "per_column" : mode == 1 ? "one_copy" : "gather_kernel",
             duplex, best_in,
             total / best_in / 1e6, duplex ? out_bytes / best_out / 1e6 : 0.0);
    }
  }
  return 0;
}
