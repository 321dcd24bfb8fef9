// copybw.hip — what mixed read+write HBM rate is achievable on this box?
// (diagnostic tool, not product code). Build:
//   hipcc -O3 --offload-arch=gfx950 copybw.hip -o copybw
// Variants: hipMemcpy D2D; grid-stride 16-B copy at several grids / block sizes;
// one-shot (non-persistent) copies with U chunks per lane; contiguous per-WG
// blocks; non-temporal loads / stores; read-only and write-only references.
// Prints one JSON line per (variant, size); GB/s counts read + written bytes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NTL, bool NTS>
__global__ void copy_gs(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const size_t s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) {
    u32x4 x = NTL ? __builtin_nontemporal_load(a + i) : a[i];
    if (NTS) __builtin_nontemporal_store(x, b + i);
    else b[i] = x;
  }
}

// one-shot: workgroup of 256 handles 256*U consecutive chunks, all loads first
template <int U, bool NTS>
__global__ __launch_bounds__(256) void copy_once(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
  const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  u32x4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = base + u * 256 < n ? a[base + u * 256] : u32x4{0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (base + u * 256 < n) {
      if (NTS) __builtin_nontemporal_store(x[u], b + base + u * 256);
      else b[base + u * 256] = x[u];
    }
}

// persistent, each WG walks contiguous blocks of 256*U chunks, loads of block k+1
// issued before stores of block k (depth-2 register pipeline)
template <int U>
__global__ __launch_bounds__(256) void copy_blk(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
  const size_t nb = n / (256 * U);
  size_t k = blockIdx.x;
  if (k >= nb) return;
  u32x4 x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = a[k * 256 * U + u * 256 + threadIdx.x];
  for (;;) {
    const size_t k2 = k + gridDim.x;
    const size_t kl = k2 < nb ? k2 : k;
#pragma unroll
    for (int u = 0; u < U; ++u) y[u] = a[kl * 256 * U + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < U; ++u) b[k * 256 * U + u * 256 + threadIdx.x] = x[u];
    if (k2 >= nb) break;
    k = k2;
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = y[u];
  }
}

// persistent, tiles of 256*U chunks handed out in order by an atomic counter
// (next tile fetched while the current one is in flight): in-flight addresses
// stay a compact window like the one-shot grid's, without per-WG drift.
template <int U>
__global__ __launch_bounds__(256) void copy_dyn(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n,
                                                unsigned* ctr) {
  __shared__ unsigned nxt[2];
  const size_t nt = n / (256 * U);
  if (threadIdx.x == 0) nxt[0] = atomicAdd(ctr, 1u);
  __syncthreads();
  unsigned c = nxt[0];
  int par = 1;
  while (c < nt) {
    if (threadIdx.x == 0) nxt[par] = atomicAdd(ctr, 1u);
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = a[(size_t)c * 256 * U + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < U; ++u) b[(size_t)c * 256 * U + u * 256 + threadIdx.x] = x[u];
    __syncthreads();
    c = nxt[par];
    par ^= 1;
  }
}

__global__ void read_only(const u32x4* __restrict__ a, size_t n, unsigned* sink) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const size_t s = (size_t)gridDim.x * blockDim.x;
  unsigned acc = 0;
  for (; i < n; i += s) {
    u32x4 x = a[i];
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ void write_only(u32x4* __restrict__ b, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const size_t s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) b[i] = u32x4{(unsigned)i, 1, 2, 3};
}

template <class F>
float time_ms(F f, int reps = 5) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  f();
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(e0, 0));
    f();
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  CHECK(hipGetLastError());
  return best;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const size_t maxb = 16L << 30;
  u32x4 *a, *b;
  unsigned* sink;
  CHECK(hipMalloc(&a, maxb));
  CHECK(hipMalloc(&b, maxb));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(a, 1, maxb));
  CHECK(hipMemset(b, 0, maxb));
  auto out = [](const char* t, size_t bytes, int grid, int blk, float ms, double moved) {
    printf("{\"test\":\"%s\",\"bytes\":%zu,\"grid\":%d,\"block\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", t, bytes, grid, blk, ms,
           moved / ms / 1e6);
    fflush(stdout);
  };
  for (size_t nb : {4L << 30, 16L << 30}) {
    const size_t n = nb / 16;
    float ms = time_ms([&] { CHECK(hipMemcpyAsync(b, a, nb, hipMemcpyDeviceToDevice, 0)); });
    out("memcpy_d2d", nb, 0, 0, ms, 2.0 * nb);
    for (int blk : {256}) {
      for (int wpc : {2, 4, 8, 16}) {
        const int g = cus * wpc * 256 / blk;
        ms = time_ms([&] { hipLaunchKernelGGL((copy_gs<false, false>), dim3(g), dim3(blk), 0, 0, a, b, n); });
        out("copy_gs", nb, g, blk, ms, 2.0 * nb);
      }
    }
    for (int wpc : {4, 8}) {
      const int g = cus * wpc;
      ms = time_ms([&] { hipLaunchKernelGGL((copy_gs<true, false>), dim3(g), dim3(256), 0, 0, a, b, n); });
      out("copy_gs_ntload", nb, g, 256, ms, 2.0 * nb);
      ms = time_ms([&] { hipLaunchKernelGGL((copy_gs<false, true>), dim3(g), dim3(256), 0, 0, a, b, n); });
      out("copy_gs_ntstore", nb, g, 256, ms, 2.0 * nb);
      ms = time_ms([&] { hipLaunchKernelGGL((copy_gs<true, true>), dim3(g), dim3(256), 0, 0, a, b, n); });
      out("copy_gs_nt_both", nb, g, 256, ms, 2.0 * nb);
      ms = time_ms([&] { hipLaunchKernelGGL((copy_blk<4>), dim3(g), dim3(256), 0, 0, a, b, n); });
      out("copy_blk4", nb, g, 256, ms, 2.0 * nb);
      ms = time_ms([&] { hipLaunchKernelGGL((copy_blk<8>), dim3(g), dim3(256), 0, 0, a, b, n); });
      out("copy_blk8", nb, g, 256, ms, 2.0 * nb);
      ms = time_ms([&] { hipLaunchKernelGGL(read_only, dim3(g), dim3(256), 0, 0, a, n, sink); });
      out("read_only", nb, g, 256, ms, 1.0 * nb);
      ms = time_ms([&] { hipLaunchKernelGGL(write_only, dim3(g), dim3(256), 0, 0, b, n); });
      out("write_only", nb, g, 256, ms, 1.0 * nb);
    }
    unsigned* ctr = sink + 4;
    for (int wpc : {4, 8}) {
      const int g = cus * wpc;
      ms = time_ms([&] {
        CHECK(hipMemsetAsync(ctr, 0, 4, 0));
        hipLaunchKernelGGL((copy_dyn<1>), dim3(g), dim3(256), 0, 0, a, b, n, ctr);
      });
      out("copy_dyn1", nb, g, 256, ms, 2.0 * nb);
      ms = time_ms([&] {
        CHECK(hipMemsetAsync(ctr, 0, 4, 0));
        hipLaunchKernelGGL((copy_dyn<4>), dim3(g), dim3(256), 0, 0, a, b, n, ctr);
      });
      out("copy_dyn4", nb, g, 256, ms, 2.0 * nb);
    }
    {
      int g = (int)(n / 256);
      ms = time_ms([&] { hipLaunchKernelGGL((copy_once<1, false>), dim3(g), dim3(256), 0, 0, a, b, n); });
      out("copy_once1", nb, g, 256, ms, 2.0 * nb);
      g = (int)(n / 1024);
      ms = time_ms([&] { hipLaunchKernelGGL((copy_once<4, false>), dim3(g), dim3(256), 0, 0, a, b, n); });
      out("copy_once4", nb, g, 256, ms, 2.0 * nb);
      ms = time_ms([&] { hipLaunchKernelGGL((copy_once<4, true>), dim3(g), dim3(256), 0, 0, a, b, n); });
      out("copy_once4_ntstore", nb, g, 256, ms, 2.0 * nb);
    }
  }
  return 0;
}
