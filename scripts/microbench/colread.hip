// colread.hip — standalone HBM microbenchmarks for the encode access pattern
// (diagnostic tool, not product code). Build: hipcc -O3 --offload-arch=gfx950 colread.hip -o colread
//   copy16      : float4 copy (achievable HBM peak on this box)
//   readcols<W> : per tile of R records, read 104 column segments (26 x {4,8,4,8} B)
//                 with W-byte loads per lane — the encode's read pattern
//   writerows   : contiguous 16-B stores of R*848 bytes per tile — the encode's write pattern
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));      \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void copy16(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) b[i] = a[i];
}

// 4 independent 16-B loads in flight per lane
__global__ __launch_bounds__(256) void copy16x4(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
  const size_t s = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i + 3 * s < n; i += 4 * s) {
    u32x4 x0 = a[i], x1 = a[i + s], x2 = a[i + 2 * s], x3 = a[i + 3 * s];
    b[i] = x0; b[i + s] = x1; b[i + 2 * s] = x2; b[i + 3 * s] = x3;
  }
  for (; i < n; i += s) b[i] = a[i];
}

struct Cols {
  const unsigned char* p[104];
};

// lane = record (W = 4/8 per field width) or 16-B chunk (W = 16): loads all
// 104 segments of a tile of R records, XOR-reduces, one store per workgroup.
template <int R, int W>
__global__ __launch_bounds__(256) void readcols(Cols c, long nrows, unsigned* sink) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long tiles = nrows / R;
  unsigned acc = 0;
  for (long t = blockIdx.x; t < tiles; t += gridDim.x) {
    const long r0 = t * R;
    if (W == 16) {
      // segment of field f: R*w bytes = R*w/16 chunks; chunks spread over the block
      unsigned v[26];
#pragma unroll
      for (int u = 0; u < 26; ++u) {
        const int f = __builtin_amdgcn_readfirstlane(wave + 4 * u);
        const int w = (f & 1) ? 8 : 4;
        const int nch = R * w / 16;
        u32x4 x = {0, 0, 0, 0};
        if (lane < nch) x = *(const u32x4*)(c.p[f] + r0 * w + lane * 16);
        v[u] = x.x ^ x.y ^ x.z ^ x.w;
      }
#pragma unroll
      for (int u = 0; u < 26; ++u) acc ^= v[u];
    } else {
      unsigned v[26];
#pragma unroll
      for (int u = 0; u < 26; ++u) {
        const int f = __builtin_amdgcn_readfirstlane(wave + 4 * u);
        if (f & 1) {
          unsigned long long x = 0;
#pragma unroll
          for (int k = 0; k < R / 64; ++k) x ^= *(const unsigned long long*)(c.p[f] + (r0 + lane + 64 * k) * 8);
          v[u] = (unsigned)x ^ (unsigned)(x >> 32);
        } else {
          unsigned x = 0;
#pragma unroll
          for (int k = 0; k < R / 64; ++k) x ^= *(const unsigned*)(c.p[f] + (r0 + lane + 64 * k) * 4);
          v[u] = x;
        }
      }
#pragma unroll
      for (int u = 0; u < 26; ++u) acc ^= v[u];
    }
  }
  if (acc == 0x12345678) sink[blockIdx.x] = acc;
}

// The encode's HBM traffic without LDS: per tile of R records, 16-B/lane
// loads of the 104 column segments, then R*848 contiguous bytes stored
// (values derived from the loads so they are live).
template <int R>
__global__ __launch_bounds__(256) void enc_traffic(Cols c, long nrows, unsigned char* __restrict__ out) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long tiles = nrows / R;
  for (long t = blockIdx.x; t < tiles; t += gridDim.x) {
    const long r0 = t * R;
    unsigned acc = 0;
    // instruction list: int64 fields (R*8/16 chunks each) then int32 fields
    constexpr int C8 = R * 8 / 16, C4 = R * 4 / 16;
    constexpr int I8 = 52 * C8 / 64, I4 = 52 * C4 / 64;
    u32x4 v[(I8 + I4 + 3) / 4];
#pragma unroll
    for (int k = 0; k < (I8 + I4 + 3) / 4; ++k) {
      const int i = wave + 4 * k;
      u32x4 x = {0, 0, 0, 0};
      if (i < I8) {
        const int q = i * 64 + lane;      // chunk among the int64 fields
        const int f = 2 * (q / C8) + 1;   // odd fields are int64
        x = *(const u32x4*)(c.p[f] + r0 * 8 + (q % C8) * 16);
      } else if (i < I8 + I4) {
        const int q = (i - I8) * 64 + lane;
        const int f = 2 * (q / C4);
        x = *(const u32x4*)(c.p[f] + r0 * 4 + (q % C4) * 16);
      }
      v[k] = x;
    }
#pragma unroll
    for (int k = 0; k < (I8 + I4 + 3) / 4; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    unsigned char* d = out + r0 * 848;
    const int n16 = R * 848 / 16;
    u32x4 y = {acc, acc + 1, acc + 2, acc + 3};
    for (int q = tid; q < n16; q += 256) *(u32x4*)(d + q * 16) = y;
  }
}

// The decode's HBM traffic without LDS: per tile of R records, read R*848
// contiguous bytes (16 B/lane), then store the 104 column segments either
// lane = record (4/8-B stores, W=0) or as 16-B chunks (W=16).
template <int R, int W>
__global__ __launch_bounds__(256) void dec_traffic(Cols c, long nrows, const unsigned char* __restrict__ rows) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long tiles = nrows / R;
  for (long t = blockIdx.x; t < tiles; t += gridDim.x) {
    const long r0 = t * R;
    const unsigned char* s = rows + r0 * 848;
    unsigned acc = 0;
    const int n16 = R * 848 / 16;
    u32x4 v[(R * 848 / 16 + 255) / 256];
#pragma unroll
    for (int k = 0; k < (R * 848 / 16 + 255) / 256; ++k) {
      const int q = k * 256 + tid;
      u32x4 x = {0, 0, 0, 0};
      if (q < n16) x = *(const u32x4*)(s + q * 16);
      v[k] = x;
    }
#pragma unroll
    for (int k = 0; k < (R * 848 / 16 + 255) / 256; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    if (W == 16) {
      constexpr int C8 = R * 8 / 16, C4 = R * 4 / 16;
      constexpr int I8 = 52 * C8 / 64, I4 = 52 * C4 / 64;
      for (int i = wave; i < I8 + I4; i += 4) {
        u32x4 y = {acc, acc, acc, acc};
        if (i < I8) {
          const int q = i * 64 + lane;
          *(u32x4*)(c.p[2 * (q / C8) + 1] + r0 * 8 + (q % C8) * 16) = y;
        } else {
          const int q = (i - I8) * 64 + lane;
          *(u32x4*)(c.p[2 * (q / C4)] + r0 * 4 + (q % C4) * 16) = y;
        }
      }
    } else {
      for (int f = wave; f < 104; f += 4) {
        for (int k = 0; k < R / 64; ++k) {
          const long r = r0 + lane + 64 * k;
          if (f & 1) *(unsigned long long*)(c.p[f] + r * 8) = acc;
          else *(unsigned*)(c.p[f] + r * 4) = acc;
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void writerows(unsigned char* __restrict__ out, long nrows, int stride) {
  const long tiles = nrows / 64;
  const int tid = threadIdx.x;
  for (long t = blockIdx.x; t < tiles; t += gridDim.x) {
    unsigned char* d = out + t * 64 * stride;
    const int n16 = 64 * stride / 16;
    u32x4 x = {(unsigned)t, 1u, 2u, 3u};
    for (int c = tid; c < n16; c += 256) *(u32x4*)(d + c * 16) = x;
  }
}

template <typename F>
float time_ms(F f, int iters = 5) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  f();
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int i = 0; i < iters; ++i) {
    CHECK(hipEventRecord(a));
    f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  return best;
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : (64L << 20);
  int cus = 0;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  cus = prop.multiProcessorCount;
  // columns
  Cols c;
  std::vector<void*> bufs;
  size_t colbytes = 0;
  for (int f = 0; f < 104; ++f) {
    size_t b = n * ((f & 1) ? 8 : 4);
    void* p;
    CHECK(hipMalloc(&p, b));
    CHECK(hipMemset(p, f, b));
    c.p[f] = (const unsigned char*)p;
    bufs.push_back(p);
    colbytes += b;
  }
  unsigned* sink;
  CHECK(hipMalloc(&sink, 1 << 20));
  unsigned char* rows;
  const size_t rowbytes = (size_t)n * 848;
  CHECK(hipMalloc(&rows, rowbytes));
  // copy peak: rows -> columns area reused as a 40 GB buffer pair
  {
    size_t nb = 16L << 30;  // 16 GiB copy
    u32x4 *a, *b;
    CHECK(hipMalloc(&a, nb));
    CHECK(hipMalloc(&b, nb));
    CHECK(hipMemset(a, 1, nb));
    for (int g : {cus * 4, cus * 8, cus * 16}) {
      float ms = time_ms([&] { hipLaunchKernelGGL(copy16, dim3(g), dim3(256), 0, 0, a, b, nb / 16); });
      printf("{\"test\":\"copy16\",\"grid\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", g, ms, 2.0 * nb / ms / 1e6);
      ms = time_ms([&] { hipLaunchKernelGGL(copy16x4, dim3(g), dim3(256), 0, 0, a, b, nb / 16); });
      printf("{\"test\":\"copy16x4\",\"grid\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", g, ms, 2.0 * nb / ms / 1e6);
    }
    CHECK(hipFree(a));
    CHECK(hipFree(b));
  }
  for (int wpc : {2, 4, 8}) {
    const int g = cus * wpc;
    float ms;
    ms = time_ms([&] { hipLaunchKernelGGL((dec_traffic<64, 0>), dim3(g), dim3(256), 0, 0, c, n, rows); });
    printf("{\"test\":\"dec_traffic R64 lane=row\",\"wg_per_cu\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", wpc, ms, (colbytes + rowbytes) / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((dec_traffic<64, 16>), dim3(g), dim3(256), 0, 0, c, n, rows); });
    printf("{\"test\":\"dec_traffic R64 16B\",\"wg_per_cu\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", wpc, ms, (colbytes + rowbytes) / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((dec_traffic<128, 16>), dim3(g), dim3(256), 0, 0, c, n, rows); });
    printf("{\"test\":\"dec_traffic R128 16B\",\"wg_per_cu\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", wpc, ms, (colbytes + rowbytes) / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((dec_traffic<128, 0>), dim3(g), dim3(256), 0, 0, c, n, rows); });
    printf("{\"test\":\"dec_traffic R128 lane=row\",\"wg_per_cu\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", wpc, ms, (colbytes + rowbytes) / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((enc_traffic<64>), dim3(g), dim3(256), 0, 0, c, n, rows); });
    printf("{\"test\":\"enc_traffic R64\",\"wg_per_cu\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", wpc, ms, (colbytes + rowbytes) / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((enc_traffic<128>), dim3(g), dim3(256), 0, 0, c, n, rows); });
    printf("{\"test\":\"enc_traffic R128\",\"wg_per_cu\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", wpc, ms, (colbytes + rowbytes) / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((readcols<64, 4>), dim3(g), dim3(256), 0, 0, c, n, sink); });
    printf("{\"test\":\"readcols R64 lane=row\",\"wg_per_cu\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", wpc, ms, colbytes / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((readcols<128, 4>), dim3(g), dim3(256), 0, 0, c, n, sink); });
    printf("{\"test\":\"readcols R128 lane=row\",\"wg_per_cu\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", wpc, ms, colbytes / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((readcols<256, 4>), dim3(g), dim3(256), 0, 0, c, n, sink); });
    printf("{\"test\":\"readcols R256 lane=row\",\"wg_per_cu\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", wpc, ms, colbytes / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((readcols<128, 16>), dim3(g), dim3(256), 0, 0, c, n, sink); });
    printf("{\"test\":\"readcols R128 16B/lane\",\"wg_per_cu\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", wpc, ms, colbytes / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL(writerows, dim3(g), dim3(256), 0, 0, rows, n, 848); });
    printf("{\"test\":\"writerows\",\"wg_per_cu\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", wpc, ms, rowbytes / ms / 1e6);
  }
  return 0;
}
