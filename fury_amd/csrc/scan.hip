// scan.hip — device-wide scans (row offsets, Arrow offsets) and fixed-stride
// row offsets, shared by the varlen encode/decode and the frame index.
#include "kcommon.h"

namespace fory_amd {

namespace {

__global__ void fill_offsets_kernel(int64_t* offs, int64_t n, int64_t stride) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= n) offs[i] = i * stride;
}

// ---------------------------------------------------------------------------
// Device-wide scan (3 kernels): block reduce, scan of partials, downsweep.
// ---------------------------------------------------------------------------
constexpr int kScanItems = 16;
constexpr int kScanTile = kWG * kScanItems;  // 4096 items per block

__device__ __forceinline__ int64_t wave_incl_scan(int64_t x, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// Returns the exclusive prefix of `x` over the workgroup; *total = sum.
__device__ __forceinline__ int64_t block_excl_scan(int64_t x, int64_t* smem, int64_t* total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t inc = wave_incl_scan(x, lane);
  if (lane == 63) smem[w] = inc;
  __syncthreads();
  int64_t wpre = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kWaves; ++k) {
    const int64_t s = smem[k];
    if (k < w) wpre += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return wpre + inc - x;
}

// MODE 0: int64 data, exclusive, data[n] = total.
// MODE 1: int32 Arrow offsets: lengths at offs[1..n], inclusive into offs[1..n].
template <int MODE>
__device__ __forceinline__ int64_t scan_load(void* data, int64_t i) {
  if (MODE == 0) return reinterpret_cast<const int64_t*>(data)[i];
  return reinterpret_cast<const int32_t*>(data)[i + 1];
}

template <int MODE>
__global__ __launch_bounds__(kWG) void scan_reduce_kernel(void* data, int64_t n, int64_t* partials) {
  __shared__ int64_t smem[kWaves];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k < n) s += scan_load<MODE>(data, base + k);
  int64_t tot;
  block_excl_scan(s, smem, &tot);
  if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

// Single workgroup: exclusive scan of the partials in place (any count).
__global__ __launch_bounds__(kWG) void scan_partials_kernel(int64_t* partials, int64_t nb) {
  __shared__ int64_t smem[kWaves];
  int64_t carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += kScanTile) {
    const int64_t base = b0 + (int64_t)threadIdx.x * kScanItems;
    int64_t v[kScanItems];
    int64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
      v[k] = base + k < nb ? partials[base + k] : 0;
      s += v[k];
    }
    int64_t tot;
    int64_t pre = block_excl_scan(s, smem, &tot) + carry;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
      if (base + k < nb) partials[base + k] = pre;
      pre += v[k];
    }
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) partials[nb] = carry;
}

// SEG (MODE 1): a segment of a longer offsets array: data[0] already holds the
// previous segment's last offset (the carry; 0 for the first) and is left as is.
template <int MODE, bool SEG = false>
__global__ __launch_bounds__(kWG) void scan_down_kernel(void* data, int64_t n, const int64_t* partials,
                                                        int32_t* status) {
  __shared__ int64_t smem[kWaves];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int64_t v[kScanItems];
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    v[k] = base + k < n ? scan_load<MODE>(data, base + k) : 0;
    s += v[k];
  }
  int64_t tot;
  int64_t pre = block_excl_scan(s, smem, &tot) + partials[blockIdx.x];
  if (SEG) pre += reinterpret_cast<const int32_t*>(data)[0];
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    if (base + k < n) {
      if (MODE == 0) {
        reinterpret_cast<int64_t*>(data)[base + k] = pre;
        pre += v[k];
      } else {
        pre += v[k];
        if (pre > 0x7fffffffLL) set_status(status, FORY_ERR_CAPACITY);
        reinterpret_cast<int32_t*>(data)[base + k + 1] = (int32_t)pre;
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (MODE == 0) reinterpret_cast<int64_t*>(data)[n] = partials[gridDim.x];
    else if (!SEG) reinterpret_cast<int32_t*>(data)[0] = 0;
  }
}

// Host decode pipeline (host.cpp): a chunk's Arrow offsets (0-based) moved to their
// place in the batch, and its validity bits (from bit 0) moved to bit `shift` of
// their first byte (the chunk's first element is not on a byte boundary there).
__global__ void offsets_add_kernel(int32_t* offs, int64_t n, int32_t base) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= n) offs[i] += base;
}

__global__ void bits_shift_kernel(const uint8_t* __restrict__ src, int64_t nbits, uint8_t* __restrict__ dst,
                                  int shift) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= (shift + nbits + 7) >> 3) return;
  uint32_t out = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int64_t t = 8 * j + q - shift;
    if (t >= 0 && t < nbits) out |= ((uint32_t)(src[t >> 3] >> (t & 7)) & 1u) << q;
  }
  dst[j] = (uint8_t)out;
}

}  // namespace

hipError_t launch_offsets_add(int32_t* offs, int64_t n, int32_t base, hipStream_t s) {
  if (base == 0) return hipSuccess;
  const int64_t blocks = (n + 1 + kWG - 1) / kWG;
  hipLaunchKernelGGL(offsets_add_kernel, dim3((unsigned)blocks), dim3(kWG), 0, s, offs, n, base);
  return hipGetLastError();
}

hipError_t launch_bits_shift(const uint8_t* src, int64_t nbits, uint8_t* dst, int shift, hipStream_t s) {
  const int64_t bytes = (shift + nbits + 7) >> 3;
  if (bytes <= 0) return hipSuccess;
  hipLaunchKernelGGL(bits_shift_kernel, dim3((unsigned)((bytes + kWG - 1) / kWG)), dim3(kWG), 0, s, src, nbits, dst,
                     shift);
  return hipGetLastError();
}

hipError_t launch_fill_offsets(int64_t* offs, int64_t n, int64_t stride, hipStream_t s) {
  const int64_t blocks = (n + 1 + kWG - 1) / kWG;
  hipLaunchKernelGGL(fill_offsets_kernel, dim3((unsigned)blocks), dim3(kWG), 0, s, offs, n, stride);
  return hipGetLastError();
}

int64_t scan_partials(int64_t n) { return (n + kScanTile - 1) / kScanTile + 1; }

hipError_t launch_scan_i64(int64_t* data, int64_t n, int64_t* partials, hipStream_t s) {
  const int64_t nb = (n + kScanTile - 1) / kScanTile;
  if (n <= 0) {
    (void)hipMemsetAsync(data, 0, sizeof(int64_t), s);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(scan_reduce_kernel<0>, dim3((unsigned)nb), dim3(kWG), 0, s, (void*)data, n, partials);
  hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(kWG), 0, s, partials, nb);
  hipLaunchKernelGGL(scan_down_kernel<0>, dim3((unsigned)nb), dim3(kWG), 0, s, (void*)data, n,
                     (const int64_t*)partials, (int32_t*)nullptr);
  return hipGetLastError();
}

hipError_t launch_scan_offsets_i32(int32_t* offs, int64_t n, int64_t* partials, int32_t* status,
                                   hipStream_t s) {
  const int64_t nb = (n + kScanTile - 1) / kScanTile;
  if (n <= 0) {
    (void)hipMemsetAsync(offs, 0, sizeof(int32_t), s);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(scan_reduce_kernel<1>, dim3((unsigned)nb), dim3(kWG), 0, s, (void*)offs, n, partials);
  hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(kWG), 0, s, partials, nb);
  hipLaunchKernelGGL(scan_down_kernel<1>, dim3((unsigned)nb), dim3(kWG), 0, s, (void*)offs, n,
                     (const int64_t*)partials, status);
  return hipGetLastError();
}

hipError_t launch_scan_offsets_i32_segmented(int32_t* offs, int64_t n, int64_t* partials, int64_t partial_words,
                                             int32_t* status, hipStream_t s) {
  (void)hipMemsetAsync(offs, 0, sizeof(int32_t), s);
  const int64_t seg = kScanTile * (partial_words - 1);
  if (n <= 0) return hipGetLastError();
  if (seg <= 0) return hipErrorInvalidValue;
  for (int64_t a = 0; a < n; a += seg) {
    const int64_t m = n - a < seg ? n - a : seg;
    const int64_t nb = (m + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(scan_reduce_kernel<1>, dim3((unsigned)nb), dim3(kWG), 0, s, (void*)(offs + a), m, partials);
    hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(kWG), 0, s, partials, nb);
    hipLaunchKernelGGL((scan_down_kernel<1, true>), dim3((unsigned)nb), dim3(kWG), 0, s, (void*)(offs + a), m,
                       (const int64_t*)partials, status);
  }
  return hipGetLastError();
}

}  // namespace fory_amd
