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

// Batched scans (blockIdx.y = segment): data and partials of segment y start at
// y * dstride elements / y * pstride words (0 / 0: one scan).
template <int MODE>
__global__ __launch_bounds__(kWG) void scan_reduce_kernel(void* data, int64_t n, int64_t* partials, int64_t dstride = 0,
                                                          int64_t pstride = 0) {
  __shared__ int64_t smem[kWaves];
  if (MODE == 0) data = reinterpret_cast<int64_t*>(data) + blockIdx.y * dstride;
  partials += blockIdx.y * pstride;
  const int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x;  // lanes in element order: a sum needs no runs
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k * kWG < n) s += scan_load<MODE>(data, base + k * kWG);
  int64_t tot;
  block_excl_scan(s, smem, &tot);
  if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

// A tile's elements through LDS: read and written by lanes in element order (coalesced),
// scanned by threads as runs of kScanItems consecutive elements (a padded run per thread:
// no bank is hit by every lane).
constexpr int kRunPad = kScanItems + 1;
__device__ __forceinline__ int tile_pos(int e) { return (e / kScanItems) * kRunPad + e % kScanItems; }

// Inclusive (INCL) or exclusive prefix + base of each element of the tile at `base`
// (n elements from 0), in place in the LDS tile; returns nothing, the tile holds them.
template <int MODE>
__device__ __forceinline__ void tile_scan(void* data, int64_t base, int64_t n, int64_t add, int64_t* tile,
                                          int64_t* smem) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int e = k * kWG + tid;
    tile[tile_pos(e)] = base + e < n ? scan_load<MODE>(data, base + e) : 0;
  }
  __syncthreads();
  int64_t v[kScanItems];
  int64_t x = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    v[k] = tile[tid * kRunPad + k];
    x += v[k];
  }
  int64_t tot;
  int64_t pre = block_excl_scan(x, smem, &tot) + add;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    if (MODE == 1) pre += v[k];  // Arrow offsets: inclusive
    tile[tid * kRunPad + k] = pre;
    if (MODE == 0) pre += v[k];
  }
  __syncthreads();
}

// Single workgroup: exclusive scan of the partials in place (any count).
__device__ __forceinline__ void scan_partials_body(int64_t* partials, int64_t nb) {
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

__global__ __launch_bounds__(kWG) void scan_partials_kernel(int64_t* partials, int64_t nb, int64_t pstride = 0) {
  scan_partials_body(partials + blockIdx.y * pstride, nb);
}

// SEG (MODE 1): a segment of a longer offsets array: data[0] already holds the
// previous segment's last offset (the carry; 0 for the first) and is left as is.
template <int MODE, bool SEG = false>
__global__ __launch_bounds__(kWG) void scan_down_kernel(void* data, int64_t n, const int64_t* partials,
                                                        int32_t* status, int64_t dstride = 0, int64_t pstride = 0) {
  __shared__ int64_t smem[kWaves];
  __shared__ int64_t tile[kWG * kRunPad];
  if (MODE == 0) data = reinterpret_cast<int64_t*>(data) + blockIdx.y * dstride;
  partials += blockIdx.y * pstride;
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  int64_t add = partials[blockIdx.x];
  if (SEG) add += reinterpret_cast<const int32_t*>(data)[0];
  tile_scan<MODE>(data, base, n, add, tile, smem);
  bool over = false;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int e = k * kWG + threadIdx.x;
    if (base + e >= n) continue;
    const int64_t pre = tile[tile_pos(e)];
    if (MODE == 0) {
      reinterpret_cast<int64_t*>(data)[base + e] = pre;
    } else {
      over = over || pre > 0x7fffffffLL;
      reinterpret_cast<int32_t*>(data)[base + e + 1] = (int32_t)pre;
    }
  }
  if (over) set_status(status, FORY_ERR_CAPACITY);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (MODE == 0) reinterpret_cast<int64_t*>(data)[n] = partials[gridDim.x];
    else if (!SEG) reinterpret_cast<int32_t*>(data)[0] = 0;
  }
}

// Batched Arrow offsets scans (blockIdx.y = column): each column's lengths at
// offs[1..n] scanned inclusive in place, offs[0] = 0; partials at seg.pofs.
__global__ __launch_bounds__(kWG) void scan_reduce_batch_kernel(OffsScanBatch B, int64_t* partials) {
  __shared__ int64_t smem[kWaves];
  const OffsScanSeg g = B.seg[blockIdx.y];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x;
  if ((int64_t)blockIdx.x * kScanTile >= g.n) return;  // (uniform per workgroup)
  int64_t x = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k * kWG < g.n) x += g.offs[base + k * kWG + 1];
  int64_t tot;
  block_excl_scan(x, smem, &tot);
  if (threadIdx.x == 0) partials[g.pofs + blockIdx.x] = tot;
}

__global__ __launch_bounds__(kWG) void scan_partials_batch_kernel(OffsScanBatch B, int64_t* partials) {
  const OffsScanSeg g = B.seg[blockIdx.y];
  scan_partials_body(partials + g.pofs, (g.n + kScanTile - 1) / kScanTile);
}

__global__ __launch_bounds__(kWG) void scan_down_batch_kernel(OffsScanBatch B, const int64_t* partials,
                                                              int32_t* status) {
  __shared__ int64_t smem[kWaves];
  __shared__ int64_t tile[kWG * kRunPad];
  const OffsScanSeg g = B.seg[blockIdx.y];
  if ((int64_t)blockIdx.x * kScanTile >= g.n) return;
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  tile_scan<1>(g.offs, base, g.n, partials[g.pofs + blockIdx.x], tile, smem);
  bool over = false;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int e = k * kWG + threadIdx.x;
    if (base + e >= g.n) continue;
    const int64_t pre = tile[tile_pos(e)];
    over = over || pre > 0x7fffffffLL;
    g.offs[base + e + 1] = (int32_t)pre;
  }
  if (over) set_status(status, FORY_ERR_CAPACITY);
  if (blockIdx.x == 0 && threadIdx.x == 0) g.offs[0] = 0;
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

// `count` exclusive int64 scans at once: segment y = data[y * stride .. + n) (data[y * stride
// + n] = its total), partials: count * (scan_partials(n) + 1) words.
hipError_t launch_scan_i64_multi(int64_t* data, int64_t n, int64_t stride, int count, int64_t* partials,
                                 hipStream_t s) {
  if (count <= 0) return hipSuccess;
  const int64_t nb = (n + kScanTile - 1) / kScanTile;
  const int64_t ps = nb + 2;
  if (n <= 0) {
    for (int y = 0; y < count; ++y) (void)hipMemsetAsync(data + y * stride, 0, sizeof(int64_t), s);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(scan_reduce_kernel<0>, dim3((unsigned)nb, (unsigned)count), dim3(kWG), 0, s, (void*)data, n,
                     partials, stride, ps);
  hipLaunchKernelGGL(scan_partials_kernel, dim3(1, (unsigned)count), dim3(kWG), 0, s, partials, nb, ps);
  hipLaunchKernelGGL(scan_down_kernel<0>, dim3((unsigned)nb, (unsigned)count), dim3(kWG), 0, s, (void*)data, n,
                     (const int64_t*)partials, (int32_t*)nullptr, stride, ps);
  return hipGetLastError();
}

int64_t scan_batch_partials(int64_t n) { return (n + kScanTile - 1) / kScanTile + 2; }

// Scans `count` Arrow offsets columns (cols[i] with lengths at [1..n[i]]) in three launches
// per kMaxScanSeg columns; partials: the sum of scan_batch_partials(n[i]) words.
hipError_t launch_scan_offsets_batch(int32_t* const* cols, const int64_t* n, int count, int64_t* partials,
                                     int32_t* status, hipStream_t s) {
  for (int c0 = 0; c0 < count; c0 += kMaxScanSeg) {
    OffsScanBatch B{};
    int64_t pofs = 0, maxnb = 0;
    B.count = count - c0 < kMaxScanSeg ? count - c0 : kMaxScanSeg;
    for (int y = 0; y < B.count; ++y) {
      B.seg[y] = OffsScanSeg{cols[c0 + y], n[c0 + y], pofs};
      pofs += scan_batch_partials(n[c0 + y]);
      const int64_t nb = (n[c0 + y] + kScanTile - 1) / kScanTile;
      maxnb = nb > maxnb ? nb : maxnb;
      if (n[c0 + y] <= 0) (void)hipMemsetAsync(cols[c0 + y], 0, sizeof(int32_t), s);
    }
    if (maxnb == 0) continue;
    hipLaunchKernelGGL(scan_reduce_batch_kernel, dim3((unsigned)maxnb, (unsigned)B.count), dim3(kWG), 0, s, B, partials);
    hipLaunchKernelGGL(scan_partials_batch_kernel, dim3(1, (unsigned)B.count), dim3(kWG), 0, s, B, partials);
    hipLaunchKernelGGL(scan_down_batch_kernel, dim3((unsigned)maxnb, (unsigned)B.count), dim3(kWG), 0, s, B,
                       (const int64_t*)partials, status);
    partials += pofs;
  }
  return hipGetLastError();
}

int64_t scan_multi_partials(int64_t n, int count) { return (int64_t)count * ((n + kScanTile - 1) / kScanTile + 2); }

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
