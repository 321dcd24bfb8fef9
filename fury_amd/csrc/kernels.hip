// kernels.hip — gfx950 (CDNA4) kernels for Fory's row format.
//
// Byte layout restated from the Java writer (the spec doc is empty,
// docs/specification/row_format_spec.md:22-24). F = java/fory-format/src/
// main/java/org/apache/fory/format:
//   row   = [null bitmap ((n+63)/64)*8 B, bit i = byte i>>3 bit i&7, 1 = null]
//           [n x 8-B slots][variable section]      F/row/binary/writer/BinaryRowWriter.java:46-124
//   fixed = value in the slot's low bytes, zero-extended            BinaryRowWriter.java:92-124
//   var   = slot (relOffset<<32 | size), data appended in ordinal
//           order, zero-padded to 8                                F/.../writer/BinaryWriter.java:106-194
//   array = [i64 n][bitmap][n x elemSize padded to 8]              F/.../writer/BinaryArrayWriter.java:93-118
//   frame = [i32 8+rowSize][i64 schemaHash][row]                   F/encoder/Encoders.java:213-225
//
// Fixed-width schemas (every top-level field 1/2/4/8 bytes) take the tiled
// path: one workgroup per tile of TR records, one lane per record. Columns
// are read with coalesced per-lane loads (lane = record, consecutive
// addresses), scattered into an LDS image of the tile's rows, and the whole
// tile (TR * stride contiguous bytes) leaves with 16-B stores. Decode is the
// inverse: the tile image comes in through LDS-DMA (global_load_lds_dwordx4),
// each lane reads its record's slots from LDS and stores coalesced columns.
// No MFMA: this is byte shuffling bound by HBM.
//
// Varlen / nested schemas run a per-record op program (plan.cpp) in one lane
// per record, with a device-wide scan for row offsets.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace fory_amd {

namespace {

constexpr int kWG = 256;         // 4 waves
constexpr int kWaves = kWG / 64;

__device__ __forceinline__ void st32(uint8_t* p, uint32_t v) { *reinterpret_cast<uint32_t*>(p) = v; }
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }

// Loads the `width` low bytes of element `i` (little-endian, zero-extended).
__device__ __forceinline__ uint64_t load_elem(const uint8_t* __restrict__ base, int width, int64_t i) {
  switch (width) {
    case 8: return *reinterpret_cast<const uint64_t*>(base + i * 8);
    case 4: return *reinterpret_cast<const uint32_t*>(base + i * 4);
    case 2: return *reinterpret_cast<const uint16_t*>(base + i * 2);
    default: return base[i];
  }
}

__device__ __forceinline__ void store_elem(uint8_t* __restrict__ base, int width, int64_t i, uint64_t v) {
  switch (width) {
    case 8: *reinterpret_cast<uint64_t*>(base + i * 8) = v; break;
    case 4: *reinterpret_cast<uint32_t*>(base + i * 4) = (uint32_t)v; break;
    case 2: *reinterpret_cast<uint16_t*>(base + i * 2) = (uint16_t)v; break;
    default: base[i] = (uint8_t)v; break;
  }
}

__device__ __forceinline__ void set_status(int32_t* status, int32_t code) {
  if (status) atomicCAS(status, 0, code);
}

// ---------------------------------------------------------------------------
// Fixed-width encode: columns -> rows (tiled through LDS)
// ---------------------------------------------------------------------------
// TR = records per tile (64 -> one field per wave-instruction; 32/16/8 for
// wide rows -> 64/TR fields per wave-instruction). U = fields each lane keeps
// in flight before writing LDS (memory-level parallelism).
template <int TR, bool FRAME>
__global__ __launch_bounds__(kWG) void encode_fixed_kernel(FixedLaunch L, uint8_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int FPW = 64 / TR;       // fields per wave-instruction
  constexpr int FSTEP = kWaves * FPW;
  constexpr int U = 16;
  constexpr int HDR = FRAME ? 12 : 0;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane % TR;
  const int fsub = lane / TR;
  const int64_t r0 = (int64_t)blockIdx.x * TR;
  const int64_t left = L.num_rows - r0;
  const int rows = left < TR ? (int)left : TR;
  const int stride = L.stride;
  const int nf = L.num_fields;
  const int bm = L.bitmap_bytes;
  uint8_t* row = lds + r * stride;
  const int64_t grow = r0 + r;
  const bool live = r < rows;

  // Phase 0: frame header + zeroed null bitmap, one writer per record.
  if (wave == 0 && fsub == 0) {
    if (FRAME) {
      st32(row, (uint32_t)(8 + L.fixed_size));
      st32(row + 4, (uint32_t)(uint64_t)L.schema_hash);
      st32(row + 8, (uint32_t)((uint64_t)L.schema_hash >> 32));
    }
    for (int b = 0; b < bm; b += 4) st32(row + HDR + b, 0u);
  }
  if (L.any_nullable) __syncthreads();  // null bits are OR-ed into the bitmap below

  // Phase 1: column loads (coalesced: lane = record) -> LDS slots.
  for (int fb = wave * FPW; fb < nf; fb += FSTEP * U) {
    uint64_t v[U];
    bool isnull[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int f = fb + u * FSTEP + fsub;
      v[u] = 0;
      isnull[u] = false;
      if (f < nf && live) {
        const FixedFieldDev fd = L.fields[f];
        v[u] = load_elem(fd.values, fd.width, grow);
        if ((fd.flags & 1) && fd.validity)
          isnull[u] = !((fd.validity[grow >> 3] >> (grow & 7)) & 1);
        if (fd.flags & 2) v[u] = v[u] ? 1 : 0;  // MemoryBuffer.putBoolean
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int f = fb + u * FSTEP + fsub;
      if (f < nf) {
        uint64_t x = v[u];
        if (isnull[u]) {  // BinaryWriter.setNullAt: bit set, slot left zero
          x = 0;
          atomicOr(reinterpret_cast<uint32_t*>(row + HDR + ((f >> 5) << 2)), 1u << (f & 31));
        }
        uint8_t* slot = row + HDR + bm + 8 * f;
        if (FRAME) {  // 4-byte aligned only (frame = 12-byte header)
          st32(slot, (uint32_t)x);
          st32(slot + 4, (uint32_t)(x >> 32));
        } else {
          *reinterpret_cast<uint64_t*>(slot) = x;
        }
      }
    }
  }
  __syncthreads();

  // Phase 2: the tile's rows are TR*stride contiguous bytes -> 16-B stores.
  const int64_t bytes = (int64_t)rows * stride;
  uint8_t* dst = out + r0 * stride;
  const int n16 = (int)(bytes >> 4);
  for (int c = tid; c < n16; c += kWG) {
    const uint4 x = *reinterpret_cast<const uint4*>(lds + c * 16);
    *reinterpret_cast<uint4*>(dst + c * 16) = x;
  }
  const int tail4 = (int)(bytes & 15) >> 2;
  if (tid < tail4) st32(dst + n16 * 16 + tid * 4, ld32(lds + n16 * 16 + tid * 4));
}

// ---------------------------------------------------------------------------
// Fixed-width decode: rows -> columns
// ---------------------------------------------------------------------------
template <int TR, bool FRAME>
__global__ __launch_bounds__(kWG) void decode_fixed_kernel(FixedLaunch L, const uint8_t* __restrict__ in,
                                                           int32_t* status) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int FPW = 64 / TR;
  constexpr int FSTEP = kWaves * FPW;
  constexpr int HDR = FRAME ? 12 : 0;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane % TR;
  const int fsub = lane / TR;
  const int64_t r0 = (int64_t)blockIdx.x * TR;
  const int64_t left = L.num_rows - r0;
  const int rows = left < TR ? (int)left : TR;
  const int stride = L.stride;
  const int nf = L.num_fields;
  const int bm = L.bitmap_bytes;

  // Phase 1: tile image HBM -> LDS by LDS-DMA (1 KiB per wave-instruction,
  // lane-linear destination = the contiguous tile image).
  const int64_t bytes = (int64_t)rows * stride;
  const uint8_t* src = in + r0 * stride;
  const int n16 = (int)(bytes >> 4);
  const int nfull = n16 & ~(kWG - 1);
  for (int c0 = 0; c0 < nfull; c0 += kWG) {
    const int c = c0 + tid;
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(src + (int64_t)c * 16),
        (__attribute__((address_space(3))) void*)(lds + (c0 + wave * 64) * 16), 16, 0, 0);
  }
  for (int c = nfull + tid; c < n16; c += kWG)
    *reinterpret_cast<uint4*>(lds + c * 16) = *reinterpret_cast<const uint4*>(src + (int64_t)c * 16);
  const int tail4 = (int)(bytes & 15) >> 2;
  if (tid < tail4) st32(lds + n16 * 16 + tid * 4, ld32(src + n16 * 16 + tid * 4));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const uint8_t* row = lds + r * stride;
  const int64_t grow = r0 + r;
  const bool live = r < rows;

  if (FRAME && wave == 0 && fsub == 0 && live) {
    // Encoders.decode (Encoders.java:177-190): size, then schema hash check.
    const uint32_t len = ld32(row);
    const uint64_t h = (uint64_t)ld32(row + 4) | ((uint64_t)ld32(row + 8) << 32);
    if (h != (uint64_t)L.schema_hash) set_status(status, FORY_ERR_SCHEMA_MISMATCH);
    else if (len != (uint32_t)(8 + L.fixed_size)) set_status(status, FORY_ERR_CORRUPT);
  }

  // Phase 2: per field, lane = record: slot from LDS -> coalesced column store.
  for (int fb = wave * FPW; fb < nf; fb += FSTEP) {
    const int f = fb + fsub;
    if (f >= nf) continue;
    const FixedFieldDev fd = L.fields[f];
    const uint32_t bw = ld32(row + HDR + ((f >> 5) << 2));
    const bool isnull = (bw >> (f & 31)) & 1;  // BinaryRow.isNullAt
    const uint8_t* slot = row + HDR + bm + 8 * f;
    uint64_t x;
    if (FRAME || fd.width < 8) {
      x = ld32(slot);
      if (fd.width == 8) x |= (uint64_t)ld32(slot + 4) << 32;
    } else {
      x = *reinterpret_cast<const uint64_t*>(slot);
    }
    if (isnull) x = 0;                         // Java default for a null field
    if (fd.flags & 2) x = (x & 0xff) ? 1 : 0;  // getBoolean: byte != 0
    if (live) store_elem(fd.out_values, fd.width, grow, x);
    if ((fd.flags & 1) && fd.out_validity) {
      const uint64_t m = __ballot(!isnull && live);
      if (r == 0) {
        const uint64_t mine = (m >> (fsub * TR)) & (TR == 64 ? ~0ull : ((1ull << TR) - 1));
        uint8_t* vb = fd.out_validity + (r0 >> 3);
        const int nb = (rows + 7) >> 3;
        for (int b = 0; b < nb; ++b) vb[b] = (uint8_t)(mine >> (8 * b));
      }
    }
  }
}

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

template <int MODE>
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
    else reinterpret_cast<int32_t*>(data)[0] = 0;
  }
}

// ---------------------------------------------------------------------------
// Varlen / nested: per-record op program, one lane per record.
// ---------------------------------------------------------------------------
constexpr int kMaxDepth = 8;

__device__ __forceinline__ int64_t round8(int64_t n) { return (n + 7) & ~int64_t(7); }
__device__ __forceinline__ int32_t bitmap_bytes(int64_t n) { return (int32_t)(((n + 63) >> 6) << 3); }

__device__ __forceinline__ bool col_valid(const ColumnDev& c, int64_t i) {
  return !c.validity || ((c.validity[i >> 3] >> (i & 7)) & 1);
}

// Global stores that may be only 4-byte aligned (frame mode).
__device__ __forceinline__ void gst64(uint8_t* p, uint64_t v) {
  if ((reinterpret_cast<uintptr_t>(p) & 7) == 0) {
    *reinterpret_cast<uint64_t*>(p) = v;
  } else {
    st32(p, (uint32_t)v);
    st32(p + 4, (uint32_t)(v >> 32));
  }
}
__device__ __forceinline__ uint64_t gld64(const uint8_t* p) {
  if ((reinterpret_cast<uintptr_t>(p) & 7) == 0) return *reinterpret_cast<const uint64_t*>(p);
  return (uint64_t)ld32(p) | ((uint64_t)ld32(p + 4) << 32);
}

__device__ __forceinline__ void set_null_bit(uint8_t* bitmap, int32_t ordinal) {
  bitmap[ordinal >> 3] |= (uint8_t)(1u << (ordinal & 7));  // BitUtils.set
}

// Copies n bytes (any alignment) and zero-pads to round8(n) (BinaryWriter.writeUnaligned).
__device__ __forceinline__ void copy_padded(uint8_t* dst, const uint8_t* src, int64_t n) {
  int64_t k = 0;
  for (; k < n; ++k) dst[k] = src[k];
  const int64_t e = round8(n);
  for (; k < e; ++k) dst[k] = 0;
}

// Row/frame size of record i (BinaryRowWriter.reset + all appends).
__global__ __launch_bounds__(kWG) void var_sizes_kernel(VarLaunch L, int64_t* sizes) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i >= L.num_rows) return;
  int64_t size = L.fixed_size + (L.frame ? 12 : 0);
  int absent_depth = 0;  // >0: inside a null struct
  for (int pc = 0; pc < L.num_ops; ++pc) {
    const Op op = L.prog[pc];
    const ColumnDev& c = L.cols[op.b];
    switch (op.code) {
      case OP_FIXED:
        break;
      case OP_BYTES:
        if (!absent_depth && (!(op.d & 1) || col_valid(c, i))) size += round8((int64_t)c.offsets[i + 1] - c.offsets[i]);
        break;
      case OP_STRUCT_BEGIN:
        if (absent_depth || ((op.d & 1) && !col_valid(c, i))) absent_depth++;
        else size += bitmap_bytes(op.c) + 8LL * op.c;
        break;
      case OP_STRUCT_END:
        if (absent_depth) absent_depth--;
        break;
      case OP_LIST:
        if (!absent_depth && (!(op.d & 1) || col_valid(c, i))) {
          const int64_t n = (int64_t)c.offsets[i + 1] - c.offsets[i];
          const int w = op.e & 0xff;
          size += 8 + bitmap_bytes(n) + round8(n * w);
        }
        break;
    }
  }
  sizes[i] = size;
}

__global__ __launch_bounds__(kWG) void var_encode_kernel(VarLaunch L, const int64_t* __restrict__ offs,
                                                         uint8_t* __restrict__ out, int64_t capacity,
                                                         int32_t* status) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i >= L.num_rows) return;
  const int64_t beg = offs[i], end = offs[i + 1];
  if (end > capacity || beg < 0 || end < beg) {
    set_status(status, FORY_ERR_CAPACITY);
    return;
  }
  uint8_t* base = out + beg;
  uint8_t* row = base;
  if (L.frame) {  // Encoders.encode(MemoryBuffer,T): [i32 8+rowSize][i64 hash]
    st32(base, (uint32_t)(end - beg - 4));
    gst64(base + 4, (uint64_t)L.schema_hash);
    row = base + 12;
  }
  // writer stack: start (relative to row), header bytes, ordinal in parent
  int32_t st_start[kMaxDepth], st_hdr[kMaxDepth], st_ord[kMaxDepth];
  int depth = 0;
  st_start[0] = 0;
  st_hdr[0] = L.bitmap_bytes;
  st_ord[0] = 0;
  int absent = 0;
  int64_t wi = L.fixed_size;  // writerIndex relative to row (BinaryRowWriter.reset)
  for (int b = 0; b < L.bitmap_bytes; b += 8) gst64(row + b, 0);
  for (int pc = 0; pc < L.num_ops; ++pc) {
    const Op op = L.prog[pc];
    const ColumnDev& c = L.cols[op.b];
    if (absent) {
      if (op.code == OP_STRUCT_BEGIN) absent++;
      else if (op.code == OP_STRUCT_END) absent--;
      continue;
    }
    uint8_t* slot = row + st_start[depth] + st_hdr[depth] + 8 * op.a;
    uint8_t* bitmap = row + st_start[depth];
    const bool isnull = (op.d & 1) && !col_valid(c, i);
    switch (op.code) {
      case OP_FIXED: {
        uint64_t v = 0;
        if (isnull) set_null_bit(bitmap, op.a);
        else v = load_elem(c.values, op.c, i);
        if (op.d & 2) v = v ? 1 : 0;
        gst64(slot, v);
        break;
      }
      case OP_BYTES: {
        if (isnull) {
          set_null_bit(bitmap, op.a);
          gst64(slot, 0);
          break;
        }
        const int64_t s0 = c.offsets[i], n = (int64_t)c.offsets[i + 1] - s0;
        copy_padded(row + wi, c.values + s0, n);
        gst64(slot, ((uint64_t)(wi - st_start[depth]) << 32) | (uint32_t)n);
        wi += round8(n);
        break;
      }
      case OP_STRUCT_BEGIN: {
        if (isnull) {
          set_null_bit(bitmap, op.a);
          gst64(slot, 0);
          absent = 1;
          break;
        }
        // serializeForBean (BaseBinaryEncoderBuilder.java:473-486): child row inline
        depth++;
        st_start[depth] = (int32_t)wi;
        st_hdr[depth] = bitmap_bytes(op.c);
        st_ord[depth] = op.a;
        for (int b = 0; b < st_hdr[depth]; b += 8) gst64(row + wi + b, 0);
        wi += st_hdr[depth] + 8LL * op.c;
        break;
      }
      case OP_STRUCT_END: {
        const int64_t size = wi - st_start[depth];
        const int32_t rel = st_start[depth] - st_start[depth - 1];
        const int32_t ord = st_ord[depth];
        depth--;
        gst64(row + st_start[depth] + st_hdr[depth] + 8 * ord, ((uint64_t)(uint32_t)rel << 32) | (uint32_t)size);
        break;
      }
      case OP_LIST: {
        if (isnull) {
          set_null_bit(bitmap, op.a);
          gst64(slot, 0);
          break;
        }
        // BinaryArrayWriter.reset(n) + per-element write (BinaryArrayWriter.java:93-158)
        const ColumnDev& it = L.cols[op.c];
        const int w = op.e & 0xff;
        const int iflags = op.e >> 8;
        const int64_t e0 = c.offsets[i], n = (int64_t)c.offsets[i + 1] - e0;
        const int64_t astart = wi;
        const int32_t ahdr = 8 + bitmap_bytes(n);
        uint8_t* arr = row + astart;
        gst64(arr, (uint64_t)n);
        for (int b = 8; b < ahdr; b += 8) gst64(arr + b, 0);
        uint8_t* data = arr + ahdr;
        for (int64_t j = 0; j < n; ++j) {
          const bool enull = (iflags & 1) && !col_valid(it, e0 + j);
          uint64_t v = 0;
          if (enull) arr[8 + (j >> 3)] |= (uint8_t)(1u << (j & 7));
          else v = load_elem(it.values, w, e0 + j);
          if (iflags & 2) v = v ? 1 : 0;
          switch (w) {
            case 8: gst64(data + 8 * j, v); break;
            case 4: st32(data + 4 * j, (uint32_t)v); break;
            case 2: data[2 * j] = (uint8_t)v; data[2 * j + 1] = (uint8_t)(v >> 8); break;
            default: data[j] = (uint8_t)v; break;
          }
        }
        const int64_t dsz = n * w, fixed_part = round8(dsz);
        for (int64_t k = dsz; k < fixed_part; ++k) data[k] = 0;
        wi += ahdr + fixed_part;
        gst64(slot, ((uint64_t)(astart - st_start[depth]) << 32) | (uint32_t)(wi - astart));
        break;
      }
    }
  }
}

// Decode, pass 1: lengths of every varlen column of record i into
// out_offsets[i+1] (bytes for STRING/BINARY, elements for LIST).
// Pass 2 (WRITE=true): values, validity, list items.
template <bool WRITE>
__global__ __launch_bounds__(kWG) void var_decode_kernel(VarLaunch L, const uint8_t* __restrict__ in,
                                                         const int64_t* __restrict__ offs, int32_t* status) {
  const int64_t i0 = (int64_t)blockIdx.x * kWG + threadIdx.x;
  const bool live = i0 < L.num_rows;
  const int64_t i = live ? i0 : 0;
  const uint8_t* base = in + offs[i];
  const uint8_t* row = base;
  int64_t row_len = offs[i + 1] - offs[i];
  bool bad = !live;
  if (live && L.frame) {
    const uint32_t len = ld32(base);
    const uint64_t h = gld64(base + 4);
    if (h != (uint64_t)L.schema_hash) { if (WRITE) set_status(status, FORY_ERR_SCHEMA_MISMATCH); bad = true; }
    else if ((int64_t)len + 4 != row_len || len < (uint32_t)(8 + L.fixed_size)) { if (WRITE) set_status(status, FORY_ERR_CORRUPT); bad = true; }
    row = base + 12;
    row_len -= 12;
  }
  int32_t st_start[kMaxDepth], st_hdr[kMaxDepth];
  int depth = 0;
  st_start[0] = 0;
  st_hdr[0] = L.bitmap_bytes;
  int absent = bad ? 1 << 20 : 0;  // >0: this record's subtree is null/absent
  for (int pc = 0; pc < L.num_ops; ++pc) {
    const Op op = L.prog[pc];
    const ColumnDev& c = L.cols[op.b];
    bool isnull = true;
    const uint8_t* slot = nullptr;
    if (!absent) {
      const uint8_t* bm = row + st_start[depth];
      isnull = (bm[op.a >> 3] >> (op.a & 7)) & 1;  // BinaryRow.isNullAt
      slot = row + st_start[depth] + st_hdr[depth] + 8 * op.a;
    }
    // Row-level validity of this column (rows of a wave are consecutive).
    if (WRITE && (op.d & 1) && c.out_validity && op.code != OP_STRUCT_END) {
      const uint64_t m = __ballot(live && !isnull);
      const int lane = threadIdx.x & 63;
      const int64_t w0 = i0 - lane;
      if (lane == 0 && w0 < L.num_rows) {
        const int64_t nrow = L.num_rows - w0 < 64 ? L.num_rows - w0 : 64;
        uint8_t* vb = c.out_validity + (w0 >> 3);
        for (int b = 0; b < (int)((nrow + 7) >> 3); ++b) vb[b] = (uint8_t)(m >> (8 * b));
      }
    }
    switch (op.code) {
      case OP_FIXED: {
        if (WRITE && live) {
          uint64_t v = isnull ? 0 : gld64(slot);
          if (op.d & 2) v = (v & 0xff) ? 1 : 0;
          store_elem(c.out_values, op.c, i, v);
        }
        break;
      }
      case OP_BYTES: {
        int64_t n = 0, rel = 0;
        if (!isnull) {
          const uint64_t os = gld64(slot);
          rel = (int32_t)(os >> 32);
          n = (int32_t)(uint32_t)os;
          if (n < 0 || rel < 0 || rel + n > row_len) { set_status(status, FORY_ERR_CORRUPT); n = 0; }
        }
        if (live) {
          if (!WRITE) c.out_offsets[i + 1] = (int32_t)n;
          else {
            uint8_t* dst = c.out_values + c.out_offsets[i];
            const uint8_t* s = row + st_start[depth] + rel;
            for (int64_t k = 0; k < n; ++k) dst[k] = s[k];
          }
        }
        break;
      }
      case OP_STRUCT_BEGIN: {
        if (absent || isnull) {
          absent++;
          break;
        }
        const uint64_t os = gld64(slot);
        const int64_t rel = (int32_t)(os >> 32);
        depth++;
        st_start[depth] = st_start[depth - 1] + (int32_t)rel;
        st_hdr[depth] = bitmap_bytes(op.c);
        break;
      }
      case OP_STRUCT_END:
        if (absent) absent--;
        else depth--;
        break;
      case OP_LIST: {
        int64_t n = 0, rel = 0;
        if (!isnull) {
          const uint64_t os = gld64(slot);
          rel = (int32_t)(os >> 32);
          n = (int64_t)gld64(row + st_start[depth] + rel);  // BinaryArray.pointTo
          n = (int32_t)n;
          if (n < 0 || rel + 8 > row_len) { set_status(status, FORY_ERR_CORRUPT); n = 0; }
        }
        if (live) {
          if (!WRITE) {
            c.out_offsets[i + 1] = (int32_t)n;
          } else if (n > 0) {
            const ColumnDev& it = L.cols[op.c];
            const int w = op.e & 0xff;
            const int iflags = op.e >> 8;
            const uint8_t* arr = row + st_start[depth] + rel;
            const int32_t ahdr = 8 + bitmap_bytes(n);
            const int64_t e0 = c.out_offsets[i];
            for (int64_t j = 0; j < n; ++j) {
              const bool en = (arr[8 + (j >> 3)] >> (j & 7)) & 1;  // BinaryArray.isNullAt
              uint64_t v = 0;
              if (!en) {
                const uint8_t* p = arr + ahdr + j * w;
                switch (w) {
                  case 8: v = gld64(p); break;
                  case 4: v = ld32(p); break;
                  case 2: v = (uint64_t)p[0] | ((uint64_t)p[1] << 8); break;
                  default: v = p[0]; break;
                }
              }
              if (iflags & 2) v = (v & 0xff) ? 1 : 0;
              store_elem(it.out_values, w, e0 + j, v);
              if ((iflags & 1) && it.out_validity) {
                const int64_t q = e0 + j;
                const uint32_t bit = 1u << (q & 31);
                uint32_t* word = reinterpret_cast<uint32_t*>(it.out_validity) + (q >> 5);
                if (en) atomicAnd(word, ~bit);
                else atomicOr(word, bit);
              }
            }
          }
        }
        break;
      }
    }
  }
}

template <int TR, bool FRAME>
hipError_t launch_encode_tr(const FixedLaunch& L, uint8_t* out, hipStream_t s) {
  const int64_t tiles = (L.num_rows + TR - 1) / TR;
  const size_t lds = (size_t)TR * L.stride;
  static bool init = false;  // raise the dynamic-LDS cap once (160 KiB per CU)
  if (!init) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&encode_fixed_kernel<TR, FRAME>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    init = true;
  }
  hipLaunchKernelGGL((encode_fixed_kernel<TR, FRAME>), dim3((unsigned)tiles), dim3(kWG), lds, s, L, out);
  return hipGetLastError();
}

template <int TR, bool FRAME>
hipError_t launch_decode_tr(const FixedLaunch& L, const uint8_t* in, int32_t* status, hipStream_t s) {
  const int64_t tiles = (L.num_rows + TR - 1) / TR;
  const size_t lds = (size_t)TR * L.stride;
  static bool init = false;
  if (!init) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&decode_fixed_kernel<TR, FRAME>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    init = true;
  }
  hipLaunchKernelGGL((decode_fixed_kernel<TR, FRAME>), dim3((unsigned)tiles), dim3(kWG), lds, s, L, in,
                     status);
  return hipGetLastError();
}

}  // namespace

// Records per tile: 64 (one field per wave-instruction) while a tile fits
// 80 KiB of LDS (two workgroups per CU), else fewer records, more fields.
static int pick_tr(int stride) {
  if (64 * stride <= 80 * 1024) return 64;
  if (32 * stride <= 80 * 1024) return 32;
  if (16 * stride <= 80 * 1024) return 16;
  if (8 * stride <= 160 * 1024) return 8;
  return 0;
}

hipError_t launch_encode_fixed(const FixedLaunch& L, uint8_t* out, hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  switch (pick_tr(L.stride) * 2 + (L.frame ? 1 : 0)) {
    case 128: return launch_encode_tr<64, false>(L, out, s);
    case 129: return launch_encode_tr<64, true>(L, out, s);
    case 64: return launch_encode_tr<32, false>(L, out, s);
    case 65: return launch_encode_tr<32, true>(L, out, s);
    case 32: return launch_encode_tr<16, false>(L, out, s);
    case 33: return launch_encode_tr<16, true>(L, out, s);
    case 16: return launch_encode_tr<8, false>(L, out, s);
    case 17: return launch_encode_tr<8, true>(L, out, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_decode_fixed(const FixedLaunch& L, const uint8_t* in, int32_t* status, hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  switch (pick_tr(L.stride) * 2 + (L.frame ? 1 : 0)) {
    case 128: return launch_decode_tr<64, false>(L, in, status, s);
    case 129: return launch_decode_tr<64, true>(L, in, status, s);
    case 64: return launch_decode_tr<32, false>(L, in, status, s);
    case 65: return launch_decode_tr<32, true>(L, in, status, s);
    case 32: return launch_decode_tr<16, false>(L, in, status, s);
    case 33: return launch_decode_tr<16, true>(L, in, status, s);
    case 16: return launch_decode_tr<8, false>(L, in, status, s);
    case 17: return launch_decode_tr<8, true>(L, in, status, s);
    default: return hipErrorInvalidValue;
  }
}

bool fixed_tiled_supported(int stride) { return pick_tr(stride) != 0; }

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

hipError_t launch_var_sizes(const VarLaunch& L, int64_t* d_row_offsets, hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  const int64_t blocks = (L.num_rows + kWG - 1) / kWG;
  hipLaunchKernelGGL(var_sizes_kernel, dim3((unsigned)blocks), dim3(kWG), 0, s, L, d_row_offsets);
  return hipGetLastError();
}

hipError_t launch_var_encode(const VarLaunch& L, const int64_t* offs, uint8_t* out, int64_t capacity,
                             int32_t* status, hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  const int64_t blocks = (L.num_rows + kWG - 1) / kWG;
  hipLaunchKernelGGL(var_encode_kernel, dim3((unsigned)blocks), dim3(kWG), 0, s, L, offs, out, capacity,
                     status);
  return hipGetLastError();
}

hipError_t launch_var_decode_lengths(const VarLaunch& L, const uint8_t* rows, const int64_t* offs,
                                     int32_t* status, hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  const int64_t blocks = (L.num_rows + kWG - 1) / kWG;
  hipLaunchKernelGGL(var_decode_kernel<false>, dim3((unsigned)blocks), dim3(kWG), 0, s, L, rows, offs,
                     status);
  return hipGetLastError();
}

hipError_t launch_var_decode(const VarLaunch& L, const uint8_t* rows, const int64_t* offs, int32_t* status,
                             hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  const int64_t blocks = (L.num_rows + kWG - 1) / kWG;
  hipLaunchKernelGGL(var_decode_kernel<true>, dim3((unsigned)blocks), dim3(kWG), 0, s, L, rows, offs,
                     status);
  return hipGetLastError();
}

}  // namespace fory_amd
