// varlen.hip — gfx950 kernels for varlen / nested row-format schemas
// (strings, binary, lists, maps, nested structs, collection frames).
//
// Byte layout restated from the Java writer (F = java/fory-format/src/main/java/
// org/apache/fory/format):
//   var   = slot (relOffset<<32 | size), data appended in ordinal
//           order, zero-padded to 8                                F/row/binary/writer/BinaryWriter.java:106-194
//   array = [i64 n][bitmap][n x elemSize padded to 8]              F/row/binary/writer/BinaryArrayWriter.java:93-118
//   map   = [i64 keyArrayBytes][key array][value array]            F/row/binary/BinaryMap.java:30-77
//   struct= child row inline at the field's writerIndex           F/encoder/BaseBinaryEncoderBuilder.java:436-490
//   frame = [i32 8+rowSize][i64 schemaHash][row]                   F/encoder/Encoders.java:213-225
//
// Row sizes come from a sizes pass + device scan (row offsets); the encode and
// decode run either the cooperative tile kernels (one workgroup per 64-record
// tile, row image in LDS), the generic one-wave tile interpreter (maps, List<Bean>,
// string list elements, collection frames) or the per-record global interpreter
// (tiles beyond every LDS budget).
#include <mutex>

#include "kcommon.h"

namespace fory_amd {

namespace {

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

// Copies n bytes from global `src` (any alignment) to `dst` (4-byte aligned;
// LDS image or global row) and zero-pads to round8(n): BinaryWriter.writeUnaligned
// + zeroOutPaddingBytes (BinaryWriter.java:117-121,162-194). Source dwords are
// read aligned (each holds at least one byte of the string, so never crosses
// the column's end) and funnel-shifted.
__device__ __forceinline__ void copy_padded(uint8_t* dst, const uint8_t* src, int64_t n) {
  const uintptr_t sa = reinterpret_cast<uintptr_t>(src);
  const int sb = (int)(sa & 3);
  const uint8_t* s0 = reinterpret_cast<const uint8_t*>(sa - sb);
  const int64_t n4 = (n + 3) & ~int64_t(3);
  for (int64_t k = 0, q = 0; k < n4; k += 4, ++q) {
    const uint32_t a = *gp(reinterpret_cast<const uint32_t*>(s0 + 4 * q));
    const int64_t lastb = sb + (k + 4 < n ? k + 4 : n) - 1;  // last needed byte, relative to s0
    const uint32_t b = (lastb >> 2) > q ? *gp(reinterpret_cast<const uint32_t*>(s0 + 4 * q + 4)) : 0u;
    uint32_t w = sb ? (a >> (8 * sb)) | (b << (32 - 8 * sb)) : a;
    const int64_t valid = n - k;
    if (valid < 4) w &= (1u << (8 * valid)) - 1u;
    st32(dst + k, w);
  }
  if (round8(n) > n4) st32(dst + n4, 0);
}

// Copies n bytes from `src` (row bytes: LDS image or global, any alignment)
// to the global column buffer `dst` (any alignment): byte head up to a 4-byte
// aligned destination, dword body, byte tail.
__device__ __forceinline__ void copy_out(uint8_t* dst, const uint8_t* src, int64_t n) {
  int64_t k = 0;
  const int64_t head0 = (int64_t)((4 - (reinterpret_cast<uintptr_t>(dst) & 3)) & 3);
  const int64_t head = head0 < n ? head0 : n;
  for (; k < head; ++k) store_byte(dst + k, src[k]);
  for (; k + 4 <= n; k += 4) {
    const uint32_t w = (uint32_t)src[k] | ((uint32_t)src[k + 1] << 8) | ((uint32_t)src[k + 2] << 16) |
                       ((uint32_t)src[k + 3] << 24);
    *gp(reinterpret_cast<uint32_t*>(dst + k)) = w;
  }
  for (; k < n; ++k) store_byte(dst + k, src[k]);
}

// Bytes of a BinaryArray of n elements of column `it` starting at element e0
// (BinaryArrayWriter.reset(n) + appends, BinaryArrayWriter.java:93-118): header,
// bitmap, fixed part padded to 8, and for string/binary elements (iflags bit2)
// each non-null element's bytes padded to 8.
__device__ __forceinline__ int64_t array_bytes(const ColumnDev& it, int w, int iflags, int64_t e0, int64_t n) {
  int64_t s = 8 + bitmap_bytes(n) + round8(n * w);
  if (iflags & 4)
    for (int64_t j = 0; j < n; ++j)
      if (!(iflags & 1) || col_valid(it, e0 + j)) s += round8((int64_t)it.offsets[e0 + j + 1] - it.offsets[e0 + j]);
  return s;
}

// Row/frame size of record i (BinaryRowWriter.reset + all appends).
__global__ __launch_bounds__(kWG) void var_sizes_kernel(VarLaunch L, const Op* __restrict__ prog, const ColumnDev* __restrict__ cols, int64_t* sizes) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i >= L.num_rows) return;
  // FORY_FRAME_COLLECTION (ArrayEncoder/MapEncoder.encode(MemoryBuffer, T), Encoders.java:418-431,
  // 559-572): [i32 size][the single field's BinaryArray / BinaryMap], no row around it
  const bool coll = L.frame == FORY_FRAME_COLLECTION;
  int64_t size = coll ? 4 : L.fixed_size + frame_header_bytes(L.frame);
  int absent_depth = 0;  // >0: inside a null struct
  for (int pc = 0; pc < L.num_ops; ++pc) {
    const Op op = prog[pc];
    const ColumnDev& c = cols[op.b];
    switch (op.code) {
      case OP_FIXED:
        break;
      case OP_BYTES:
        if (!absent_depth && (!(op.d & 1) || coll || col_valid(c, i))) size += round8((int64_t)c.offsets[i + 1] - c.offsets[i]);
        break;
      case OP_STRUCT_BEGIN:
        if (absent_depth || ((op.d & 1) && !col_valid(c, i))) absent_depth++;
        else size += bitmap_bytes(op.c) + 8LL * op.c;
        break;
      case OP_STRUCT_END:
        if (absent_depth) absent_depth--;
        break;
      case OP_LIST:
        if (!absent_depth && (!(op.d & 1) || coll || col_valid(c, i))) {
          const int64_t e0 = c.offsets[i], n = (int64_t)c.offsets[i + 1] - e0;
          size += array_bytes(cols[op.c], op.e & 0xff, op.e >> 8, e0, n);
        }
        break;
      case OP_LIST_STRUCT: {  // [i64 n][bitmap][n slots][child row per non-null element]
        if (!absent_depth && (!(op.d & 1) || coll || col_valid(c, i))) {
          const int64_t e0 = c.offsets[i], n = (int64_t)c.offsets[i + 1] - e0;
          const int nf = op.e - pc - 1;
          const int64_t ssize = bitmap_bytes(nf) + 8LL * nf;
          int64_t m = n;
          if (op.d & 4) {
            const ColumnDev& sc = cols[op.c];
            m = 0;
            for (int64_t j = 0; j < n; ++j) m += col_valid(sc, e0 + j);
          }
          size += 8 + bitmap_bytes(n) + 8 * n + m * ssize;
        }
        pc = op.e - 1;
        break;
      }
      case OP_MAP:  // [i64 keyArrayBytes][key array][value array]
        if (!absent_depth && (!(op.d & 1) || coll || col_valid(c, i))) {
          const int64_t e0 = c.offsets[i], n = (int64_t)c.offsets[i + 1] - e0;
          size += 8 + array_bytes(cols[op.c], op.e & 0xff, (op.e >> 16) & 0xff, e0, n) +
                  array_bytes(cols[op.c + 1], (op.e >> 8) & 0xff, (op.e >> 24) & 0xff, e0, n);
        }
        break;
    }
  }
  sizes[i] = size;
}

// The same sizes for flat plans (L.flat: top-level and nested-struct strings and
// list<fixed>, no maps / string elements / collection frames), from the var-field
// and struct tables instead of the op program: every validity byte and offsets pair
// is loaded before any is used (unrolled batches), so a row costs one memory latency
// per batch rather than one per op.
constexpr int kSizeBatch = 8;
// Rows per thread of the sizing kernel: the rows of a workgroup's 256 x kSizeRows block,
// kWG apart, so every load stays coalesced; all their loads are issued before any is used.
// One row per thread left each wave bound by two serial round trips (the field table,
// then the columns): round 6, Mixed encode sizing 0.47 -> 0.27 ms.
constexpr int kSizeRows = 4;

__global__ __launch_bounds__(kWG) void var_sizes_flat_kernel(VarLaunch L, const VarFieldDev* __restrict__ vf,
                                                             const StructDev* __restrict__ st, int64_t* sizes) {
  const int64_t i0 = (int64_t)blockIdx.x * (kWG * kSizeRows) + threadIdx.x;
  int64_t size[kSizeRows];
  uint32_t present[kSizeRows];  // bit id: struct id present (id 0 = the row)
#pragma unroll
  for (int r = 0; r < kSizeRows; ++r) {
    size[r] = L.fixed_size + frame_header_bytes(L.frame);
    present[r] = 1;
  }
  if (L.num_struct) {
    uint32_t valid[kSizeRows];  // bit s: struct s's validity bit (a mask, not a bool array: no scratch)
#pragma unroll
    for (int r = 0; r < kSizeRows; ++r) valid[r] = 0;
#pragma unroll
    for (int s = 0; s < kMaxTileStructs; ++s) {
      const bool nullable = s < L.num_struct && (st[s].flags & 1) && st[s].validity;
#pragma unroll
      for (int r = 0; r < kSizeRows; ++r) {
        const int64_t i = i0 + r * kWG;
        uint32_t v = 1;
        if (nullable && i < L.num_rows) v = (gp(st[s].validity)[i >> 3] >> (i & 7)) & 1;
        valid[r] |= v << s;
      }
    }
#pragma unroll
    for (int s = 0; s < kMaxTileStructs; ++s) {
      if (s >= L.num_struct) break;
#pragma unroll
      for (int r = 0; r < kSizeRows; ++r)
        if (((valid[r] >> s) & 1) && ((present[r] >> st[s].parent) & 1)) {
          present[r] |= 1u << (s + 1);
          size[r] += st[s].hdr + 8LL * st[s].nfields;
        }
    }
  }
  for (int v0 = 0; v0 < L.num_var; v0 += kSizeBatch) {
    int32_t a[kSizeRows][kSizeBatch], b[kSizeRows][kSizeBatch];
    uint32_t vb[kSizeRows][kSizeBatch];
#pragma unroll
    for (int k = 0; k < kSizeBatch; ++k) {
      const int v = v0 + k;
#pragma unroll
      for (int r = 0; r < kSizeRows; ++r) a[r][k] = b[r][k] = 0, vb[r][k] = 0xffu;
      if (v < L.num_var) {
        const VarFieldDev& f = vf[v];
        const bool nullable = (f.flags & 1) && f.validity;
#pragma unroll
        for (int r = 0; r < kSizeRows; ++r) {
          const int64_t i = i0 + r * kWG;
          if (i >= L.num_rows) continue;
          if (nullable) vb[r][k] = gp(f.validity)[i >> 3];
          a[r][k] = gp(f.offsets)[i];
          b[r][k] = gp(f.offsets)[i + 1];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kSizeBatch; ++k) {
      const int v = v0 + k;
      if (v >= L.num_var) break;
      const VarFieldDev& f = vf[v];
#pragma unroll
      for (int r = 0; r < kSizeRows; ++r) {
        const int64_t i = i0 + r * kWG;
        if (!((present[r] >> f.parent) & 1) || !((vb[r][k] >> (i & 7)) & 1)) continue;
        const int64_t n = (int64_t)b[r][k] - a[r][k];
        size[r] += f.is_list ? 8 + bitmap_bytes(n) + round8(n * f.w) : round8(n);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < kSizeRows; ++r) {
    const int64_t i = i0 + r * kWG;
    if (i < L.num_rows) *gp(sizes + i) = size[r];
  }
}

constexpr int kFixBatch = 8;  // consecutive OP_FIXED ops whose loads are issued together

// A var/struct/list/map slot store; slot == null for the top-level field of a
// collection frame, which has none.
__device__ __forceinline__ void slot_put(uint8_t* slot, uint64_t v) {
  if (slot) gst64(slot, v);
}

// A BinaryArray of string/binary elements at row + wi: reset(n) with 8-byte element
// slots (BinaryArrayWriter.java:75-85,93-118), then per element write(j, bytes) ->
// writeUnaligned (BinaryWriter.java:162-194): bytes appended at the writerIndex,
// zero-padded to 8, slot = (offset from the array start, size); a null element sets
// its bit, slot 0. Returns the new writerIndex.
__device__ __forceinline__ int64_t enc_bytes_array(uint8_t* row, int64_t wi, const ColumnDev& it, int iflags,
                                                   int64_t e0, int64_t n) {
  const int64_t astart = wi;
  uint8_t* arr = row + astart;
  const int32_t ahdr = 8 + bitmap_bytes(n);
  gst64(arr, (uint64_t)n);
  for (int b = 8; b < ahdr; b += 8) gst64(arr + b, 0);
  wi += ahdr + 8 * n;
  for (int64_t j = 0; j < n; ++j) {
    uint8_t* eslot = arr + ahdr + 8 * j;
    if ((iflags & 1) && !col_valid(it, e0 + j)) {
      arr[8 + (j >> 3)] |= (uint8_t)(1u << (j & 7));
      gst64(eslot, 0);
      continue;
    }
    const int64_t s0 = it.offsets[e0 + j], len = (int64_t)it.offsets[e0 + j + 1] - s0;
    copy_padded(row + wi, it.values + s0, len);
    gst64(eslot, ((uint64_t)(wi - astart) << 32) | (uint32_t)len);
    wi += round8(len);
  }
  return wi;
}

// Reads a BinaryArray of string/binary elements at row + at (n elements, bounds
// row_len): BinaryArray.isNullAt + getString/getBinary per element (UnsafeTrait.java:
// 68-197, offsets relative to the array). LENGTHS: element sizes into
// it.out_offsets[e0 + j + 1] (the caller scans them); else bytes to
// it.out_values + it.out_offsets[e0 + j] and item validity.
template <bool LENGTHS>
__device__ __forceinline__ void dec_bytes_array(const uint8_t* row, int64_t row_len, int64_t at, int64_t n,
                                                const ColumnDev& it, int iflags, int64_t e0, int32_t* status) {
  const uint8_t* arr = row + at;
  const int32_t ahdr = 8 + bitmap_bytes(n);
  for (int64_t j = 0; j < n; ++j) {
    const int64_t q = e0 + j;
    bool en = (arr[8 + (j >> 3)] >> (j & 7)) & 1;
    int64_t len = 0, rel = 0;
    if (!en) {
      const uint64_t os = gld64(arr + ahdr + 8 * j);
      rel = (int32_t)(os >> 32);
      len = (int32_t)(uint32_t)os;
      if (rel < 0 || len < 0 || at + rel + len > row_len) {
        set_status(status, FORY_ERR_CORRUPT);
        len = 0;
      }
    }
    if (LENGTHS) {
      it.out_offsets[q + 1] = (int32_t)len;
    } else {
      if (len > 0) copy_out(it.out_values + it.out_offsets[q], arr + rel, len);
      if ((iflags & 1) && it.out_validity) {
        const uint32_t bit = 1u << (q & 31);
        uint32_t* word = reinterpret_cast<uint32_t*>(it.out_validity) + (q >> 5);
        if (en) g_and(word, ~bit);
        else g_or(word, bit);
      }
    }
  }
}

// Encodes record i into `base` (its frame in STREAM mode, else its row;
// `size` bytes; an LDS tile image or global memory). Generated toRow
// (RowEncoderBuilder.java:177-208) with BaseBinaryEncoderBuilder's per-type
// branches (:149-490) as an op program.
__device__ __forceinline__ void enc_record(const VarLaunch& L, const Op* __restrict__ prog, const ColumnDev* __restrict__ cols, int64_t i, uint8_t* base, int64_t size) {
  uint8_t* row = base;
  // collection frames: the payload sits where the single field's var data would
  // (row + fixed_size); the row's bitmap and slot are never written
  const bool coll = L.frame == FORY_FRAME_COLLECTION;
  if (coll) {
    st32(base, (uint32_t)(size - 4));
    row = base + 4 - L.fixed_size;
  } else if (L.frame == FORY_FRAME_STREAM) {  // Encoders.encode(MemoryBuffer,T): [i32 8+rowSize][i64 hash]
    st32(base, (uint32_t)(size - 4));
    gst64(base + 4, (uint64_t)L.schema_hash);
    row = base + 12;
  } else if (L.frame == FORY_FRAME_HASHED) {  // Encoders.encode(T): [i64 hash][row]
    gst64(base, (uint64_t)L.schema_hash);
    row = base + 8;
  }
  // writer stack: start (relative to row), header bytes, ordinal in parent
  int32_t st_start[kMaxDepth], st_hdr[kMaxDepth], st_ord[kMaxDepth];
  int depth = 0;
  st_start[0] = 0;
  st_hdr[0] = L.bitmap_bytes;
  st_ord[0] = 0;
  int absent = 0;
  int64_t wi = L.fixed_size;  // writerIndex relative to row (BinaryRowWriter.reset)
  if (!coll)
    for (int b = 0; b < L.bitmap_bytes; b += 8) gst64(row + b, 0);
  // pc and the fixed-batch length stay wave-uniform (advanced outside the
  // per-lane branches) so the program and column tables load as scalars.
  for (int pc = 0, cnt = 1; pc < L.num_ops; pc += cnt) {
    const Op op = prog[pc];
    const ColumnDev& c = cols[op.b];
    cnt = 1;
    if (op.code == OP_FIXED)
      while (cnt < kFixBatch && pc + cnt < L.num_ops && prog[pc + cnt].code == OP_FIXED) ++cnt;
    if (op.code == OP_LIST_STRUCT) cnt = op.e - pc;  // the element fields are its sub-program
    if (absent) {
      if (op.code == OP_STRUCT_BEGIN) absent++;
      else if (op.code == OP_STRUCT_END) absent--;
      continue;
    }
    uint8_t* slots = row + st_start[depth] + st_hdr[depth];
    uint8_t* bitmap = row + st_start[depth];
    // collection frames: the top-level field has no slot (slot = null: its writes
    // are skipped) and is never null (a null collection is written from its
    // offsets, i.e. empty; Java's toArray(null) would throw)
    const bool top_coll = coll && depth == 0;
    uint8_t* slot = top_coll ? nullptr : slots + 8 * op.a;
    const bool isnull = !top_coll && (op.d & 1) && !col_valid(c, i);
    switch (op.code) {
      case OP_FIXED: {  // BinaryRowWriter.write(ordinal, v) / setNullAt, batched
        uint64_t v[kFixBatch];
#pragma unroll
        for (int k = 0; k < kFixBatch; ++k) {
          v[k] = 0;
          if (k < cnt) {
            const Op o = prog[pc + k];
            const ColumnDev& cc = cols[o.b];
            if (!(o.d & 1) || col_valid(cc, i)) v[k] = load_elem(cc.values, o.c, i);
          }
        }
#pragma unroll
        for (int k = 0; k < kFixBatch; ++k) {
          if (k < cnt) {
            const Op o = prog[pc + k];
            if ((o.d & 1) && !col_valid(cols[o.b], i)) set_null_bit(bitmap, o.a);
            uint64_t x = v[k];
            if (o.d & 2) x = x ? 1 : 0;
            gst64(slots + 8 * o.a, x);
          }
        }
        break;
      }
      case OP_BYTES: {
        if (isnull) {
          set_null_bit(bitmap, op.a);
          slot_put(slot, 0);
          break;
        }
        const int64_t s0 = c.offsets[i], n = (int64_t)c.offsets[i + 1] - s0;
        copy_padded(row + wi, c.values + s0, n);
        slot_put(slot, ((uint64_t)(wi - st_start[depth]) << 32) | (uint32_t)n);
        wi += round8(n);
        break;
      }
      case OP_STRUCT_BEGIN: {
        if (isnull) {
          set_null_bit(bitmap, op.a);
          slot_put(slot, 0);
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
        const int64_t sz = wi - st_start[depth];
        const int32_t rel = st_start[depth] - st_start[depth - 1];
        const int32_t ord = st_ord[depth];
        depth--;
        gst64(row + st_start[depth] + st_hdr[depth] + 8 * ord, ((uint64_t)(uint32_t)rel << 32) | (uint32_t)sz);
        break;
      }
      case OP_LIST: {
        if (isnull) {
          set_null_bit(bitmap, op.a);
          slot_put(slot, 0);
          break;
        }
        // BinaryArrayWriter.reset(n) + per-element write (BinaryArrayWriter.java:93-158)
        const ColumnDev& it = cols[op.c];
        const int w = op.e & 0xff;
        const int iflags = op.e >> 8;
        const int64_t e0 = c.offsets[i], n = (int64_t)c.offsets[i + 1] - e0;
        const int64_t astart = wi;
        if (iflags & 4) {  // string/binary elements
          wi = enc_bytes_array(row, wi, it, iflags, e0, n);
          slot_put(slot, ((uint64_t)(astart - st_start[depth]) << 32) | (uint32_t)(wi - astart));
          break;
        }
        const int32_t ahdr = 8 + bitmap_bytes(n);
        uint8_t* arr = row + astart;
        gst64(arr, (uint64_t)n);
        for (int b = 8; b < ahdr; b += 8) gst64(arr + b, 0);
        uint8_t* data = arr + ahdr;
        const int64_t dsz = n * w, fixed_part = round8(dsz);
        if (w == 8 && !(iflags & 3)) {  // fromPrimitiveArray fast path: 8-byte elements, no nulls
          for (int64_t j = 0; j < n; j += 4) {
            uint64_t x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = j + u < n ? load_elem(it.values, 8, e0 + j + u) : 0;
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (j + u < n) gst64(data + 8 * (j + u), x[u]);
          }
        } else {
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
          for (int64_t k = dsz; k < fixed_part; ++k) data[k] = 0;
        }
        wi += ahdr + fixed_part;
        slot_put(slot, ((uint64_t)(astart - st_start[depth]) << 32) | (uint32_t)(wi - astart));
        break;
      }
      case OP_LIST_STRUCT: {
        if (isnull) {
          set_null_bit(bitmap, op.a);
          slot_put(slot, 0);
          break;
        }
        // BinaryArrayWriter.reset(n) with 8-byte element slots, then per element
        // serializeForBean (BaseBinaryEncoderBuilder.java:436-490): child row at the
        // writerIndex, element slot = (offset from the array start, child size);
        // a null element only sets its bit (slot 0).
        const ColumnDev& sc = cols[op.c];
        const int nf = op.e - pc - 1;
        const int32_t shdr = bitmap_bytes(nf);
        const int64_t ssize = shdr + 8LL * nf;
        const int64_t e0 = c.offsets[i], n = (int64_t)c.offsets[i + 1] - e0;
        const int64_t astart = wi;
        const int32_t ahdr = 8 + bitmap_bytes(n);
        uint8_t* arr = row + astart;
        gst64(arr, (uint64_t)n);
        for (int b = 8; b < ahdr; b += 8) gst64(arr + b, 0);
        wi += ahdr + 8 * n;
        for (int64_t j = 0; j < n; ++j) {
          const int64_t q = e0 + j;
          if ((op.d & 4) && !col_valid(sc, q)) {
            arr[8 + (j >> 3)] |= (uint8_t)(1u << (j & 7));
            gst64(arr + ahdr + 8 * j, 0);
            continue;
          }
          uint8_t* srow = row + wi;
          for (int b = 0; b < shdr; b += 8) gst64(srow + b, 0);
          for (int f = 0; f < nf; ++f) {  // BinaryRowWriter.write / setNullAt of each field
            const Op o = prog[pc + 1 + f];
            const ColumnDev& cc = cols[o.b];
            uint64_t v = 0;
            if ((o.d & 1) && !col_valid(cc, q)) set_null_bit(srow, f);
            else v = load_elem(cc.values, o.c, q);
            if (o.d & 2) v = v ? 1 : 0;
            gst64(srow + shdr + 8 * f, v);
          }
          gst64(arr + ahdr + 8 * j, ((uint64_t)(wi - astart) << 32) | (uint32_t)ssize);
          wi += ssize;
        }
        slot_put(slot, ((uint64_t)(astart - st_start[depth]) << 32) | (uint32_t)(wi - astart));
        break;
      }
      case OP_MAP: {
        if (isnull) {
          set_null_bit(bitmap, op.a);
          slot_put(slot, 0);
          break;
        }
        // serializeForMap (BaseBinaryEncoderBuilder.java:370-427): reserve 8 bytes,
        // key array (serializeForArray of keySet), back-patch its size
        // (writeDirectly(offset, size), BinaryWriter.java:239-241), value array,
        // then setOffsetAndSize(ordinal, offset, writerIndex - offset).
        const int64_t e0 = c.offsets[i], n = (int64_t)c.offsets[i + 1] - e0;
        const int64_t mstart = wi;
        wi += 8;
        int64_t keybytes = 0;
        for (int part = 0; part < 2; ++part) {  // keys, then values
          const ColumnDev& it = cols[op.c + part];
          const int w = (op.e >> (8 * part)) & 0xff;
          const int iflags = (op.e >> (16 + 8 * part)) & 0xff;
          if (iflags & 4) {  // string/binary keys or values
            const int64_t a0 = wi;
            wi = enc_bytes_array(row, wi, it, iflags, e0, n);
            if (part == 0) keybytes = wi - a0;
            continue;
          }
          uint8_t* arr = row + wi;
          const int32_t ahdr = 8 + bitmap_bytes(n);
          gst64(arr, (uint64_t)n);  // BinaryArrayWriter.reset(n) (BinaryArrayWriter.java:93-118)
          for (int b = 8; b < ahdr; b += 8) gst64(arr + b, 0);
          uint8_t* data = arr + ahdr;
          const int64_t fixed_part = round8(n * w);
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
          for (int64_t k = n * w; k < fixed_part; ++k) data[k] = 0;
          wi += ahdr + fixed_part;
          if (part == 0) keybytes = ahdr + fixed_part;
        }
        gst64(row + mstart, (uint64_t)keybytes);
        slot_put(slot, ((uint64_t)(mstart - st_start[depth]) << 32) | (uint32_t)(wi - mstart));
        break;
      }
    }
  }
}

// Decodes record i from `base` (frame or row; `row_len` bytes; LDS image or
// global). Pass 1 (WRITE = false): lengths of every varlen column into
// out_offsets[i+1] (bytes for STRING/BINARY, elements for LIST). Pass 2:
// values, validity, list items. Generated fromRow (RowEncoderBuilder.java:
// 215-318) over BinaryRow/UnsafeTrait getters (UnsafeTrait.java:68-197).
// Called by all 64 lanes of a wave whose records are consecutive (ballots).
template <bool WRITE>
__device__ __forceinline__ void dec_record(const VarLaunch& L, const Op* __restrict__ prog, const ColumnDev* __restrict__ cols, int64_t i0, bool live, const uint8_t* base, int64_t row_len,
                           int32_t* status) {
  const int64_t i = live ? i0 : 0;
  const uint8_t* row = base;
  bool bad = !live;
  const bool coll = L.frame == FORY_FRAME_COLLECTION;
  if (live && coll) {  // ArrayEncoder/MapEncoder.decode(MemoryBuffer): [i32 size][payload] (Encoders.java:394-404)
    const uint32_t len = ld32(base);
    if ((int64_t)len + 4 != row_len || len < 8) {
      if (WRITE) set_status(status, FORY_ERR_CORRUPT);
      bad = true;
    }
    row = base + 4 - L.fixed_size;  // the payload sits where the field's var data would
    row_len += L.fixed_size - 4;
  } else if (live && L.frame == FORY_FRAME_STREAM) {
    const uint32_t len = ld32(base);
    const uint64_t h = gld64(base + 4);
    if (h != (uint64_t)L.schema_hash) { if (WRITE) set_status(status, FORY_ERR_SCHEMA_MISMATCH); bad = true; }
    else if ((int64_t)len + 4 != row_len || len < (uint32_t)(8 + L.fixed_size)) { if (WRITE) set_status(status, FORY_ERR_CORRUPT); bad = true; }
    row = base + 12;
    row_len -= 12;
  } else if (live && L.frame == FORY_FRAME_HASHED) {  // Encoder.decode(byte[]) (Encoders.java:195-197)
    const uint64_t h = gld64(base);
    if (h != (uint64_t)L.schema_hash) { if (WRITE) set_status(status, FORY_ERR_SCHEMA_MISMATCH); bad = true; }
    else if (row_len < 8 + L.fixed_size) { if (WRITE) set_status(status, FORY_ERR_CORRUPT); bad = true; }
    row = base + 8;
    row_len -= 8;
  }
  int32_t st_start[kMaxDepth], st_hdr[kMaxDepth];
  int depth = 0;
  st_start[0] = 0;
  st_hdr[0] = L.bitmap_bytes;
  int absent = bad ? 1 << 20 : 0;  // >0: this record's subtree is null/absent
  const int lane = threadIdx.x & 63;
  for (int pc = 0; pc < L.num_ops; ++pc) {
    const Op op = prog[pc];
    const ColumnDev& c = cols[op.b];
    if (WRITE && op.code == OP_FIXED) {  // batch of consecutive fixed fields: reads first, then stores
      int cnt = 1;
      while (cnt < kFixBatch && pc + cnt < L.num_ops && prog[pc + cnt].code == OP_FIXED) ++cnt;
      uint64_t v[kFixBatch];
      bool nul[kFixBatch];
#pragma unroll
      for (int k = 0; k < kFixBatch; ++k) {
        v[k] = 0;
        nul[k] = true;
        if (k < cnt && !absent) {
          const Op o = prog[pc + k];
          const uint8_t* bm = row + st_start[depth];
          nul[k] = (bm[o.a >> 3] >> (o.a & 7)) & 1;  // BinaryRow.isNullAt
          if (!nul[k]) v[k] = gld64(row + st_start[depth] + st_hdr[depth] + 8 * o.a);
        }
      }
#pragma unroll
      for (int k = 0; k < kFixBatch; ++k) {
        if (k < cnt) {
          const Op o = prog[pc + k];
          const ColumnDev& cc = cols[o.b];
          if ((o.d & 1) && cc.out_validity) {
            const uint64_t m = __ballot(live && !nul[k]);
            const int64_t w0 = i0 - lane;
            if (lane == 0 && w0 < L.num_rows) {
              const int64_t nrow = L.num_rows - w0 < 64 ? L.num_rows - w0 : 64;
              uint8_t* vb = cc.out_validity + (w0 >> 3);
              for (int b = 0; b < (int)((nrow + 7) >> 3); ++b) store_byte(vb + b, (uint8_t)(m >> (8 * b)));
            }
          }
          if (live) {
            uint64_t x = nul[k] ? 0 : v[k];
            if (o.d & 2) x = (x & 0xff) ? 1 : 0;
            store_elem(cc.out_values, o.c, i, x);
          }
        }
      }
      pc += cnt - 1;
      continue;
    }
    bool isnull = true;
    const uint8_t* slot = nullptr;  // null + !isnull: the top-level payload of a collection frame
    if (!absent) {
      if (coll && depth == 0) {
        isnull = false;
      } else {
        const uint8_t* bm = row + st_start[depth];
        isnull = (bm[op.a >> 3] >> (op.a & 7)) & 1;  // BinaryRow.isNullAt
        slot = row + st_start[depth] + st_hdr[depth] + 8 * op.a;
      }
    }
    const uint64_t coll_os = ((uint64_t)L.fixed_size << 32) | (uint32_t)(row_len - L.fixed_size);
    // Row-level validity of this column (rows of a wave are consecutive).
    if (WRITE && (op.d & 1) && c.out_validity && op.code != OP_STRUCT_END) {
      const uint64_t m = __ballot(live && !isnull);
      const int64_t w0 = i0 - lane;
      if (lane == 0 && w0 < L.num_rows) {
        const int64_t nrow = L.num_rows - w0 < 64 ? L.num_rows - w0 : 64;
        uint8_t* vb = c.out_validity + (w0 >> 3);
        for (int b = 0; b < (int)((nrow + 7) >> 3); ++b) store_byte(vb + b, (uint8_t)(m >> (8 * b)));
      }
    }
    switch (op.code) {
      case OP_FIXED: {  // pass 1 only (WRITE batches above)
        break;
      }
      case OP_BYTES: {
        int64_t n = 0, rel = 0;
        if (!isnull) {
          const uint64_t os = (slot ? gld64(slot) : coll_os);
          rel = (int32_t)(os >> 32);
          n = (int32_t)(uint32_t)os;
          if (n < 0 || rel < 0 || st_start[depth] + rel + n > row_len) { set_status(status, FORY_ERR_CORRUPT); n = 0; }
        }
        if (live) {
          if (!WRITE) {
            if (!L.level2) c.out_offsets[i + 1] = (int32_t)n;
          } else if (n > 0) {
            copy_out(c.out_values + c.out_offsets[i], row + st_start[depth] + rel, n);
          }
        }
        break;
      }
      case OP_STRUCT_BEGIN: {
        if (absent || isnull) {
          absent++;
          break;
        }
        const uint64_t os = (slot ? gld64(slot) : coll_os);
        const int64_t rel = (int32_t)(os >> 32);
        if (rel < 0 || st_start[depth] + rel + bitmap_bytes(op.c) + 8LL * op.c > row_len) {
          set_status(status, FORY_ERR_CORRUPT);
          absent++;
          break;
        }
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
          const uint64_t os = (slot ? gld64(slot) : coll_os);
          rel = (int32_t)(os >> 32);
          if (rel < 0 || st_start[depth] + rel + 8 > row_len) {
            set_status(status, FORY_ERR_CORRUPT);
          } else {
            n = (int32_t)(int64_t)gld64(row + st_start[depth] + rel);  // BinaryArray.pointTo
            const int w = op.e & 0xff;
            if (n < 0 || st_start[depth] + rel + 8 + bitmap_bytes(n) + n * w > row_len) {
              set_status(status, FORY_ERR_CORRUPT);
              n = 0;
            }
          }
        }
        if (live) {
          const ColumnDev& it = cols[op.c];
          const int iflags = op.e >> 8;
          if (!WRITE) {
            if (!L.level2) c.out_offsets[i + 1] = (int32_t)n;
            else if ((iflags & 4) && it.out_offsets && n > 0)  // element sizes (list offsets final)
              dec_bytes_array<true>(row, row_len, st_start[depth] + rel, n, it, iflags, c.out_offsets[i], status);
          } else if (n > 0 && (iflags & 4)) {
            dec_bytes_array<false>(row, row_len, st_start[depth] + rel, n, it, iflags, c.out_offsets[i], status);
          } else if (n > 0) {
            const int w = op.e & 0xff;
            const uint8_t* arr = row + st_start[depth] + rel;
            const int32_t ahdr = 8 + bitmap_bytes(n);
            const int64_t e0 = c.out_offsets[i];
            if (w == 8 && !(iflags & 3)) {  // BinaryArray.toLongArray fast path
              for (int64_t j = 0; j < n; j += 4) {
                uint64_t x[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) x[u] = j + u < n ? gld64(arr + ahdr + 8 * (j + u)) : 0;
#pragma unroll
                for (int u = 0; u < 4; ++u)
                  if (j + u < n) {
                    // BinaryArray null bits still apply for a not-null item field written by a peer
                    const bool en = (arr[8 + ((j + u) >> 3)] >> ((j + u) & 7)) & 1;
                    store_elem(it.out_values, 8, e0 + j + u, en ? 0 : x[u]);
                  }
              }
            } else {
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
                  if (en) g_and(word, ~bit);
                  else g_or(word, bit);
                }
              }
            }
          }
        }
        break;
      }
      case OP_LIST_STRUCT: {  // getArray + per element getStruct (UnsafeTrait.java:160-186)
        const int nf = op.e - pc - 1;
        const int32_t shdr = bitmap_bytes(nf);
        const int64_t ssize = shdr + 8LL * nf;
        int64_t n = 0, at = 0;
        if (!isnull) {
          const uint64_t os = (slot ? gld64(slot) : coll_os);
          at = st_start[depth] + (int32_t)(os >> 32);
          if ((int32_t)(os >> 32) < 0 || at + 8 > row_len) {
            set_status(status, FORY_ERR_CORRUPT);
          } else {
            n = (int32_t)(int64_t)gld64(row + at);
            if (n < 0 || at + 8 + bitmap_bytes(n) + 8 * n > row_len) {
              set_status(status, FORY_ERR_CORRUPT);
              n = 0;
            }
          }
        }
        if (live) {
          if (!WRITE) {
            if (!L.level2) c.out_offsets[i + 1] = (int32_t)n;
          } else if (n > 0) {
            const ColumnDev& sc = cols[op.c];
            const uint8_t* arr = row + at;
            const int32_t ahdr = 8 + bitmap_bytes(n);
            const int64_t e0 = c.out_offsets[i];
            for (int64_t j = 0; j < n; ++j) {
              const int64_t q = e0 + j;
              bool en = (arr[8 + (j >> 3)] >> (j & 7)) & 1;  // BinaryArray.isNullAt
              const uint8_t* srow = nullptr;
              if (!en) {
                const uint64_t os2 = gld64(arr + ahdr + 8 * j);
                const int64_t r2 = (int32_t)(os2 >> 32);
                if (r2 < 0 || at + r2 + ssize > row_len) {
                  set_status(status, FORY_ERR_CORRUPT);
                  en = true;
                } else {
                  srow = arr + r2;
                }
              }
              const uint32_t bit = 1u << (q & 31);
              if ((op.d & 4) && sc.out_validity) {
                uint32_t* word = reinterpret_cast<uint32_t*>(sc.out_validity) + (q >> 5);
                if (en) g_and(word, ~bit);
                else g_or(word, bit);
              }
              for (int f = 0; f < nf; ++f) {
                const Op o = prog[pc + 1 + f];
                const ColumnDev& cc = cols[o.b];
                const bool nul = en || ((srow[f >> 3] >> (f & 7)) & 1);
                uint64_t v = 0;
                if (!nul) v = gld64(srow + shdr + 8 * f);
                if (o.d & 2) v = (v & 0xff) ? 1 : 0;
                store_elem(cc.out_values, o.c, q, v);
                if ((o.d & 1) && cc.out_validity) {
                  uint32_t* word = reinterpret_cast<uint32_t*>(cc.out_validity) + (q >> 5);
                  if (nul) g_and(word, ~bit);
                  else g_or(word, bit);
                }
              }
            }
          }
        }
        pc = op.e - 1;  // the element fields were this op's sub-program
        break;
      }
      case OP_MAP: {  // BinaryMap.pointTo (BinaryMap.java:62-77): keys + values arrays
        int64_t n = 0, rel = 0, kat = 0, vat = 0;
        if (!isnull) {
          const uint64_t os = (slot ? gld64(slot) : coll_os);
          rel = (int32_t)(os >> 32);
          const int64_t msz = (int32_t)(uint32_t)os;
          const int64_t at = st_start[depth] + rel;
          if (rel < 0 || msz < 8 || at + msz > row_len) {
            set_status(status, FORY_ERR_CORRUPT);
          } else {
            const int64_t kbytes = (int32_t)ld32(row + at);  // buf.getInt32(offset)
            kat = at + 8;
            vat = kat + kbytes;
            const int kw = op.e & 0xff, vw = (op.e >> 8) & 0xff;
            if (kbytes < 8 || vat + 8 > at + msz) {
              set_status(status, FORY_ERR_CORRUPT);
            } else {
              n = (int32_t)(int64_t)gld64(row + kat);
              const int64_t nv = (int32_t)(int64_t)gld64(row + vat);
              if (n < 0 || n != nv || kat + 8 + bitmap_bytes(n) + n * kw > vat ||
                  vat + 8 + bitmap_bytes(n) + n * vw > at + msz) {
                set_status(status, FORY_ERR_CORRUPT);  // keys.numElements() != values.numElements()
                n = 0;
              }
            }
          }
        }
        if (live) {
          if (!WRITE) {
            if (!L.level2) {
              c.out_offsets[i + 1] = (int32_t)n;
            } else if (n > 0) {  // string/binary key or value sizes (entry offsets final)
              for (int part = 0; part < 2; ++part) {
                const ColumnDev& it = cols[op.c + part];
                const int iflags = (op.e >> (16 + 8 * part)) & 0xff;
                if ((iflags & 4) && it.out_offsets)
                  dec_bytes_array<true>(row, row_len, part ? vat : kat, n, it, iflags, c.out_offsets[i], status);
              }
            }
          } else if (n > 0) {
            const int64_t e0 = c.out_offsets[i];
            for (int part = 0; part < 2; ++part) {
              const ColumnDev& it = cols[op.c + part];
              const int w = (op.e >> (8 * part)) & 0xff;
              const int iflags = (op.e >> (16 + 8 * part)) & 0xff;
              if (iflags & 4) {
                dec_bytes_array<false>(row, row_len, part ? vat : kat, n, it, iflags, e0, status);
                continue;
              }
              const uint8_t* arr = row + (part ? vat : kat);
              const int32_t ahdr = 8 + bitmap_bytes(n);
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
                  if (en) g_and(word, ~bit);
                  else g_or(word, bit);
                }
              }
            }
          }
        }
        break;
      }
    }
  }
}

// Global-memory interpreters (one lane per record): tiles whose rows exceed
// the LDS budget, and the FORY_ROWFMT_VARTILE=0 A/B baseline.
__global__ __launch_bounds__(kWG) void var_encode_kernel(VarLaunch L, const Op* __restrict__ prog, const ColumnDev* __restrict__ cols, const int64_t* __restrict__ offs,
                                                         uint8_t* __restrict__ out, int64_t capacity,
                                                         int32_t* status) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i >= L.num_rows) return;
  const int64_t beg = offs[i], end = offs[i + 1];
  if (end > capacity || beg < 0 || end < beg) {
    set_status(status, FORY_ERR_CAPACITY);
    return;
  }
  enc_record(L, prog, cols, i, out + beg, end - beg);
}

template <bool WRITE>
__global__ __launch_bounds__(kWG) void var_decode_kernel(VarLaunch L, const Op* __restrict__ prog, const ColumnDev* __restrict__ cols, const uint8_t* __restrict__ in,
                                                         const int64_t* __restrict__ offs, int32_t* status) {
  const int64_t i0 = (int64_t)blockIdx.x * kWG + threadIdx.x;
  const bool live = i0 < L.num_rows;
  const int64_t i = live ? i0 : 0;
  dec_record<WRITE>(L, prog, cols, i0, live, in + offs[i], offs[i + 1] - offs[i], status);
}

// Tiles whose image exceeds a launch's LDS budget are appended to `list`
// (atomic `count`) by the main launch and processed by a small persistent
// launch of the same kernel with a big image (`cap` = its budget); only tiles
// beyond that (or with misaligned bases) take the per-record global path.
struct SpillArgs {
  int32_t* list;
  int32_t* count;
  int32_t cap;  // LDS image budget of the spill launch
  int32_t pad;
};

// Tile engine: one wave per tile of 64 consecutive records. The tile's bytes
// [offs[r0], offs[r0+64]) are one contiguous run of the output/input, so the
// wave assembles (encode) or stages (decode) them in an LDS image placed at
// the run's 16-byte phase, and HBM sees aligned 16-B stores/loads instead of
// 64 lanes each touching its own row. Tiles bigger than the LDS budget (or
// with malformed offsets) fall back to the per-record global interpreter.
__device__ __forceinline__ bool var_tile_bounds(const int64_t* offs, int64_t n, int64_t r0, int lane, int64_t* B0,
                                                int64_t* B1, int64_t* beg, int64_t* end, bool* live) {
  const int rows = n - r0 < 64 ? (int)(n - r0) : 64;
  *live = lane < rows;
  *B0 = offs[r0];
  *B1 = offs[r0 + rows];
  *beg = *live ? offs[r0 + lane] : *B0;
  *end = *live ? offs[r0 + lane + 1] : *B0;
  const bool ok = !*live || (*beg >= *B0 && *end >= *beg && *end <= *B1);
  return __ballot(!ok) == 0 && ((*B0 | *B1) & 3) == 0 && *B1 >= *B0;
}

// logical tile of workgroup b under FORY_ROWFMT_VARXCD=C (A/B): dispatch b runs on XCD
// b % 8, so runs of C consecutive tiles per XCD keep each XCD's concurrent tiles
// adjacent (its L2 and TLB see one region); C < 0: one run per XCD over the grid
__device__ __forceinline__ int64_t var_tile(int64_t b, int64_t tiles, int64_t C) {
  if (C < 0) C = tiles / 8;
  if (C <= 0) return b;
  const int64_t blk = b / (8 * C);
  if ((blk + 1) * 8 * C > tiles) return b;
  const int64_t x = b - blk * 8 * C;
  return blk * 8 * C + (x % 8) * C + x / 8;
}

template <bool SPILL>
__global__ __launch_bounds__(64) void var_encode_tile_kernel(VarLaunch L, const Op* __restrict__ prog, const ColumnDev* __restrict__ cols, const int64_t* __restrict__ offs,
                                                             uint8_t* __restrict__ out, int64_t capacity,
                                                             int32_t* status, int cap, SpillArgs sp) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x;
  auto body = [&](int64_t tile) {
  const int64_t r0 = tile * 64;
  int64_t B0, B1, beg, end;
  bool live;
  const bool sane = var_tile_bounds(offs, L.num_rows, r0, lane, &B0, &B1, &beg, &end, &live);
  if (live && (end > capacity || beg < 0 || end < beg)) set_status(status, FORY_ERR_CAPACITY);
  if (__ballot(live && (end > capacity || beg < 0 || end < beg))) return;
  const int mis = (int)(reinterpret_cast<uintptr_t>(out + B0) & 15);
  const int64_t total = mis + (B1 - B0);
  if (!sane || (mis & 3) || total > cap) {
    if (!SPILL && sane && !(mis & 3) && total <= sp.cap) {  // spill: the big-image launch takes it
      if (threadIdx.x == 0) sp.list[atomicAdd(sp.count, 1)] = (int32_t)tile;
      return;
    }
    if (live) enc_record(L, prog, cols, r0 + lane, out + beg, end - beg);
    return;
  }
  if (live) enc_record(L, prog, cols, r0 + lane, lds + mis + (beg - B0), end - beg);
  __syncthreads();
  uint8_t* g = out + B0 - mis;  // 16-byte aligned
  const int tot = (int)total;
  const int nch = (tot + 15) >> 4;
  for (int c = lane; c < nch; c += 64) {
    const int lo = c * 16;
    if (lo >= mis && lo + 16 <= tot) {
      *gp(reinterpret_cast<u32x4*>(g + lo)) = *reinterpret_cast<const u32x4*>(lds + lo);
    } else {
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int o = lo + 4 * d;
        if (o >= mis && o + 4 <= tot) *gp(reinterpret_cast<uint32_t*>(g + o)) = ld32(lds + o);
      }
    }
  }
  };
  if (!SPILL) {
    body(var_tile(blockIdx.x, gridDim.x, L.kn.var_xcd));
    return;
  }
  const int64_t count = *sp.count;  // tiles the main launch spilled
  for (int64_t k = blockIdx.x; k < count; k += gridDim.x) {
    body(sp.list[k]);
    __syncthreads();
  }
}


template <bool WRITE, bool SPILL>
__global__ __launch_bounds__(64) void var_decode_tile_kernel(VarLaunch L, const Op* __restrict__ prog, const ColumnDev* __restrict__ cols, const uint8_t* __restrict__ in,
                                                             const int64_t* __restrict__ offs, int32_t* status,
                                                             int cap, SpillArgs sp) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x;
  auto body = [&](int64_t tile) {
  const int64_t r0 = tile * 64;
  int64_t B0, B1, beg, end;
  bool live;
  const bool sane = var_tile_bounds(offs, L.num_rows, r0, lane, &B0, &B1, &beg, &end, &live);
  const int mis = (int)(reinterpret_cast<uintptr_t>(in + B0) & 15);
  const int64_t total = mis + (B1 - B0);
  if (!sane || (mis & 3) || total > cap) {
    if (!SPILL && sane && !(mis & 3) && total <= sp.cap) {  // spill: the big-image launch takes it
      if (threadIdx.x == 0) sp.list[atomicAdd(sp.count, 1)] = (int32_t)tile;
      return;
    }
    dec_record<WRITE>(L, prog, cols, r0 + lane, live, in + beg, end - beg, status);
    return;
  }
  const uint8_t* g = in + B0 - mis;  // 16-byte aligned
  const int nch = (int)((total + 15) >> 4);
  for (int c0 = 0; c0 < nch; c0 += 64) {  // LDS-DMA, 1 KiB per instruction, all in flight
    if (c0 + lane < nch)
      __builtin_amdgcn_global_load_lds((const GAS void*)(g + (int64_t)(c0 + lane) * 16),
                                       (__attribute__((address_space(3))) void*)(lds + c0 * 16), 16, 0, 2);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  dec_record<WRITE>(L, prog, cols, r0 + lane, live, lds + mis + (beg - B0), end - beg, status);
  };
  if (!SPILL) {
    body(var_tile(blockIdx.x, gridDim.x, L.kn.var_xcd));
    return;
  }
  const int64_t count = *sp.count;  // tiles the main launch spilled
  for (int64_t k = blockIdx.x; k < count; k += gridDim.x) {
    body(sp.list[k]);
    __syncthreads();
  }
}


// ---------------------------------------------------------------------------
// Flat varlen tile kernels: every top-level field FIXED/BOOL, STRING/BINARY or
// LIST<fixed> (VarLaunch::flat). One workgroup of NW (4 or 8) waves per 64-record
// tile; lane = record within each wave.
//   encode: wave 0 writes headers, null bitmaps and the variable-region layout
//   (slot words; payload offsets into LDS `pos`) while all waves fill fixed
//   slots with batched column loads; then each wave takes whole var fields:
//   the tile's span of a string/list column is contiguous in its Arrow
//   buffer, so the wave loads it coalesced into an LDS staging buffer and
//   every lane copies its record's bytes LDS -> LDS; finally the row image
//   leaves as aligned 16-B stores.
//   decode: the mirror image (coalesced row staging in, per-field output
//   spans staged in LDS and stored coalesced).
// Spans larger than the staging buffer, bool/nullable list items and tiles
// bigger than the LDS image take per-lane paths with the same results.
// ---------------------------------------------------------------------------

// Waves that place var payloads in the encode tile kernel: all NW when num_var >= NW
// (wave 0 takes its fields after the layout), else waves 1..NW-1 (wave 0 lays the
// rows out). Keeping wave 0 to the layout always was slower (Mixed encode 6.42 ->
// 6.77 ms); pl_all = 0 selects it.
__host__ __device__ __forceinline__ int var_placers(int num_var, int nw, int pl_all) {
  return pl_all && num_var >= nw ? nw : nw - 1;
}

__device__ __forceinline__ void wave_lds_sync() {
  // LDS ops of one wave execute in order; keep the compiler from reordering.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LDS -> LDS copy of n bytes (src any alignment, dst 4-byte aligned), zero
// padded to round8(n). Reads up to 4 bytes past the source span (staging slack).
// Bytes [8 sb, 8 sb + 32) of the 64-bit pair (hi:lo) -- v_alignbyte_b32.
__device__ __forceinline__ uint32_t funnel(uint32_t lo, uint32_t hi, int sb) {
  return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)sb);
}

// 16 bytes per step with all five source dwords read before the four stores (the
// per-dword loop waited out one LDS round trip per dword: src and dst may alias as
// far as the compiler knows).
__device__ __forceinline__ void lds_copy_padded(uint8_t* dst, const uint8_t* src, int64_t n) {
  const int sb = (int)(reinterpret_cast<uintptr_t>(src) & 3);
  const uint8_t* s0 = src - sb;
  const int64_t n4 = (n + 3) & ~int64_t(3);
  int64_t k = 0;
  for (; k + 16 <= n; k += 16) {
    const uint32_t a0 = ld32(s0 + k), a1 = ld32(s0 + k + 4), a2 = ld32(s0 + k + 8), a3 = ld32(s0 + k + 12);
    const uint32_t a4 = sb ? ld32(s0 + k + 16) : 0u;
    st32(dst + k, funnel(a0, a1, sb));
    st32(dst + k + 4, funnel(a1, a2, sb));
    st32(dst + k + 8, funnel(a2, a3, sb));
    st32(dst + k + 12, funnel(a3, a4, sb));
  }
  for (; k < n4; k += 4) {
    const uint32_t a = ld32(s0 + k);
    uint32_t w = sb ? funnel(a, ld32(s0 + k + 4), sb) : a;
    if (n - k < 4) w &= (1u << (8 * (n - k))) - 1u;
    st32(dst + k, w);
  }
  if (round8(n) > n4) st32(dst + n4, 0);
}

// LDS -> LDS copy of n bytes, any alignments: byte head to a 4-byte aligned
// dst, funnel-shifted dwords, byte tail. Reads up to 4 bytes past the source.
__device__ __forceinline__ void lds_copy_any(uint8_t* dst, const uint8_t* src, int n) {
  int k = (int)((4 - (reinterpret_cast<uintptr_t>(dst) & 3)) & 3);
  if (k > n) k = n;
  for (int j = 0; j < k; ++j) dst[j] = src[j];
  const uint8_t* s = src + k;
  const int sb = (int)(reinterpret_cast<uintptr_t>(s) & 3);
  const uint8_t* s0 = s - sb;
  const int m = (n - k) & ~3;
  int j = 0;
  for (; j + 16 <= m; j += 16) {  // loads before stores, as lds_copy_padded
    const uint32_t a0 = ld32(s0 + j), a1 = ld32(s0 + j + 4), a2 = ld32(s0 + j + 8), a3 = ld32(s0 + j + 12);
    const uint32_t a4 = sb ? ld32(s0 + j + 16) : 0u;
    st32(dst + k + j, funnel(a0, a1, sb));
    st32(dst + k + j + 4, funnel(a1, a2, sb));
    st32(dst + k + j + 8, funnel(a2, a3, sb));
    st32(dst + k + j + 12, funnel(a3, a4, sb));
  }
  for (; j < m; j += 4) {
    const uint32_t a = ld32(s0 + j);
    st32(dst + k + j, sb ? funnel(a, ld32(s0 + j + 4), sb) : a);
  }
  for (int q = k + m; q < n; ++q) dst[q] = src[q];
}

__device__ __forceinline__ void st64_lds(uint8_t* p, uint64_t v) {  // 4-byte aligned LDS
  st32(p, (uint32_t)v);
  st32(p + 4, (uint32_t)(v >> 32));
}

__device__ __forceinline__ void write_validity64(uint8_t* validity, int64_t r0, int rows, uint64_t m) {
  for (int b = 0; b < (rows + 7) >> 3; ++b) store_byte(validity + (r0 >> 3) + b, (uint8_t)(m >> (8 * b)));
}

// Fixed fields of width W (one width group of L.fix): column -> slot, batches of
// kFixBatch loads per wave issued together (branch-free: clamped field index,
// row 0 for idle lanes, nulls selected to 0 afterwards).
// Fields of nested structs go to their child row (sbase, -1 = absent: skipped).
// Batch j (numbered across the width groups from j0) belongs to wave
// fix_owner(j): waves 1..NW-1 first, since wave 0 lays the rows out meanwhile.
__device__ __forceinline__ int fix_owner(int j, int nbatch, int nw) {
  return nbatch <= 2 * (nw - 1) ? 1 + j % (nw - 1) : j % nw;
}

template <int W, int NW, bool NEST = true>
__device__ __forceinline__ void flat_enc_fixed(const VarLaunch& L, const FixedFieldDev* __restrict__ fix, int g0, int g1,
                                               int j0, int nbatch, int wave, int lane, bool live, int64_t i,
                                               uint8_t* row, const StructDev* __restrict__ st,
                                               const int32_t* sbase) {
  const int64_t ii = live ? i : 0;
  for (int k0 = g0, j = j0; k0 < g1; k0 += kFixBatch, ++j) {
    if (fix_owner(j, nbatch, NW) != wave) continue;
    uint64_t v[kFixBatch];
    uint32_t vb[kFixBatch];
#pragma unroll
    for (int k = 0; k < kFixBatch; ++k) {
      const FixedFieldDev& f = fix[min(k0 + k, g1 - 1)];
      v[k] = ldw<W>(f.values, ii);
      vb[k] = f.validity ? load_byte(f.validity + (ii >> 3)) : 0xffu;
    }
#pragma unroll
    for (int k = 0; k < kFixBatch; ++k) {
      if (k0 + k < g1 && live) {
        const FixedFieldDev& f = fix[k0 + k];
        uint64_t x = ((vb[k] >> (ii & 7)) & 1) ? v[k] : 0;
        if (f.flags & 2) x = x ? 1 : 0;
        if (!NEST || !f.parent) {
          st64_lds(row + L.bitmap_bytes + 8 * f.slot, x);
        } else {
          const int32_t b = sbase[f.parent * 64 + lane];
          if (b >= 0) st64_lds(row + b + st[f.parent - 1].hdr + 8 * f.slot, x);
        }
      }
    }
  }
}

// Var payloads are staged per RECORD GROUP: records [lo, hi) of the tile whose
// span of var field f (string bytes or list items, contiguous in the Arrow
// buffer) fits the wave's staging buffer, with the span's item-validity bytes
// behind it (nullable list items). A record too big on its own, and bool items
// (0/1 normalisation), take the per-lane path. e0/e1: the lane's item range
// (nondecreasing over lanes; dead lanes hold the tile's end).
__device__ __forceinline__ int staged_vofs(int phase, int64_t S) { return (int)((phase + S + 4 + 15) & ~15); }

__device__ __forceinline__ int flat_group(const VarFieldDev& f, int64_t e0, int64_t e1, int lo, int rows, int lane,
                                          int stg_bytes, bool* fits) {
  const int64_t base = __shfl(e0, lo);
  int64_t need = (e1 - base) * f.w + 16 + 4 + 16;  // phase + funnel-copy slack + vofs rounding
  if (f.item_validity) need += ((e1 + 7) >> 3) - ((base >> 3) & ~int64_t(3)) + 4;
  const bool ok = (f.iflags & 2) == 0 && lane >= lo && lane < rows && need <= stg_bytes;
  const uint64_t m = __ballot(ok) >> lo;  // a prefix of the lanes from lo (e1 nondecreasing)
  const int cnt = ~m == 0 ? 64 - lo : (int)__builtin_ctzll(~m);
  *fits = cnt > 0;
  return lo + (cnt > 0 ? cnt : 1);
}

// Items [sa, sb) of f (and their validity bytes) -> staging, by LDS-DMA (1 KiB
// per wave instruction; asynchronous: wait vmcnt(0) before reading).
__device__ __forceinline__ void flat_stage_span(const VarFieldDev& f, int64_t sa, int64_t sb, int lane, uint8_t* stg,
                                                int* phase_out, int* vofs_out) {
  const int64_t S = (sb - sa) * f.w;
  const uint8_t* gsrc = f.values + sa * f.w;
  const int phase = (int)(reinterpret_cast<uintptr_t>(gsrc) & 15);
  *phase_out = phase;
  *vofs_out = staged_vofs(phase, S);
  const uint8_t* ga = gsrc - phase;
  const int nch = (int)((phase + S + 15) >> 4);
  for (int c0 = 0; c0 < nch; c0 += 64)
    if (c0 + lane < nch)
      __builtin_amdgcn_global_load_lds((const GAS void*)(ga + (int64_t)(c0 + lane) * 16),
                                       (__attribute__((address_space(3))) void*)(stg + c0 * 16), 16, 0, 0);
  if (f.item_validity && sb > sa) {
    const int64_t A = (sa >> 3) & ~int64_t(3);
    const int nvw = (int)((((sb + 7) >> 3) - A + 3) >> 2);
    const uint8_t* gv = f.item_validity + A;
    for (int k0 = 0; k0 < nvw; k0 += 64)
      if (k0 + lane < nvw)
        __builtin_amdgcn_global_load_lds((const GAS void*)(gv + (int64_t)(k0 + lane) * 4),
                                         (__attribute__((address_space(3))) void*)(stg + *vofs_out + k0 * 4), 4, 0, 0);
  }
}

// Copies the lane's payload of var field f (items e0 .. e0+n) into its row image
// at row + p (staged: from LDS, the group's span starting at item `base`; else
// per lane from global, incl. item null bits and bool items).
__device__ __forceinline__ void flat_place(const VarFieldDev& f, bool staged, const uint8_t* stg, int phase,
                                           int64_t base, int vofs, int p, int64_t e0, int64_t n, uint8_t* row) {
  if (p < 0) return;
  const int w = f.w;
  uint8_t* dst = row + p + (f.is_list ? 8 + bitmap_bytes(n) : 0);
  if (staged) {
    lds_copy_padded(dst, stg + phase + (e0 - base) * w, n * w);
    if (f.item_validity && n > 0) {  // BinaryArrayWriter.setNullAt: item bit set, element left 0
      const uint8_t* sv = stg + vofs;
      const int64_t A = (base >> 3) & ~int64_t(3);  // first staged bitmap byte
      uint8_t* abm = row + p + 8;
      for (int64_t j = 0; j < n;) {  // a staged validity byte at a time: all-valid runs skip
        const int64_t q = e0 + j;
        const int bi = (int)(q & 7);
        const int take = (int)(n - j < 8 - bi ? n - j : 8 - bi);
        const uint32_t m = ((1u << take) - 1u) << bi;
        const uint32_t byte = sv[(q >> 3) - A];
        if ((byte & m) != m) {
          for (int t = 0; t < take; ++t) {
            if ((byte >> (bi + t)) & 1) continue;
            const int64_t jj = j + t;
            abm[jj >> 3] |= (uint8_t)(1u << (jj & 7));
            for (int b = 0; b < w; ++b) dst[jj * w + b] = 0;
          }
        }
        j += take;
      }
    }
  } else if (!f.is_list) {
    copy_padded(dst, f.values + e0, n);
  } else {
    uint8_t* arr = row + p;
    for (int64_t j = 0; j < n; ++j) {
      const bool enull = f.item_validity && !((*gp(f.item_validity + ((e0 + j) >> 3)) >> ((e0 + j) & 7)) & 1);
      uint64_t x = 0;
      if (enull) arr[8 + (j >> 3)] |= (uint8_t)(1u << (j & 7));
      else x = load_elem(f.values, w, e0 + j);
      if (f.iflags & 2) x = x ? 1 : 0;
      switch (w) {
        case 8: st64_lds(dst + 8 * j, x); break;
        case 4: st32(dst + 4 * j, (uint32_t)x); break;
        case 2: dst[2 * j] = (uint8_t)x; dst[2 * j + 1] = (uint8_t)(x >> 8); break;
        default: dst[j] = (uint8_t)x; break;
      }
    }
    for (int64_t k = n * w; k < round8(n * w); ++k) dst[k] = 0;
  }
}

// A validity byte as the aligned dword holding it (a byte load's zero-extension would
// be placed by the compiler right after the load, waiting for it there).
__device__ __forceinline__ uint32_t vbyte_issue(const uint8_t* p) {
  return *gp(reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(3)));
}
__device__ __forceinline__ uint32_t vbyte_get(uint32_t w, const uint8_t* p) {
  return w >> (8 * (reinterpret_cast<uintptr_t>(p) & 3));
}

// Layout of record i for plans with nested struct fields (wave 0 of the encode
// tile kernel): the per-record program walk of enc_record without the value
// copies. One writerIndex is shared by the row and its child rows
// (BinaryRowWriter(schema, parent), BinaryRowWriter.java:54-62): a struct
// field's child row starts at the writerIndex its field is reached
// (serializeForBean, BaseBinaryEncoderBuilder.java:436-490), its fixed part
// is reserved and zero-bitmapped there, its var payloads follow, and the
// parent slot gets (offset relative to the parent, child size) at the END op.
// Outputs: null bits and var/struct slot words in the LDS row image,
// pos[v][lane] (payload offset from the row, -1 = none), sbase[s][lane]
// (child row offset from the row, -1 = null/absent struct).
__device__ __forceinline__ void flat_enc_layout_nested(const VarLaunch& L, const Op* __restrict__ prog,
                                                       const ColumnDev* __restrict__ cols, bool live, int64_t i,
                                                       const StructDev* __restrict__ st, int lane, uint8_t* row,
                                                       int32_t* pos, int32_t* sbase) {
  // the enclosing struct `cur` is wave-uniform (only absence is per record): no
  // per-lane writer stack, starts live in sbase, headers in the struct table
  int cur = 0;
  int32_t cstart = 0, chdr = L.bitmap_bytes;  // this lane's current row start / header bytes
  int absent = live ? 0 : 1 << 20;
  const int64_t ii = live ? i : 0;
  int64_t wi = L.fixed_size;
  int vi = 0, si = 0;  // wave-uniform: var field / struct ids in program order
  for (int pc0 = 0; pc0 < L.num_ops; pc0 += kFixBatch) {
    // this batch's per-record inputs (validity bits, var-field lengths), loads issued together
    bool nul[kFixBatch];
    int32_t nn[kFixBatch];
#pragma unroll
    for (int k = 0; k < kFixBatch; ++k) {
      nul[k] = false;
      nn[k] = 0;
      if (pc0 + k < L.num_ops) {
        const Op op = prog[pc0 + k];
        const ColumnDev& c = cols[op.b];
        if ((op.d & 1) && op.code != OP_STRUCT_END && c.validity)
          nul[k] = !((load_byte(c.validity + (ii >> 3)) >> (ii & 7)) & 1);
        if (op.code == OP_BYTES || op.code == OP_LIST) nn[k] = *gp(c.offsets + ii + 1) - *gp(c.offsets + ii);
      }
    }
#pragma unroll
    for (int k = 0; k < kFixBatch; ++k) {
      if (pc0 + k >= L.num_ops) break;
      const Op op = prog[pc0 + k];
      const bool isnull = nul[k];
      uint8_t* base = row + cstart;
      uint8_t* slot = base + chdr + 8 * op.a;
      switch (op.code) {
        case OP_FIXED:  // BinaryWriter.setNullAt; the value phase writes the slot
          if (!absent && isnull) set_null_bit(base, op.a);
          break;
        case OP_BYTES:
        case OP_LIST: {
          int32_t p = -1;
          if (!absent) {
            if (isnull) {
              set_null_bit(base, op.a);
              st64_lds(slot, 0);
            } else {
              const int64_t n = nn[k];
              const int64_t rel = wi - cstart;
              if (op.code == OP_BYTES) {  // writeUnaligned: (offset<<32 | size), padded payload
                st64_lds(slot, ((uint64_t)rel << 32) | (uint32_t)n);
                p = (int32_t)wi;
                wi += round8(n);
              } else {  // BinaryArrayWriter.reset(n): [i64 n][null bitmap][n * w bytes, padded to 8]
                const int32_t ahdr = 8 + bitmap_bytes(n);
                const int64_t size = ahdr + round8(n * (op.e & 0xff));
                st64_lds(row + wi, (uint64_t)n);
                for (int b = 8; b < ahdr; b += 4) st32(row + wi + b, 0);
                st64_lds(slot, ((uint64_t)rel << 32) | (uint32_t)size);
                p = (int32_t)wi;
                wi += size;
              }
            }
          }
          pos[vi * 64 + lane] = p;
          ++vi;
          break;
        }
        case OP_STRUCT_BEGIN: {
          ++si;
          cur = si;
          int32_t b = -1;
          if (absent) {
            ++absent;
          } else if (isnull) {
            set_null_bit(base, op.a);
            st64_lds(slot, 0);
            absent = 1;
          } else {
            const int32_t h = bitmap_bytes(op.c);
            for (int q = 0; q < h; q += 4) st32(row + wi + q, 0);
            b = (int32_t)wi;
            cstart = b;
            chdr = h;
            wi += h + 8LL * op.c;
          }
          sbase[si * 64 + lane] = b;
          break;
        }
        case OP_STRUCT_END: {
          cur = __builtin_amdgcn_readfirstlane(cur);  // uniform by construction: scalar table loads
          const int par = st[cur - 1].parent;
          const int32_t pstart = par ? sbase[par * 64 + lane] : 0;
          const int32_t phdr = par ? st[par - 1].hdr : L.bitmap_bytes;
          if (absent) {
            --absent;
          } else {
            const int64_t sz = wi - cstart;
            const int32_t rel = cstart - pstart;
            st64_lds(row + pstart + phdr + 8 * op.a, ((uint64_t)(uint32_t)rel << 32) | (uint32_t)sz);
          }
          cur = par;
          cstart = pstart;  // (unused while absent)
          chdr = phdr;
          break;
        }
      }
    }
  }
}

// Child-row offsets of the staged record (decode; wave 0): struct s's row
// starts at its parent's start + the offset in its slot (BinaryRow.getStruct,
// UnsafeTrait.java:160-175); -1 when it or an ancestor is null. Struct ids are
// pre-order, so parents come first. Writes the struct columns' validity.
template <bool WRITE>
__device__ __forceinline__ void flat_dec_struct_bases(const VarLaunch& L, const StructDev* __restrict__ st, bool bad,
                                                      bool live, int lane, int64_t r0, int rows, const uint8_t* row,
                                                      int64_t row_len, int32_t* sbase, int32_t* status) {
  for (int s = 1; s <= L.num_struct; ++s) {
    const StructDev& sd = st[s - 1];
    const int32_t pb = sd.parent ? sbase[sd.parent * 64 + lane] : (bad ? -1 : 0);
    const int32_t ph = sd.parent ? st[sd.parent - 1].hdr : L.bitmap_bytes;
    int32_t b = -1;
    if (pb >= 0 && !((row[pb + (sd.slot >> 3)] >> (sd.slot & 7)) & 1)) {
      const uint8_t* sp = row + pb + ph + 8 * sd.slot;
      const int64_t rel = (int32_t)ld32(sp + 4);
      if (rel < 0 || pb + rel + sd.hdr + 8LL * sd.nfields > row_len) set_status(status, FORY_ERR_CORRUPT);
      else b = (int32_t)(pb + rel);
    }
    sbase[s * 64 + lane] = b;
    if (WRITE && sd.out_validity) {
      const uint64_t m = __ballot(live && b >= 0);
      if (lane == 0) write_validity64(sd.out_validity, r0, rows, m);
    }
  }
}

// Debug timeline (FORY_ROWFMT_VARPROF=1, L.prof set): thread 0 stamps
// s_memrealtime (100 MHz) at phase boundaries into L.prof[tile * 8 + k] (a uniform
// branch when off).
#define FLAT_STAMP(k)                                                                            \
  do {                                                                                          \
    if (L.prof && tid == 0) L.prof[tile * 8 + (k)] = __builtin_amdgcn_s_memrealtime();          \
  } while (0)

// Encode tile kernel body, compiled as two kernels: the default register budget
// (Mixed-like plans are LDS-limited at 4 workgroups per CU anyway) and a lean one for
// 5 waves per SIMD (small-row plans such as Nested are register-limited: encode
// 1.49 -> 1.26 ms; its spills would cost Mixed 27 %). launch_flat_enc_t picks by occupancy.
template <int HDR, int NW, bool NEST, bool SPILL>
__device__ __forceinline__ void var_encode_flat_body(VarLaunch L, const Op* __restrict__ prog, const ColumnDev* __restrict__ cols,
                                                                  const FixedFieldDev* __restrict__ fix, const VarFieldDev* __restrict__ vf,
                                                                  const StructDev* __restrict__ st,
                                                                  const int64_t* __restrict__ offs,
                                                                  uint8_t* __restrict__ out, int64_t capacity,
                                                                  int32_t* status, int cap, SpillArgs sp) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int stg_bytes = L.stg_bytes;
  uint8_t* img = lds;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // var placement: up to 3 fields per wave stay off wave 0 (it lays the rows out)
  const int nplc = var_placers(L.num_var, NW, L.pl_all);
  const int pi = nplc < NW ? wave - 1 : (wave + NW - 1) % NW;  // placer index (-1: none)
  const int nslot = L.num_var < nplc ? L.num_var : nplc;  // staging slots: one per placing wave
  int32_t* pos = reinterpret_cast<int32_t*>(lds + cap + nslot * stg_bytes);  // [num_var][64]
  int32_t* sbase = pos + L.num_var * 64;                                  // [1 + num_struct][64]
  auto body = [&](int64_t tile) {
  FLAT_STAMP(0);
  const int64_t r0 = tile * 64;
  const int64_t i = r0 + lane;
  const int rows = L.num_rows - r0 < 64 ? (int)(L.num_rows - r0) : 64;
  const bool lv = lane < rows;  // == live below
  // Item ranges this wave needs, loaded BEFORE the row bounds (they do not depend on
  // them) so the two round trips overlap: the first var field it places, its later
  // fields, and (wave 0 of a struct-free plan) the layout's first batch of var fields.
  const int v_first = pi < 0 ? L.num_var : pi;
  int64_t pf_e0 = 0, pf_e1 = 0;
  if (wave != 0 && v_first < L.num_var) {
    const VarFieldDev& f = vf[v_first];
    const int64_t ee = *gp(f.offsets + r0 + rows);
    pf_e0 = lv ? *gp(f.offsets + i) : ee;
    pf_e1 = lv ? *gp(f.offsets + i + 1) : ee;
  }
  constexpr int kPre = 3;
  int64_t pe0[kPre], pe1[kPre];
#pragma unroll
  for (int k = 0; k < kPre; ++k) {
    const int v = v_first + (k + 1) * nplc;
    pe0[k] = pe1[k] = 0;
    if (v < L.num_var) {
      const VarFieldDev& f = vf[v];
      const int64_t ee = *gp(f.offsets + r0 + rows);
      pe0[k] = lv ? *gp(f.offsets + i) : ee;
      pe1[k] = lv ? *gp(f.offsets + i + 1) : ee;
    }
  }
  const bool pre_layout = !NEST && wave == 0 && L.num_var > 0;
  int64_t le0[kFixBatch], le1[kFixBatch];
  uint32_t lvb[kFixBatch];
  if (pre_layout) {
    const int64_t ii = lv ? i : 0;
#pragma unroll
    for (int k = 0; k < kFixBatch; ++k) {
      const VarFieldDev& f = vf[min(k, L.num_var - 1)];
      le0[k] = f.offsets[ii];
      le1[k] = f.offsets[ii + 1];
      lvb[k] = f.validity ? load_byte(f.validity + (ii >> 3)) : 0xffu;
    }
  }
  int64_t B0, B1, beg, end;
  bool live;
  const bool sane = var_tile_bounds(offs, L.num_rows, r0, lane, &B0, &B1, &beg, &end, &live);
  const bool capbad = live && (end > capacity || beg < 0 || end < beg);
  if (__ballot(capbad)) {
    if (wave == 0 && capbad) set_status(status, FORY_ERR_CAPACITY);
    return;
  }
  const int mis = (int)(reinterpret_cast<uintptr_t>(out + B0) & 15);
  const int64_t total = mis + (B1 - B0);
  if (!sane || (mis & 3) || total > cap) {
    if (!SPILL && sane && !(mis & 3) && total <= sp.cap) {  // spill: the big-image launch takes it
      if (threadIdx.x == 0) sp.list[atomicAdd(sp.count, 1)] = (int32_t)tile;
      return;
    }
    if (wave == 0 && live) enc_record(L, prog, cols, r0 + lane, out + beg, end - beg);
    return;
  }
  uint8_t* fp = img + mis + (int)(beg - B0);
  uint8_t* row = fp + HDR;
  uint8_t* slots = row + L.bitmap_bytes;
  // var field v is placed by wave (v + 1) % NW: wave 0 lays the rows out while
  // the other waves' first record groups stream into staging (LDS-DMA)
  uint8_t* stg = lds + cap + (pi < 0 ? 0 : pi) * stg_bytes;
  int pf_hi = 0, pf_phase = 0, pf_vofs = 0;
  bool pf_fits = false;
  if (wave != 0 && v_first < L.num_var) {
    const VarFieldDev& f = vf[v_first];
    pf_hi = flat_group(f, pf_e0, pf_e1, 0, rows, lane, stg_bytes, &pf_fits);
    if (pf_fits) flat_stage_span(f, __shfl(pf_e0, 0), __shfl(pf_e1, pf_hi - 1), lane, stg, &pf_phase, &pf_vofs);
  }
  FLAT_STAMP(1);
  if (wave == 0) {
    // Encoders.encode frame header; BinaryRowWriter.reset zeroes the bitmap (BinaryRowWriter.java:76-84)
    if (live) {
      if (HDR == 12) {
        st32(fp, (uint32_t)(end - beg - 4));
        st64_lds(fp + 4, (uint64_t)L.schema_hash);
      } else if (HDR == 8) {
        st64_lds(fp, (uint64_t)L.schema_hash);
      }
      for (int b = 0; b < L.bitmap_bytes; b += 4) st32(row + b, 0);
    }
    if constexpr (NEST) {  // nested struct fields: program walk
      flat_enc_layout_nested(L, prog, cols, live, i, st, lane, row, pos, sbase);
    } else {
    // null bits of nullable fixed fields (this wave only: no bitmap races)
    const int nfix = L.fix_group[4];
    for (int k0 = 0; k0 < nfix; k0 += kFixBatch) {
      uint32_t vb[kFixBatch];
      const int64_t ii = live ? i : 0;
#pragma unroll
      for (int k = 0; k < kFixBatch; ++k) {
        const FixedFieldDev& f = fix[min(k0 + k, nfix - 1)];
        vb[k] = f.validity ? load_byte(f.validity + (ii >> 3)) : 0xffu;
      }
#pragma unroll
      for (int k = 0; k < kFixBatch; ++k)
        if (k0 + k < nfix && live && !((vb[k] >> (ii & 7)) & 1)) set_null_bit(row, fix[k0 + k].slot);
    }
    // variable-region layout in field order (writeUnaligned / BinaryArrayWriter.reset)
    int64_t wi = L.fixed_size;
    for (int v0 = 0; v0 < L.num_var; v0 += kFixBatch) {
      int64_t e0[kFixBatch], e1[kFixBatch];
      uint32_t vb[kFixBatch];
      const int64_t ii = live ? i : 0;
#pragma unroll
      for (int k = 0; k < kFixBatch; ++k) {
        if (v0 == 0) {  // loaded before the row bounds
          e0[k] = le0[k];
          e1[k] = le1[k];
          vb[k] = lvb[k];
          continue;
        }
        const VarFieldDev& f = vf[min(v0 + k, L.num_var - 1)];
        e0[k] = f.offsets[ii];
        e1[k] = f.offsets[ii + 1];
        vb[k] = f.validity ? load_byte(f.validity + (ii >> 3)) : 0xffu;
      }
#pragma unroll
      for (int k = 0; k < kFixBatch; ++k) {
        if (v0 + k >= L.num_var) break;
        const VarFieldDev& f = vf[v0 + k];
        int32_t p = -1;
        if (live) {
          uint8_t* slot = slots + 8 * f.slot;
          const int64_t nn = e1[k] - e0[k];
          if (!((vb[k] >> (ii & 7)) & 1)) {
            set_null_bit(row, f.slot);
            st64_lds(slot, 0);
          } else if (!f.is_list) {
            st64_lds(slot, ((uint64_t)wi << 32) | (uint32_t)nn);
            p = (int32_t)wi;
            wi += round8(nn);
          } else {  // LIST: [i64 n][null bitmap][n * w bytes, padded to 8]
            const int32_t ahdr = 8 + bitmap_bytes(nn);
            const int64_t size = ahdr + round8(nn * f.w);
            st64_lds(row + wi, (uint64_t)nn);
            for (int b = 8; b < ahdr; b += 4) st32(row + wi + b, 0);
            st64_lds(slot, ((uint64_t)wi << 32) | (uint32_t)size);
            p = (int32_t)wi;
            wi += size;
          }
        }
        pos[(v0 + k) * 64 + lane] = p;
      }
    }
    }
  }
  FLAT_STAMP(2);
  if constexpr (NEST) __syncthreads();  // nested fixed slots need the child-row offsets
  // fixed slots (all waves): BinaryRowWriter.write(ordinal, v), null -> 0
  {
    int jb[5];
    jb[0] = 0;
    for (int g = 0; g < 4; ++g) jb[g + 1] = jb[g] + (L.fix_group[g + 1] - L.fix_group[g] + kFixBatch - 1) / kFixBatch;
    flat_enc_fixed<8, NW, NEST>(L, fix, L.fix_group[0], L.fix_group[1], jb[0], jb[4], wave, lane, live, i, row, st, sbase);
    flat_enc_fixed<4, NW, NEST>(L, fix, L.fix_group[1], L.fix_group[2], jb[1], jb[4], wave, lane, live, i, row, st, sbase);
    flat_enc_fixed<2, NW, NEST>(L, fix, L.fix_group[2], L.fix_group[3], jb[2], jb[4], wave, lane, live, i, row, st, sbase);
    flat_enc_fixed<1, NW, NEST>(L, fix, L.fix_group[3], L.fix_group[4], jb[3], jb[4], wave, lane, live, i, row, st, sbase);
  }
  if (L.prof) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  FLAT_STAMP(3);
  __syncthreads();
  FLAT_STAMP(4);
  // variable payloads: one field per wave at a time, record group by record group
  for (int v = v_first, kv = 0; v < L.num_var; v += nplc, ++kv) {
    const VarFieldDev& f = vf[v];
    int64_t e0 = pf_e0, e1 = pf_e1;
    if (kv >= 1 && kv <= kPre) {
#pragma unroll
      for (int k = 0; k < kPre; ++k)
        if (kv == k + 1) e0 = pe0[k], e1 = pe1[k];
    } else if (kv > kPre || wave == 0) {
      const int64_t ee = *gp(f.offsets + r0 + rows);
      e0 = live ? *gp(f.offsets + i) : ee;
      e1 = live ? *gp(f.offsets + i + 1) : ee;
    }
    const int p = live ? pos[v * 64 + lane] : -1;
    for (int lo = 0; lo < rows;) {
      bool fits;
      int hi, phase = 0, vofs = 0;
      if (v == v_first && wave != 0 && lo == 0) {  // prefetched group
        hi = pf_hi;
        fits = pf_fits;
        phase = pf_phase;
        vofs = pf_vofs;
      } else {
        hi = flat_group(f, e0, e1, lo, rows, lane, stg_bytes, &fits);
        if (fits) {
          wave_lds_sync();  // staging reused
          flat_stage_span(f, __shfl(e0, lo), __shfl(e1, hi - 1), lane, stg, &phase, &vofs);
        }
      }
      if (fits) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wave_lds_sync();
      }
      const int64_t base = __shfl(e0, lo);  // (all lanes: no shuffle in divergent code)
      if (lane >= lo && lane < hi) flat_place(f, fits, stg, phase, base, vofs, p, e0, e1 - e0, row);
      lo = hi;
    }
  }
  if (L.prof) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  FLAT_STAMP(5);
  __syncthreads();
  FLAT_STAMP(6);
  uint8_t* g = out + B0 - mis;  // 16-byte aligned
  const int tot = (int)total;
  const int nch = (tot + 15) >> 4;
  for (int cc = tid; cc < nch; cc += 64 * NW) {
    const int lo = cc * 16;
    if (lo >= mis && lo + 16 <= tot) {
      *gp(reinterpret_cast<u32x4*>(g + lo)) = *reinterpret_cast<const u32x4*>(img + lo);
    } else {
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int o = lo + 4 * d;
        if (o >= mis && o + 4 <= tot) *gp(reinterpret_cast<uint32_t*>(g + o)) = ld32(img + o);
      }
    }
  }
  if (L.prof) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  FLAT_STAMP(7);
  };
  if (!SPILL) {
    body(var_tile(blockIdx.x, gridDim.x, L.kn.var_xcd));
    return;
  }
  const int64_t count = *sp.count;  // tiles the main launch spilled
  for (int64_t k = blockIdx.x; k < count; k += gridDim.x) {
    body(sp.list[k]);
    __syncthreads();
  }
}

#define FORY_VAR_ENC_PARAMS                                                                              \
  VarLaunch L, const Op* __restrict__ prog, const ColumnDev* __restrict__ cols,                          \
      const FixedFieldDev* __restrict__ fix, const VarFieldDev* __restrict__ vf,                         \
      const StructDev* __restrict__ st, const int64_t* __restrict__ offs, uint8_t* __restrict__ out,    \
      int64_t capacity, int32_t* status, int cap, SpillArgs sp
template <int HDR, int NW, bool NEST, bool SPILL>
__global__ __launch_bounds__(64 * NW) void var_encode_flat_kernel(FORY_VAR_ENC_PARAMS) {
  var_encode_flat_body<HDR, NW, NEST, SPILL>(L, prog, cols, fix, vf, st, offs, out, capacity, status, cap, sp);
}
template <int HDR, int NW, bool NEST, bool SPILL>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(5, 8))) void var_encode_flat_lean_kernel(
    FORY_VAR_ENC_PARAMS) {
  var_encode_flat_body<HDR, NW, NEST, SPILL>(L, prog, cols, fix, vf, st, offs, out, capacity, status, cap, sp);
}
#undef FORY_VAR_ENC_PARAMS

// ---------------------------------------------------------------------------
// Encode v7: flat plans (fixed fields, strings / binary, list<fixed>; no nested
// struct fields), one global round trip before the payload copies.
//
// The tile kernel above is latency-bound: its tile runs a chain of
// dependent global round trips (row bounds -> wave 0's layout loads -> fixed batches
// -> the var spans, field after field per wave) separated by barriers, ~16 us per
// Mixed tile at 4 tiles per CU. Here every wave issues ALL of its loads at once --
// the row bounds, the Arrow offsets and validity of the var fields it owns
// (v = wave + k*NW), its first fixed-field batch -- and right after they land it
// puts every owned field's tile span in flight (LDS-DMA into its staging slot).
// The layout needs no walk: each wave writes its fields' padded payload sizes and
// null bits to LDS tables, one barrier, and every wave derives its fields' positions
// (BinaryWriter.writeUnaligned appends in field order: the fixed part plus the sizes
// of the var fields before it) from the table. Chain per tile: bounds + columns ->
// spans (overlapping the slot fills) -> copies -> barrier -> 16-B stores.
// Bytes are those of var_encode_flat_kernel (BinaryRowWriter.java:76-84 reset,
// BinaryWriter.java:106-194 write/writeUnaligned, BinaryArrayWriter.java:93-118 reset).
// ---------------------------------------------------------------------------
constexpr int kOwnVar = 4;  // var fields a wave owns: plans with num_var <= kOwnVar * NW

// Fixed-field batch j: kFixBatch consecutive fields [k0, k1) of the width-sorted table
// (widths mixed; each field loads at its own width), so a plan with <= kFixBatch * NW
// fixed fields gives every wave at most one batch, loaded with the row bounds.
__device__ __forceinline__ bool fix_batch(const VarLaunch& L, int j, int* k0, int* k1) {
  const int nf = L.fix_group[4];
  *k0 = j * kFixBatch;
  *k1 = *k0 + kFixBatch < nf ? *k0 + kFixBatch : nf;
  return *k0 < nf;
}

// Fixed values through registers, loaded branch-free: every lane issues the same two
// dword loads whatever the field's width -- the element's dword(s): for w = 8 the two
// halves (any alignment), for w <= 4 the aligned dwords holding its first and last
// bytes (never past the page of a byte of the column). A switch over widths instead
// merges differently typed loads, and the compiler then waits for each load before
// the next (a round trip per field).
struct FixRegs {
  uint32_t lo[kFixBatch], hi[kFixBatch];
  uint32_t vb[kFixBatch];  // validity byte (fields without validity: any byte, unused)
};

__device__ __forceinline__ void elem_issue(const uint8_t* base, int w, int64_t i, uint32_t* lo, uint32_t* hi) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(base) + (uintptr_t)(i * w);
  const bool w8 = w == 8;
  const uintptr_t la = w8 ? a : a & ~uintptr_t(3);
  const uintptr_t ha = w8 ? a + 4 : (a + w - 1) & ~uintptr_t(3);
  *lo = *gp(reinterpret_cast<const uint32_t*>(la));
  *hi = *gp(reinterpret_cast<const uint32_t*>(ha));
}

__device__ __forceinline__ uint64_t elem_value(const uint8_t* base, int w, int64_t i, uint32_t lo, uint32_t hi) {
  const uint64_t d = ((uint64_t)hi << 32) | lo;
  if (w == 8) return d;
  const int sh = (int)((reinterpret_cast<uintptr_t>(base) + (uintptr_t)(i * w)) & 3) * 8;
  return (d >> sh) & ((1ull << (8 * w)) - 1);
}

// The batch's values and validity bytes of record ii, all loads issued together
// (`safe`: any readable byte, the address of fields without validity).
template <bool VB = true>
__device__ __forceinline__ void fix_load(const FixedFieldDev* __restrict__ fix, int k0, int k1, int64_t ii,
                                         FixRegs& R, const void* safe) {
#pragma unroll
  for (int k = 0; k < kFixBatch; ++k) {
    const FixedFieldDev& f = fix[min(k0 + k, k1 - 1)];
    elem_issue(f.values, f.width, ii, &R.lo[k], &R.hi[k]);
    if constexpr (VB) {
      const uint8_t* vp = f.validity ? f.validity + (ii >> 3) : reinterpret_cast<const uint8_t*>(safe);
      R.vb[k] = load_byte(vp);
    }
  }
}

// Software-pipeline fences (encode v9): ready(x) marks where loaded registers are first
// needed -- the compiler inserts its wait here and cannot hoist work on x above it --
// and sched_fence() keeps the scheduler from moving loads and work across a phase.
__device__ __forceinline__ void ready(uint32_t& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void ready(int32_t& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void ready(int64_t& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }


__device__ __forceinline__ bool fix_valid(const FixedFieldDev& f, const FixRegs& R, int k, int64_t ii) {
  return !f.validity || ((R.vb[k] >> (ii & 7)) & 1);
}

// BinaryRowWriter.write(ordinal, v) into the row image's slots (zero-extended; a null
// value writes 0 and sets its bit in the record's bitmap words, BinaryWriter.setNullAt).
__device__ __forceinline__ void fix_store(const FixedFieldDev* __restrict__ fix, int k0, int k1, const FixRegs& R,
                                          bool live, int64_t ii, uint8_t* slots, uint32_t* bmrow) {
#pragma unroll
  for (int k = 0; k < kFixBatch; ++k) {
    if (k0 + k >= k1 || !live) continue;
    const FixedFieldDev& f = fix[k0 + k];
    const bool valid = fix_valid(f, R, k, ii);
    uint64_t x = valid ? elem_value(f.values, f.width, ii, R.lo[k], R.hi[k]) : 0;
    if (f.flags & 2) x = x ? 1 : 0;
    st64_lds(slots + 8 * f.slot, x);
    if (!valid) atomicOr(bmrow + (f.slot >> 5), 1u << (f.slot & 31));
  }
}

// Strings / binary per lane through registers: 32 output bytes per chunk, from the
// kStrDw aligned source dwords that hold them at any alignment (each holds a byte of the
// string, so none lies past the column's end), all loads of a chunk issued together.
constexpr int kStrDw = 9;
struct StrRegs {
  uint32_t d[kStrDw];
};

__device__ __forceinline__ void str_load(const uint8_t* src, int64_t n, int c, StrRegs& S) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(src) + 32 * c;
  const int sb = (int)(a & 3);
  const uint32_t* p = reinterpret_cast<const uint32_t*>(a - sb);
  const int64_t left = n - 32 * c;
  const int nd = left <= 0 ? 0 : (int)((sb + (left < 32 ? left : 32) + 3) >> 2);
#pragma unroll
  for (int q = 0; q < kStrDw; ++q) S.d[q] = q < nd ? *gp(p + q) : 0u;
}

// str_load without per-lane branches (encode v9: every lane issues the same kStrDw
// loads, so the compiler can count them): dwords past the string's re-read its last one
// (an empty string reads `safe`); str_store masks the bytes past the string.
__device__ __forceinline__ void str_load_all(const uint8_t* src, int64_t n, int c, StrRegs& S, const void* safe) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(src) + 32 * c;
  const int sb = (int)(a & 3);
  const uint32_t* p = reinterpret_cast<const uint32_t*>(a - sb);
  const int64_t left = n - 32 * c;
  const int nd = left <= 0 ? 0 : (int)((sb + (left < 32 ? left : 32) + 3) >> 2);
#pragma unroll
  for (int q = 0; q < kStrDw; ++q) {
    const uint32_t* at = nd > 0 ? p + (q < nd ? q : nd - 1) : reinterpret_cast<const uint32_t*>(safe);
    S.d[q] = *gp(at);
  }
}

// Chunk c of writeUnaligned + zeroOutPaddingBytes (BinaryWriter.java:117-121,162-194):
// the string's bytes [32c, 32c + 32), zeros past n, the dwords inside round8(n), to the
// 4-byte aligned LDS image at dst.
__device__ __forceinline__ void str_store(uint8_t* dst, const uint8_t* src, int64_t n, int c, const StrRegs& S) {
  const int sb = (int)((reinterpret_cast<uintptr_t>(src) + 32 * c) & 3);
  const int64_t left = n - 32 * c;
  const int64_t outb = round8(n) - 32 * c;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    if (4 * q < outb) {
      uint32_t w = sb ? funnel(S.d[q], S.d[q + 1], sb) : S.d[q];
      const int64_t valid = left - 4 * q;
      if (valid <= 0) w = 0u;
      else if (valid < 4) w &= (1u << (8 * valid)) - 1u;
      st32(dst + 32 * c + 4 * q, w);
    }
  }
}

// List fields owned by wave w of nw (var field v belongs to wave v % nw): a bit mask.
__host__ __device__ __forceinline__ uint32_t flat7_wave_lists(uint32_t list_mask, int w, int nw) {
  uint32_t m = 0;
  for (int v = w; v < 32; v += nw) m |= list_mask & (1u << v);
  return m;
}

// NEST: plans with nested struct fields. A struct field's child row is reserved at the
// writerIndex its field is reached and its var fields follow (BinaryRowWriter(schema,
// parent), BaseBinaryEncoderBuilder.java:436-490), so positions are a prefix over the
// program's var fields and struct begins: after the size table, wave 0 walks the program
// once over LDS values only (no loads) into a position table, zeroes the bitmaps and
// writes the struct slots; every wave then writes its fields' slots and null bits into
// the image (null bits by LDS atomics: a bitmap is shared by the fields of its row).
// OWN: var fields per wave (2 or kOwnVar): registers for what the plan needs.
// Strings go lane by lane through registers (no staging LDS: the image alone sets the
// residency); lists (items + item validity) are staged per tile span by LDS-DMA.
template <int HDR, int NW, bool NEST, int OWN>
__global__ __launch_bounds__(64 * NW) void var_encode_flat7_kernel(VarLaunch L, const Op* __restrict__ prog,
                                                                   const ColumnDev* __restrict__ cols,
                                                                   const FixedFieldDev* __restrict__ fix,
                                                                   const VarFieldDev* __restrict__ vf,
                                                                   const StructDev* __restrict__ st,
                                                                   const int64_t* __restrict__ offs,
                                                                   uint8_t* __restrict__ out, int64_t capacity,
                                                                   int32_t* status, int cap, int slot, SpillArgs sp) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t* img = lds;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // list staging: one slot per wave that owns a list field, in wave order
  int sidx = 0, nslot = 0;
  for (int w = 0; w < NW; ++w) {
    const bool owns = (flat7_wave_lists(L.list_mask, w, NW)) != 0;
    sidx += owns && w < wave;
    nslot += owns;
  }
  uint8_t* stg = lds + cap + sidx * slot;                                      // this wave's list staging
  int32_t* sz = reinterpret_cast<int32_t*>(lds + cap + nslot * slot);          // [num_var][64] payload bytes
  uint32_t* bmt = reinterpret_cast<uint32_t*>(sz + L.num_var * 64);            // flat: [64][bmw] null bits
  int32_t* sbs = reinterpret_cast<int32_t*>(sz + L.num_var * 64);              // NEST: [1 + num_struct][64] child rows
  const int bmw = L.bitmap_bytes >> 2;
  const int64_t tile = var_tile(blockIdx.x, gridDim.x, L.kn.var_xcd);
  const int64_t r0 = tile * 64;
  const int rows = L.num_rows - r0 < 64 ? (int)(L.num_rows - r0) : 64;
  const bool lv = lane < rows;
  const int64_t i = r0 + lane;
  const int64_t ii = lv ? i : r0;
  // debug timeline (the plan's FORY_ROWFMT_VARPROF=1): thread 0 stamps s_memrealtime at
  // phase boundaries, waiting for its outstanding memory first (a uniform branch when off)
#define V7_STAMP(k)                                                                              \
  do {                                                                                          \
    if (L.prof) {                                                                               \
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                               \
      if (tid == 0) L.prof[tile * 8 + (k)] = __builtin_amdgcn_s_memrealtime();                  \
    }                                                                                           \
  } while (0)
  V7_STAMP(0);
  if constexpr (!NEST) {  // zeroed before any wave ORs a null bit into it (other waves' words included)
    for (int k = tid; k < 64 * bmw; k += 64 * NW) bmt[k] = 0u;
    __syncthreads();
  }
  // ---- one round trip: this wave's var fields (offsets, validity), its first fixed
  // batch, the struct validity (NEST) and the row bounds, all issued before any is used
  int32_t e0[OWN], e1[OWN];
  uint32_t vvb[OWN];
#pragma unroll
  for (int k = 0; k < OWN; ++k) {
    const int v = wave + k * NW;
    e0[k] = e1[k] = 0;
    vvb[k] = 0xffu;
    if (v < L.num_var) {
      const VarFieldDev& f = vf[v];
      e0[k] = *gp(f.offsets + (lv ? i : r0 + rows));  // dead lanes: the tile's end (empty ranges)
      e1[k] = *gp(f.offsets + (lv ? i + 1 : r0 + rows));
      vvb[k] = f.validity ? load_byte(f.validity + (ii >> 3)) : 0xffu;
    }
  }
  uint32_t svb[NEST ? kMaxTileStructs : 1];
  if constexpr (NEST) {
#pragma unroll
    for (int s = 0; s < kMaxTileStructs; ++s)
      svb[s] = s < L.num_struct && (st[s].flags & 1) && st[s].validity ? load_byte(st[s].validity + (ii >> 3)) : 0xffu;
  }
  int fk0 = 0, fk1 = 0;
  const bool has_fix = fix_batch(L, wave, &fk0, &fk1);
  FixRegs R;
  if (has_fix) fix_load(fix, fk0, fk1, ii, R, offs);
  int64_t B0, B1, beg, end;
  bool live;
  const bool sane = var_tile_bounds(offs, L.num_rows, r0, lane, &B0, &B1, &beg, &end, &live);
  // strings: the first 32 bytes of each owned field in flight now (they need only e0, e1)
  StrRegs S[OWN];
#pragma unroll
  for (int k = 0; k < OWN; ++k) {
    const int v = wave + k * NW;
    if (v < L.num_var && !vf[v].is_list) str_load(vf[v].values + e0[k], (int64_t)e1[k] - e0[k], 0, S[k]);
  }
  const bool capbad = live && (end > capacity || beg < 0 || end < beg);
  if (__ballot(capbad)) {  // (every wave sees the same bounds: the whole workgroup leaves)
    if (wave == 0 && capbad) set_status(status, FORY_ERR_CAPACITY);
    return;
  }
  const int mis = (int)(reinterpret_cast<uintptr_t>(out + B0) & 15);
  const int64_t total = mis + (B1 - B0);
  V7_STAMP(1);
  if (!sane || (mis & 3) || total > cap) {
    if (sane && !(mis & 3) && total <= sp.cap) {  // the big-image spill launch takes it
      if (tid == 0) sp.list[atomicAdd(sp.count, 1)] = (int32_t)tile;
      return;
    }
    if (wave == 0 && live) enc_record(L, prog, cols, r0 + lane, out + beg, end - beg);
    return;
  }
  uint8_t* fp = img + mis + (int)(beg - B0);
  uint8_t* row = fp + HDR;
  uint8_t* slots = row + L.bitmap_bytes;
  uint32_t* bmrow = bmt + lane * bmw;
  // NEST: structs present in this record (bit s: struct id s, bit 0 the row), pre-order
  uint32_t pm = 1;
  if constexpr (NEST) {
#pragma unroll
    for (int s = 0; s < kMaxTileStructs; ++s)
      if (s < L.num_struct && ((svb[s] >> (ii & 7)) & 1) && ((pm >> st[s].parent) & 1)) pm |= 1u << (s + 1);
  }
  // ---- owned var fields: payload sizes (-1 null, -2 under an absent struct), null bits
  // (flat), list tile spans in flight
  int so = 0;
  int sphase[OWN], svofs[OWN], soff[OWN];
  int32_t sbase[OWN];
  bool staged[OWN];
#pragma unroll
  for (int k = 0; k < OWN; ++k) {
    const int v = wave + k * NW;
    staged[k] = false;
    sphase[k] = svofs[k] = soff[k] = 0;
    sbase[k] = 0;
    if (v >= L.num_var) continue;
    const VarFieldDev& f = vf[v];
    const bool valid = (vvb[k] >> (ii & 7)) & 1;
    const bool absent = NEST && !((pm >> f.parent) & 1);
    const int64_t n = (int64_t)e1[k] - e0[k];
    const int32_t s = absent ? -2 : !valid ? -1 : (int32_t)(f.is_list ? 8 + bitmap_bytes(n) + round8(n * f.w) : round8(n));
    sz[v * 64 + lane] = live ? s : -2;
    if (!NEST && live && !valid) atomicOr(bmrow + (f.slot >> 5), 1u << (f.slot & 31));
    if (!f.is_list) continue;
    const int32_t E0 = __shfl(e0[k], 0), E1 = __shfl(e1[k], 63);  // lane 0 is live; lane 63's end is the tile's
    sbase[k] = E0;
    int64_t need = (int64_t)(E1 - E0) * f.w + 16 + 4 + 16;  // phase + funnel-copy slack + vofs rounding
    if (f.item_validity) need += ((E1 + 7) >> 3) - ((E0 >> 3) & ~3) + 4;
    need = (need + 15) & ~int64_t(15);
    if ((f.iflags & 2) == 0 && E1 > E0 && so + need <= slot) {  // bool items: per lane (0/1 normalised)
      flat_stage_span(f, E0, E1, lane, stg + so, &sphase[k], &svofs[k]);
      staged[k] = true;
      soff[k] = so;
      so += (int)need;
    }
  }
  if constexpr (!NEST) {  // fixed slots of the row: the preloaded batch, then the wave's further batches
    if (has_fix) fix_store(fix, fk0, fk1, R, live, ii, slots, bmrow);
    for (int j = wave + NW;; j += NW) {
      int a, b;
      if (!fix_batch(L, j, &a, &b)) break;
      FixRegs Q;
      fix_load(fix, a, b, ii, Q, offs);
      fix_store(fix, a, b, Q, live, ii, slots, bmrow);
    }
  }
  if (L.prof && tid == 0) L.prof[tile * 8 + 2] = __builtin_amdgcn_s_memrealtime();  // (spans in flight)
  __syncthreads();  // every field's payload size (flat: and null bits)
  if (L.prof && tid == 0) L.prof[tile * 8 + 3] = __builtin_amdgcn_s_memrealtime();
  if (wave == 0 && live) {  // Encoders.encode frame header; the bitmap (BinaryRowWriter.reset + setNullAt)
    if (HDR == 12) {
      st32(fp, (uint32_t)(end - beg - 4));
      st64_lds(fp + 4, (uint64_t)L.schema_hash);
    } else if (HDR == 8) {
      st64_lds(fp, (uint64_t)L.schema_hash);
    }
    if constexpr (!NEST) {
      for (int b = 0; b < bmw; ++b) st32(row + 4 * b, bmrow[b]);
    } else {
      for (int b = 0; b < bmw; ++b) st32(row + 4 * b, 0u);
    }
  }
  int32_t pos[OWN];
  if constexpr (!NEST) {  // positions: the fixed part + the payloads of the var fields before it (field order)
    int32_t acc = L.fixed_size;
    int u = 0;
#pragma unroll
    for (int k = 0; k < OWN; ++k) {
      const int v = wave + k * NW;
      pos[k] = -1;
      if (v >= L.num_var) continue;
      for (; u < v; ++u) {
        const int32_t s = sz[u * 64 + lane];
        acc += s > 0 ? s : 0;
      }
      pos[k] = live && sz[v * 64 + lane] >= 0 ? acc : -1;
    }
  } else {
    // wave 0: one walk of the program over the size table -> positions (in place of the
    // sizes: -1 null, -2 absent), child-row starts, zeroed child bitmaps, struct slots
    // ((offset from the parent row) << 32 | size) and null structs' bits
    if (wave == 0) {
      int32_t acc = L.fixed_size;
      int cur = 0, vi = 0, si = 0;
      sbs[lane] = 0;
      for (int pc = 0; pc < L.num_ops; ++pc) {
        const Op op = prog[pc];
        if (op.code == OP_BYTES || op.code == OP_LIST) {
          const int32_t s = sz[vi * 64 + lane];
          sz[vi * 64 + lane] = s >= 0 ? acc : s;
          acc += s > 0 ? s : 0;
          ++vi;
        } else if (op.code == OP_STRUCT_BEGIN) {
          ++si;
          cur = si;
          const StructDev& sd = st[si - 1];
          int32_t b = -1;
          if (live && ((pm >> si) & 1)) {
            b = acc;
            for (int q = 0; q < sd.hdr; q += 4) st32(row + b + q, 0u);
            acc += sd.hdr + 8 * sd.nfields;
          }
          sbs[si * 64 + lane] = b;
        } else if (op.code == OP_STRUCT_END) {
          cur = __builtin_amdgcn_readfirstlane(cur);  // uniform by construction
          const StructDev& sd = st[cur - 1];
          const int par = sd.parent;
          const int32_t pb = sbs[par * 64 + lane];
          if (live && pb >= 0) {
            const int32_t ph = par ? st[par - 1].hdr : L.bitmap_bytes;
            const int32_t b = sbs[cur * 64 + lane];
            uint8_t* sl = row + pb + ph + 8 * sd.slot;
            if (b >= 0) {
              st64_lds(sl, ((uint64_t)(uint32_t)(b - pb) << 32) | (uint32_t)(acc - b));
            } else {  // a null struct (its parent is present): setNullAt
              st64_lds(sl, 0);
              set_null_bit(row + pb, sd.slot);
            }
          }
          cur = par;
        }
      }
    }
    __syncthreads();  // positions, child rows, zeroed bitmaps
#pragma unroll
    for (int k = 0; k < OWN; ++k) {
      const int v = wave + k * NW;
      pos[k] = v < L.num_var ? sz[v * 64 + lane] : -2;
    }
    // fixed fields at their row / child row: value or 0 + null bit (absent: nothing)
    auto put_fixed = [&](int a, int b, const FixRegs& Q) {
#pragma unroll
      for (int k = 0; k < kFixBatch; ++k) {
        if (a + k >= b || !live) continue;
        const FixedFieldDev& f = fix[a + k];
        const int32_t base = sbs[f.parent * 64 + lane];
        if (base < 0) continue;
        const int32_t hdr = f.parent ? st[f.parent - 1].hdr : L.bitmap_bytes;
        const bool valid = fix_valid(f, Q, k, ii);
        uint64_t x = valid ? elem_value(f.values, f.width, ii, Q.lo[k], Q.hi[k]) : 0;
        if (f.flags & 2) x = x ? 1 : 0;
        st64_lds(row + base + hdr + 8 * f.slot, x);
        if (!valid) atomicOr(reinterpret_cast<uint32_t*>(row + base) + (f.slot >> 5), 1u << (f.slot & 31));
      }
    };
    if (has_fix) put_fixed(fk0, fk1, R);
    for (int j = wave + NW;; j += NW) {
      int a, b;
      if (!fix_batch(L, j, &a, &b)) break;
      FixRegs Q;
      fix_load(fix, a, b, ii, Q, offs);
      put_fixed(a, b, Q);
    }
  }
  // var slots (offset << 32 | size), list headers (BinaryArrayWriter.reset(n): [i64 n][zero
  // bitmap]) and the strings' first chunks (already in registers)
#pragma unroll
  for (int k = 0; k < OWN; ++k) {
    const int v = wave + k * NW;
    if (v >= L.num_var || !live) continue;
    const VarFieldDev& f = vf[v];
    int32_t base = 0, hdr = L.bitmap_bytes;
    if constexpr (NEST) {
      if (pos[k] == -2) continue;  // under an absent struct
      base = sbs[f.parent * 64 + lane];
      if (f.parent) hdr = st[f.parent - 1].hdr;
    }
    uint8_t* sl = row + base + hdr + 8 * f.slot;
    const int64_t n = (int64_t)e1[k] - e0[k];
    if (pos[k] < 0) {
      st64_lds(sl, 0);
      if (NEST) atomicOr(reinterpret_cast<uint32_t*>(row + base) + (f.slot >> 5), 1u << (f.slot & 31));
    } else if (!f.is_list) {
      st64_lds(sl, ((uint64_t)(uint32_t)(pos[k] - base) << 32) | (uint32_t)n);
      str_store(row + pos[k], f.values + e0[k], n, 0, S[k]);
    } else {
      const int32_t ahdr = 8 + bitmap_bytes(n);
      st64_lds(row + pos[k], (uint64_t)n);
      for (int b = 8; b < ahdr; b += 4) st32(row + pos[k] + b, 0);
      st64_lds(sl, ((uint64_t)(uint32_t)(pos[k] - base) << 32) | (uint32_t)(ahdr + round8(n * f.w)));
    }
  }
  // strings longer than 32 bytes: their further chunks (a round trip each)
#pragma unroll
  for (int k = 0; k < OWN; ++k) {
    const int v = wave + k * NW;
    if (v >= L.num_var || vf[v].is_list) continue;
    const int64_t n = live && pos[k] >= 0 ? (int64_t)e1[k] - e0[k] : 0;
    const int nc = (int)((n + 31) >> 5);
    for (int c = 1; __ballot(c < nc); ++c) {
      StrRegs T;
      str_load(vf[v].values + e0[k], c < nc ? n : 0, c, T);
      if (c < nc) str_store(row + pos[k], vf[v].values + e0[k], n, c, T);
    }
  }
  if (L.prof && tid == 0) L.prof[tile * 8 + 4] = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's list spans
  wave_lds_sync();
  if (L.prof && tid == 0) L.prof[tile * 8 + 5] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
  for (int k = 0; k < OWN; ++k) {
    const int v = wave + k * NW;
    if (v >= L.num_var || !vf[v].is_list) continue;
    if (live && pos[k] >= 0)
      flat_place(vf[v], staged[k], stg + soff[k], sphase[k], sbase[k], svofs[k], pos[k], e0[k],
                 (int64_t)e1[k] - e0[k], row);
  }
  __syncthreads();
  V7_STAMP(6);
  uint8_t* g = out + B0 - mis;  // 16-byte aligned
  const int tot = (int)total;
  const int nch = (tot + 15) >> 4;
  for (int cc = tid; cc < nch; cc += 64 * NW) {
    const int lo = cc * 16;
    if (lo >= mis && lo + 16 <= tot) {
      *gp(reinterpret_cast<u32x4*>(g + lo)) = *reinterpret_cast<const u32x4*>(img + lo);
    } else {
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int o = lo + 4 * d;
        if (o >= mis && o + 4 <= tot) *gp(reinterpret_cast<uint32_t*>(g + o)) = ld32(img + o);
      }
    }
  }
  V7_STAMP(7);
#undef V7_STAMP
}

// ---------------------------------------------------------------------------
// Encode v9: encode v7's tile, two consecutive tiles per workgroup as straight-line code
// (flat plans of fixed fields and strings / binary: no list or nested struct fields,
// <= kFixBatch * NW fixed fields, <= OWN * NW var fields, a bitmap of <= kV9Bmw words).
//
// v7 spends a tile's whole life (~16 us at 4 tiles per CU) on a chain of dependent
// round trips -- row bounds and offsets -> string bytes -> copies -> stores -- so each
// CU has a tile's loads in flight only part of the time. Here workgroup b takes tiles
// tb = K b .. tb + K - 1 (K = 2) and issues the second tile's loads while the first is
// assembled (no loop: at a loop back edge LLVM flushes vmcnt):
//   --  tile tb: offsets, validity, row bounds, fixed values; then its strings' first
//       32 bytes (once its offsets land); then tile tb + 1's columns -- all in flight
//   P1  sizes, null bits (partial words per wave) and row starts of tile t -> LDS
//   B1  barrier
//   P2  the records' sizes against their offsets; wave 0: header + bitmap; every wave:
//       its fields' positions (prefix of sizes)
//   P3  fixed values and the strings' first 32 bytes into the image; longer strings: a
//       round trip per further 32 bytes
//   --  tile t + 1: its strings' first 32 bytes in flight (its offsets have landed)
//   B2  barrier; the image leaves as 16-B stores
// Every wait is on loads issued a phase or more earlier. Bytes are those of
// var_encode_flat7_kernel.
// ---------------------------------------------------------------------------
constexpr int kV9Bmw = 4;  // bitmap words per row (<= 128 fields)

template <int OWN>
struct V9Cols {            // one tile's per-lane column registers
  int32_t e0[OWN], e1[OWN];
  uint32_t vvb[OWN];       // owned var fields: the dword holding the record's validity byte (NUL & 2)
  uint32_t fvb[kFixBatch]; // the wave's fixed batch: the same (NUL & 1)
  int64_t beg, end;        // the record's row bounds
};

#define FORY_V9_PARAMS                                                                                   \
  VarLaunch L, const Op* __restrict__ prog, const ColumnDev* __restrict__ cols,                          \
      const FixedFieldDev* __restrict__ fix, const VarFieldDev* __restrict__ vf,                         \
      const int64_t* __restrict__ offs, uint8_t* __restrict__ out, int64_t capacity, int32_t* status, int cap, \
      SpillArgs sp

template <int HDR, int NW, int OWN, int K, int NUL>
__device__ __forceinline__ void var_encode_flat9_body(FORY_V9_PARAMS) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t* img = lds;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int32_t* sz = reinterpret_cast<int32_t*>(lds + cap);                 // [num_var][64] payload bytes
  uint32_t* pbt = reinterpret_cast<uint32_t*>(sz + L.num_var * 64);     // [NW][64][bmw] partial null bits
  const int bmw = L.bitmap_bytes >> 2;
  uint32_t* tbad = pbt + NW * 64 * bmw;  // [2] by tile parity: a record's size disagrees with its offsets
  const int64_t ntiles = (L.num_rows + 63) / 64;
  int fk0 = 0, fk1 = 0;
  const bool has_fix = fix_batch(L, wave, &fk0, &fk1);
  // the fields whose words the loads read (a wave without a batch: the last field's, unused)
  const int fa = has_fix ? fk0 : L.fix_group[4] - 1, fb = has_fix ? fk1 : fa + 1;

  // tile tl's offsets, validity bytes and row bounds (tiles past the end: the last one);
  // branch-free (fields past num_var load field num_var - 1's words, unused): see FixRegs
  auto load_cols = [&](int64_t tl, V9Cols<OWN>& C) {
    tl = tl < ntiles ? tl : ntiles - 1;  // (past the end: the last tile, unused)
    const int64_t q0 = tl * 64;
    const int rw = L.num_rows - q0 < 64 ? (int)(L.num_rows - q0) : 64;
    const bool lq = lane < rw;
    const int64_t iq = lq ? q0 + lane : q0;
#pragma unroll
    for (int k = 0; k < OWN; ++k) {
      const int v = wave + k * NW < L.num_var ? wave + k * NW : L.num_var - 1;
      const VarFieldDev& f = vf[v];
      C.e0[k] = *gp(f.offsets + (lq ? iq : q0 + rw));  // dead lanes: the tile's end (empty ranges)
      C.e1[k] = *gp(f.offsets + (lq ? iq + 1 : q0 + rw));
      if constexpr ((NUL & 2) != 0)
        C.vvb[k] = vbyte_issue(f.validity ? f.validity + (iq >> 3) : reinterpret_cast<const uint8_t*>(offs));
    }
    if constexpr ((NUL & 1) != 0) {
#pragma unroll
      for (int k = 0; k < kFixBatch; ++k) {
        const FixedFieldDev& f = fix[min(fa + k, fb - 1)];
        C.fvb[k] = vbyte_issue(f.validity ? f.validity + (iq >> 3) : reinterpret_cast<const uint8_t*>(offs));
      }
    }
    C.beg = offs[iq];
    C.end = offs[lq ? iq + 1 : q0];
  };
  auto load_fixed = [&](int64_t tl, FixRegs& F) {
    tl = tl < ntiles ? tl : ntiles - 1;
    const int64_t q0 = tl * 64;
    const int64_t iq = q0 + lane < L.num_rows ? q0 + lane : q0;
    fix_load<false>(fix, fa, fb, iq, F, offs);
  };
  auto load_strs = [&](const V9Cols<OWN>& C, StrRegs (&S)[OWN]) {
#pragma unroll
    for (int k = 0; k < OWN; ++k) {
      const int v = wave + k * NW < L.num_var ? wave + k * NW : L.num_var - 1;
      str_load_all(vf[v].values + C.e0[k], (int64_t)C.e1[k] - C.e0[k], 0, S[k], offs);
    }
  };

  const int64_t tb = (int64_t)blockIdx.x * K;  // this workgroup's tiles tb .. tb + K - 1
  if (tb >= ntiles) return;
  V9Cols<OWN> C[K];
  FixRegs F[K];
  StrRegs S[OWN];
  auto ready_cols = [&](V9Cols<OWN>& C) {
#pragma unroll
    for (int k = 0; k < OWN; ++k) {
      ready(C.e0[k]);
      ready(C.e1[k]);
      if constexpr ((NUL & 2) != 0) ready(C.vvb[k]);
    }
    if constexpr ((NUL & 1) != 0) {
#pragma unroll
      for (int k = 0; k < kFixBatch; ++k) ready(C.fvb[k]);
    }
    ready(C.beg);
    ready(C.end);
  };
  auto ready_vals = [&](FixRegs& R) {
#pragma unroll
    for (int k = 0; k < kFixBatch; ++k) {
      ready(R.lo[k]);
      ready(R.hi[k]);
    }
#pragma unroll
    for (int k = 0; k < OWN; ++k)
#pragma unroll
      for (int q = 0; q < kStrDw; ++q) ready(S[k].d[q]);
  };
  load_cols(tb, C[0]);
  load_fixed(tb, F[0]);
  sched_fence();
  ready_cols(C[0]);
  load_strs(C[0], S);
  sched_fence();
#pragma unroll
  for (int j = 1; j < K; ++j) {
    load_cols(tb + j, C[j]);
    load_fixed(tb + j, F[j]);
  }
  sched_fence();
#define V9_STAMP(k)                                                                             \
  do {                                                                                         \
    if (L.prof && tid == 0) L.prof[t * 8 + (k)] = __builtin_amdgcn_s_memrealtime();            \
  } while (0)
  // tile t from its column registers C0 / FV and the strings' registers; then (more) the
  // next tile's strings in flight from C1
  auto step = [&](int64_t t, V9Cols<OWN>& C0, FixRegs& FV, V9Cols<OWN>& C1, bool more) {
    sched_fence();
    ready_cols(C0);
    V9_STAMP(0);
    const int64_t r0 = t * 64;
    const int rows = L.num_rows - r0 < 64 ? (int)(L.num_rows - r0) : 64;
    const bool live = lane < rows;
    const int64_t ii = live ? r0 + lane : r0;
    // ---- P1: bounds checks (uniform over the workgroup: every wave sees the same rows)
    const int64_t B0 = __shfl(C0.beg, 0), B1 = __shfl(C0.end, rows - 1);
    const bool ok = !live || (C0.beg >= B0 && C0.end >= C0.beg && C0.end <= B1);
    const bool sane = __ballot(!ok) == 0 && ((B0 | B1) & 3) == 0 && B1 >= B0;
    const bool capbad = live && (C0.end > capacity || C0.beg < 0 || C0.end < C0.beg);
    const bool skip = __ballot(capbad) != 0;
    if (skip && wave == 0 && capbad) set_status(status, FORY_ERR_CAPACITY);
    const int mis = (int)(reinterpret_cast<uintptr_t>(out + B0) & 15);
    const int64_t total = mis + (B1 - B0);
    const bool tiled = !skip && sane && !(mis & 3) && total <= cap;
    uint8_t* fp = img + mis + (int)(C0.beg - B0);
    uint8_t* row = fp + HDR;
    uint8_t* slots = row + L.bitmap_bytes;
    if (tiled) {  // sizes (-1 null, -2 dead lane) and this wave's null bits of the record
      uint64_t pl = 0, ph = 0;  // this wave's null bits of the record (no indexed array: registers)
      auto null_bit = [&](int slot) {
        const uint64_t bit = 1ull << (slot & 63);
        if (slot < 64) pl |= bit;
        else ph |= bit;
      };
#pragma unroll
      for (int k = 0; k < OWN; ++k) {
        const int v = wave + k * NW;
        if (v >= L.num_var) continue;
        const bool valid =
            (NUL & 2) == 0 || !vf[v].validity || ((vbyte_get(C0.vvb[k], vf[v].validity + (ii >> 3)) >> (ii & 7)) & 1);
        const int64_t n = (int64_t)C0.e1[k] - C0.e0[k];
        sz[v * 64 + lane] = !live ? -2 : !valid ? -1 : (int32_t)round8(n);
        if (live && !valid) null_bit(vf[v].slot);
      }
#pragma unroll
      for (int k = 0; k < kFixBatch; ++k)
        if ((NUL & 1) && fk0 + k < fk1 && live && fix[fk0 + k].validity &&
            !((vbyte_get(C0.fvb[k], fix[fk0 + k].validity + (ii >> 3)) >> (ii & 7)) & 1))
          null_bit(fix[fk0 + k].slot);
      if (tid == 0) tbad[t & 1] = 0u;  // (last read by tile t - 2's store, two barriers ago)
      uint32_t* pw = pbt + (wave * 64 + lane) * bmw;
      pw[0] = (uint32_t)pl;
      if (bmw > 1) pw[1] = (uint32_t)(pl >> 32);
      if (bmw > 2) pw[2] = (uint32_t)ph;
      if (bmw > 3) pw[3] = (uint32_t)(ph >> 32);
    }
    V9_STAMP(1);
    __syncthreads();  // B1
    V9_STAMP(2);
    if (tiled) {
      // ---- P2: the record's size against its offsets (columns changed since encoded_size:
      // its bytes would overrun its row -- nothing of it is written, the tile is not stored,
      // FORY_ERR_ENCODER), header and bitmap (wave 0), positions
      int32_t need = HDR + L.fixed_size;
      for (int u = 0; u < L.num_var; ++u) {
        const int32_t su = sz[u * 64 + lane];
        need += su > 0 ? su : 0;
      }
      const bool wr = live && need == C0.end - C0.beg;  // this lane writes its record
      if (live && !wr) {
        tbad[t & 1] = 1u;
        set_status(status, FORY_ERR_ENCODER);
      }
      if (wave == 0 && wr) {  // Encoders.encode frame header; BinaryRowWriter.reset + setNullAt
        if (HDR == 12) {
          st32(fp, (uint32_t)(C0.end - C0.beg - 4));
          st64_lds(fp + 4, (uint64_t)L.schema_hash);
        } else if (HDR == 8) {
          st64_lds(fp, (uint64_t)L.schema_hash);
        }
        for (int b = 0; b < bmw; ++b) {
          uint32_t w = 0;
          for (int q = 0; q < NW; ++q) w |= pbt[(q * 64 + lane) * bmw + b];
          st32(row + 4 * b, w);
        }
      }
      int32_t pos[OWN];
      {
        int32_t acc = L.fixed_size;
        int u = 0;
#pragma unroll
        for (int k = 0; k < OWN; ++k) {
          const int v = wave + k * NW;
          pos[k] = -1;
          if (v >= L.num_var) continue;
          for (; u < v; ++u) {
            const int32_t s = sz[u * 64 + lane];
            acc += s > 0 ? s : 0;
          }
          pos[k] = wr && sz[v * 64 + lane] >= 0 ? acc : -1;
        }
      }
      // ---- P3: fixed slots (BinaryRowWriter.write: zero-extended; null -> 0)
      sched_fence();
      ready_vals(FV);
      if (has_fix && wr) {
#pragma unroll
        for (int k = 0; k < kFixBatch; ++k) {
          if (fk0 + k >= fk1) continue;
          const FixedFieldDev& f = fix[fk0 + k];
          const bool valid =
              (NUL & 1) == 0 || !f.validity || ((vbyte_get(C0.fvb[k], f.validity + (ii >> 3)) >> (ii & 7)) & 1);
          uint64_t x = valid ? elem_value(f.values, f.width, ii, FV.lo[k], FV.hi[k]) : 0;
          if (f.flags & 2) x = x ? 1 : 0;
          st64_lds(slots + 8 * f.slot, x);
        }
      }
      // var slots (offset << 32 | size) and the strings' first chunks
#pragma unroll
      for (int k = 0; k < OWN; ++k) {
        const int v = wave + k * NW;
        if (v >= L.num_var || !wr) continue;
        const VarFieldDev& f = vf[v];
        uint8_t* sl = slots + 8 * f.slot;
        const int64_t n = (int64_t)C0.e1[k] - C0.e0[k];
        if (pos[k] < 0) {
          st64_lds(sl, 0);
        } else {
          st64_lds(sl, ((uint64_t)(uint32_t)pos[k] << 32) | (uint32_t)n);
          str_store(row + pos[k], f.values + C0.e0[k], n, 0, S[k]);
        }
      }
      // strings longer than 32 bytes: their further chunks (a round trip each)
#pragma unroll
      for (int k = 0; k < OWN; ++k) {
        const int v = wave + k * NW;
        if (v >= L.num_var) continue;
        const int64_t n = live && pos[k] >= 0 ? (int64_t)C0.e1[k] - C0.e0[k] : 0;
        const int nc = (int)((n + 31) >> 5);
        for (int c = 1; __ballot(c < nc); ++c) {
          StrRegs T;
          str_load(vf[v].values + C0.e0[k], c < nc ? n : 0, c, T);
          if (c < nc) str_store(row + pos[k], vf[v].values + C0.e0[k], n, c, T);
        }
      }
    } else if (!skip && tid == 0) {  // unaligned or big tile: the spill launch (which takes tiles
      sp.list[atomicAdd(sp.count, 1)] = (int32_t)t;  // beyond its own image per record)
    }
    V9_STAMP(3);
    sched_fence();
    if (more) {  // the next tile: its strings' first 32 bytes
      ready_cols(C1);
      load_strs(C1, S);
    }
    sched_fence();
    V9_STAMP(4);
    __syncthreads();  // B2: the image is complete
    V9_STAMP(5);
    if (tiled && !tbad[t & 1]) {  // (a record whose size disagrees with its offsets: not stored)
      uint8_t* g = out + B0 - mis;  // 16-byte aligned
      const int tot = (int)total;
      const int nch = (tot + 15) >> 4;
      for (int cc = tid; cc < nch; cc += 64 * NW) {
        const int lo = cc * 16;
        if (lo >= mis && lo + 16 <= tot) {
          *gp(reinterpret_cast<u32x4*>(g + lo)) = *reinterpret_cast<const u32x4*>(img + lo);
        } else {
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            const int o = lo + 4 * d;
            if (o >= mis && o + 4 <= tot) *gp(reinterpret_cast<uint32_t*>(g + o)) = ld32(img + o);
          }
        }
      }
    }
    V9_STAMP(6);
  };
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (tb + j < ntiles) step(tb + j, C[j], F[j], C[j + 1 < K ? j + 1 : j], j + 1 < K);  // (past the end: clamped)
#undef V9_STAMP
}

template <int HDR, int NW, int OWN, int K, int NUL>
__global__ __launch_bounds__(64 * NW) void var_encode_flat9_kernel(FORY_V9_PARAMS) {
  var_encode_flat9_body<HDR, NW, OWN, K, NUL>(L, prog, cols, fix, vf, offs, out, capacity, status, cap, sp);
}

__device__ __forceinline__ int64_t wave_incl_scan64(int64_t x, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  return x;
}

__device__ __forceinline__ int64_t wave_sum64(int64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
  return x;
}

// Tile prefixes -> Arrow offsets at tile starts: out_offsets[64 t] for every
// tile t and out_offsets[n] (= total) of each flat var field; the values pass
// fills the records in between (tile base + in-wave prefix).
__global__ __launch_bounds__(kWG) void flat_tile_bases_kernel(const VarFieldDev* __restrict__ vf, int num_var,
                                                              const int64_t* __restrict__ tile_tot, int64_t n,
                                                              int32_t* status) {
  const int64_t tiles = (n + 63) / 64;
  const int64_t k = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (k >= num_var * (tiles + 1)) return;
  const int v = (int)(k / (tiles + 1));
  const int64_t t = k - v * (tiles + 1);
  const int64_t off = tile_tot[k];
  if (off > 0x7fffffffLL) set_status(status, FORY_ERR_CAPACITY);  // int32 Arrow offsets
  vf[v].out_offsets[t == tiles ? n : t * 64] = (int32_t)off;
}

// Start and null-bitmap bytes of the row or child row holding a field of
// struct `parent` (0 = the row; sbase: child-row offsets, -1 = absent).
__device__ __forceinline__ int32_t field_base(const VarLaunch& L, const StructDev* __restrict__ st, int parent,
                                              const int32_t* sbase, int lane, int32_t* hdr) {
  if (!parent) {
    *hdr = L.bitmap_bytes;
    return 0;
  }
  *hdr = st[parent - 1].hdr;
  return sbase[parent * 64 + lane];
}

// Reads a var field's slot of a staged record: returns payload (rel from the
// row start, n) with n = bytes (STRING/BINARY) or elements (LIST); n = 0 when
// null/absent/corrupt. Returns true when null or absent.
__device__ __forceinline__ bool flat_var_slot(const VarLaunch& L, const VarFieldDev& f, const StructDev* __restrict__ st,
                                              const int32_t* sbase, int lane, const uint8_t* row,
                                              int64_t row_len, int64_t* rel, int64_t* n, bool report,
                                              int32_t* status) {
  *rel = 0;
  *n = 0;
  int32_t hdr;
  const int32_t base = field_base(L, st, f.parent, sbase, lane, &hdr);
  if (base < 0) return true;  // inside a null struct
  if ((row[base + (f.slot >> 3)] >> (f.slot & 7)) & 1) return true;  // BinaryRow.isNullAt
  const uint8_t* sp = row + base + hdr + 8 * f.slot;
  const uint64_t os = ld32(sp) | ((uint64_t)ld32(sp + 4) << 32);
  const int64_t r = base + (int64_t)(int32_t)(os >> 32);  // offsets are relative to the enclosing row
  if ((int32_t)(os >> 32) < 0) {
    if (report) set_status(status, FORY_ERR_CORRUPT);
    return false;
  }
  if (!f.is_list) {
    const int64_t len = (int32_t)(uint32_t)os;
    if (len < 0 || r + len > row_len) {
      if (report) set_status(status, FORY_ERR_CORRUPT);
      return false;
    }
    *rel = r;
    *n = len;
    return false;
  }
  if (r + 8 > row_len) {
    if (report) set_status(status, FORY_ERR_CORRUPT);
    return false;
  }
  const int64_t cnt = (int32_t)ld32(row + r);  // BinaryArray.pointTo: numElements
  if (cnt < 0 || r + 8 + bitmap_bytes(cnt) + cnt * f.w > row_len) {
    if (report) set_status(status, FORY_ERR_CORRUPT);
    return false;
  }
  *rel = r;
  *n = cnt;
  return false;
}

// Fixed fields of width W: slot (LDS) -> column, validity by ballot. Batches of
// kDecBatch fields numbered across the width groups from j0; batch j belongs to wave
// (j + num_var) % NW: the round robin starts after the waves that hold one var field
// more than the others (v = wave + k NW), so every wave gets about the same number of
// fields (it was per group from wave 0: Mixed's 32 fixed fields went 16 / 11 / 5 / 0).
constexpr int kDecBatch = 4;
template <int W, int NW>
__device__ __forceinline__ void flat_dec_fixed(const VarLaunch& L, const FixedFieldDev* __restrict__ fix, int g0, int g1,
                                               int j0, int wave, int lane, bool live,
                                               bool bad, int64_t i, int64_t r0, int rows, const uint8_t* row,
                                               const StructDev* __restrict__ st, const int32_t* sbase) {
  for (int k0 = g0, j = j0; k0 < g1; k0 += kDecBatch, ++j) {
    if ((j + L.num_var) % NW != wave) continue;
#pragma unroll
    for (int k = 0; k < kDecBatch; ++k) {
      if (k0 + k < g1) {
        const FixedFieldDev& f = fix[k0 + k];
        int32_t hdr;
        const int32_t base = field_base(L, st, f.parent, sbase, lane, &hdr);
        const bool nul = bad || base < 0 || ((row[base + (f.slot >> 3)] >> (f.slot & 7)) & 1);
        const uint8_t* sp = row + (base < 0 ? 0 : base) + hdr + 8 * f.slot;
        uint64_t x = 0;
        if (!nul) x = (uint64_t)ld32(sp) | ((uint64_t)ld32(sp + 4) << 32);
        if (f.flags & 2) x = (x & 0xff) ? 1 : 0;
        if (f.out_validity) {
          const uint64_t m = __ballot(live && !nul);
          if (lane == 0) write_validity64(f.out_validity, r0, rows, m);
        }
        if (live) stw<W>(f.out_values, i, x);
      }
    }
  }
}

// Frame header of a staged record (HDR 12: Encoders.decode(MemoryBuffer) reads the
// size then the hash, Encoders.java:177-193; HDR 8: decode(byte[]), the hash only,
// :195-197). False (and the status word set when `report`) on a mismatch.
template <int HDR>
__device__ __forceinline__ bool frame_ok(const VarLaunch& L, const uint8_t* fp, int64_t frame_len, bool report,
                                         int32_t* status) {
  const int ho = HDR == 12 ? 4 : 0;
  const uint64_t h = (uint64_t)ld32(fp + ho) | ((uint64_t)ld32(fp + ho + 4) << 32);
  if (h != (uint64_t)L.schema_hash) {
    if (report) set_status(status, FORY_ERR_SCHEMA_MISMATCH);
    return false;
  }
  const bool size_ok = HDR == 12 ? ((int64_t)ld32(fp) + 4 == frame_len && ld32(fp) >= (uint32_t)(8 + L.fixed_size))
                                 : frame_len >= 8 + L.fixed_size;
  if (!size_ok && report) set_status(status, FORY_ERR_CORRUPT);
  return size_ok;
}

// Arrow item validity of a list field's staged span [O0, O1) (1 = valid item),
// assembled in LDS words bw (BinaryArray.isNullAt of each item, a bitmap byte at a
// time) and stored; words shared with a neighbouring tile touch only this span's bits.
__device__ __forceinline__ void dec_item_validity(const VarFieldDev& f, int64_t O0, int64_t O1, int64_t e0, int64_t n,
                                                  const uint8_t* abm, bool live, int lane, uint32_t* bw) {
  const int64_t W0 = O0 >> 5;
  const int nwd = O1 > O0 ? (int)(((O1 - 1) >> 5) - W0 + 1) : 0;
  for (int k = lane; k < nwd; k += 64) bw[k] = 0;
  wave_lds_sync();
  if (live && n > 0) {  // a bitmap byte (8 items) per step, at most two words each
    for (int64_t j = 0; j < n; j += 8) {
      const int take = n - j < 8 ? (int)(n - j) : 8;
      const uint32_t vbits = ~(uint32_t)abm[j >> 3] & ((1u << take) - 1u);  // 1 = valid item
      if (!vbits) continue;
      const int64_t q = e0 + j;
      const int sh = (int)(q & 31);
      atomicOr(&bw[(q >> 5) - W0], vbits << sh);
      if (sh + take > 32 && (vbits >> (32 - sh))) atomicOr(&bw[(q >> 5) - W0 + 1], vbits >> (32 - sh));
    }
  }
  wave_lds_sync();
  uint32_t* gv = reinterpret_cast<uint32_t*>(f.out_item_validity) + W0;
  for (int k = lane; k < nwd; k += 64) {
    const int64_t lo = (W0 + k) * 32, hi = lo + 32;
    const int b0 = O0 > lo ? (int)(O0 - lo) : 0, b1 = O1 < hi ? (int)(O1 - lo) : 32;
    const uint32_t span = (b1 - b0 == 32) ? ~0u : (((1u << (b1 - b0)) - 1u) << b0);
    if (span == ~0u) {
      *gp(gv + k) = bw[k];
    } else {  // word shared with a neighbouring tile: touch only this span's bits
      g_and(gv + k, ~span);
      g_or(gv + k, bw[k]);
    }
  }
  wave_lds_sync();
}

#ifndef FORY_DEC_FR
#define FORY_DEC_FR 1
#endif

template <int HDR, bool WRITE, int NW, bool SPILL>
__global__ __launch_bounds__(64 * NW) void var_decode_flat_kernel(VarLaunch L, const Op* __restrict__ prog, const ColumnDev* __restrict__ cols,
                                                                  const FixedFieldDev* __restrict__ fix, const VarFieldDev* __restrict__ vf,
                                                                  const StructDev* __restrict__ st,
                                                                  const uint8_t* __restrict__ in,
                                                                  const int64_t* __restrict__ offs,
                                                                  int64_t* __restrict__ tile_tot, int32_t* status,
                                                                  int cap, SpillArgs sp) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int stg_bytes = L.stg_bytes;
  uint8_t* img = lds;
  const int nslot = L.num_var < NW ? L.num_var : NW;  // staging slots: waves with var fields (v = wave + k NW)
  int32_t* sbase = reinterpret_cast<int32_t*>(lds + cap + (WRITE ? nslot * stg_bytes : 0));  // [1 + num_struct][64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // debug timeline (FORY_ROWFMT_VARPROF=1, values pass only): thread 0 stamps
  // s_memrealtime at phase boundaries (uniform branch when off)
#define DEC_STAMP(k)                                                                             \
  do {                                                                                          \
    if (WRITE && L.prof && tid == 0) L.prof[tile * 8 + (k)] = __builtin_amdgcn_s_memrealtime();  \
  } while (0)
  auto body = [&](int64_t tile) {
  DEC_STAMP(0);
  const int64_t r0 = tile * 64;
  int64_t B0, B1, beg, end;
  bool live;
  const bool sane = var_tile_bounds(offs, L.num_rows, r0, lane, &B0, &B1, &beg, &end, &live);
  const int mis = (int)(reinterpret_cast<uintptr_t>(in + B0) & 15);
  const int64_t total = mis + (B1 - B0);
  const int64_t tiles = (L.num_rows + 63) / 64;
  // totals pass of string-only flat plans (fr_bytes: frame header + bitmap + slots): only
  // each record's fixed part is staged, when every record of the tile has one
  const int frb = !WRITE && !SPILL ? L.fr_bytes : 0;
  const bool fr = frb && __ballot(live && end - beg < frb) == 0;
  if (!sane || (mis & 3) || (!fr && total > cap)) {  // per-lane path on global rows (one wave)
    if (!SPILL && sane && !(mis & 3) && total <= sp.cap) {  // spill: the big-image launch takes it
      if (threadIdx.x == 0) sp.list[atomicAdd(sp.count, 1)] = (int32_t)tile;
      return;
    }
    if (wave == 0) {
      const uint8_t* fp = in + beg;
      const uint8_t* row = fp + HDR;
      int64_t row_len = end - beg;
      bool bad = !live;
      if (live && HDR) bad = !frame_ok<HDR>(L, fp, row_len, false, status);
      row_len -= HDR;
      if (L.num_struct) {
        const int rows = L.num_rows - r0 < 64 ? (int)(L.num_rows - r0) : 64;
        flat_dec_struct_bases<false>(L, st, bad, live, lane, r0, rows, row, row_len, sbase, status);
        wave_lds_sync();
      }
      for (int v = 0; v < L.num_var; ++v) {
        int64_t rel = 0, n = 0;
        if (!bad) flat_var_slot(L, vf[v], st, sbase, lane, row, row_len, &rel, &n, !WRITE, status);
        if (!WRITE) {
          const int64_t sum = wave_sum64(n);
          if (lane == 0) tile_tot[v * (tiles + 1) + tile] = sum;
        } else {
          const int64_t base = *gp(vf[v].out_offsets + r0);
          const int64_t excl = wave_incl_scan64(n, lane) - n;
          if (live) *gp(vf[v].out_offsets + r0 + lane) = (int32_t)(base + excl);
        }
      }
      if (WRITE) dec_record<true>(L, prog, cols, r0 + lane, live, in + beg, end - beg, status);
    }
    return;
  }
  int64_t obase = 0;  // tile-start Arrow offsets of every var field (lane v: field v's)
  {  // stage the tile's rows: LDS-DMA of whole 16-B chunks (1 KiB per wave
     // instruction, all in flight at once, nt policy for the once-read rows); the
     // edge chunks' bytes outside the tile (same 16-B blocks) are never read
    const uint8_t* g = in + B0 - mis;
    const int nch = (int)((total + 15) >> 4);
    if (fr) {  // record r's window [beg & ~15, end of its fixed part) at r * frc 16-B chunks
      const int frc = (frb + 15) / 16 + 1;
      const int rows = L.num_rows - r0 < 64 ? (int)(L.num_rows - r0) : 64;
      const int fch = rows * frc;
      for (int c0 = 0; c0 < fch; c0 += 64 * NW) {
        const int cc = c0 + tid;
        const int rr = cc < fch ? cc / frc : 0;
        const int64_t b = __shfl(beg, rr);
        const int64_t ws = b & ~(int64_t)15, we = (b + frb + 15) & ~(int64_t)15;
        const int64_t at = ws + (int64_t)(cc - rr * frc) * 16;
        if (cc < fch && at < we)
          __builtin_amdgcn_global_load_lds((const GAS void*)(in + at),
                                           (__attribute__((address_space(3))) void*)(img + (c0 + wave * 64) * 16), 16,
                                           0, 2);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (L.kn.dec_regs) {  // A/B: non-temporal 16-B loads into registers, kDecRegs per thread in flight, then LDS
      if (WRITE && lane < L.num_var) obase = *gp(vf[lane].out_offsets + r0);
      constexpr int kDecRegs = 8;
      const u32x4* g16 = reinterpret_cast<const u32x4*>(g);
      for (int c0 = 0; c0 < nch; c0 += 64 * NW * kDecRegs) {
        u32x4 r[kDecRegs];
#pragma unroll
        for (int q = 0; q < kDecRegs; ++q) {
          const int cc = c0 + q * 64 * NW + tid;
          r[q] = cc < nch ? __builtin_nontemporal_load(gp(g16 + cc)) : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int q = 0; q < kDecRegs; ++q) {
          const int cc = c0 + q * 64 * NW + tid;
          if (cc < nch) *reinterpret_cast<u32x4*>(img + cc * 16) = r[q];
        }
      }
    } else {
      for (int c0 = 0; c0 < nch; c0 += 64 * NW) {
        const int cc = c0 + tid;
        if (cc < nch)
          __builtin_amdgcn_global_load_lds((const GAS void*)(g + (int64_t)cc * 16),
                                           (__attribute__((address_space(3))) void*)(img + (c0 + wave * 64) * 16), 16,
                                           0, 2);
      }
      // the tile-start Arrow offsets (written by decode_sizes) behind the DMA: their
      // table-pointer load and then the value load overlap the staging
      if (WRITE && lane < L.num_var) obase = *gp(vf[lane].out_offsets + r0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  DEC_STAMP(1);
  const int64_t i = r0 + lane;
  const int rows = L.num_rows - r0 < 64 ? (int)(L.num_rows - r0) : 64;
  const uint8_t* fp = fr ? img + lane * ((frb + 15) / 16 + 1) * 16 + (int)(beg & 15) : img + mis + (int)(beg - B0);
  const uint8_t* row = fp + HDR;
  int64_t row_len = end - beg;
  bool bad = !live;
  if (live && HDR) bad = !frame_ok<HDR>(L, fp, row_len, WRITE && wave == 0, status);  // Encoders.decode
  row_len -= HDR;
  if (L.num_struct) {  // child-row offsets (+ struct validity) for every wave
    if (wave == 0) flat_dec_struct_bases<WRITE>(L, st, bad, live, lane, r0, rows, row, row_len, sbase, status);
    __syncthreads();
  }
  if (!WRITE) {  // pass 1: per-tile payload totals (scanned over tiles by the host launcher)
    for (int v = wave; v < L.num_var; v += NW) {
      int64_t rel = 0, n = 0;
      if (!bad) flat_var_slot(L, vf[v], st, sbase, lane, row, row_len, &rel, &n, true, status);
      const int64_t sum = wave_sum64(n);
      if (lane == 0) tile_tot[v * (tiles + 1) + tile] = sum;
    }
    return;
  }
  DEC_STAMP(2);
  // fixed fields: slot -> column (UnsafeTrait.getInt32/... ; null -> 0), validity by ballot
  {
    int jb[4];
    jb[0] = 0;
    for (int g = 0; g < 3; ++g) jb[g + 1] = jb[g] + (L.fix_group[g + 1] - L.fix_group[g] + kDecBatch - 1) / kDecBatch;
    flat_dec_fixed<8, NW>(L, fix, L.fix_group[0], L.fix_group[1], jb[0], wave, lane, live, bad, i, r0, rows, row, st,
                          sbase);
    flat_dec_fixed<4, NW>(L, fix, L.fix_group[1], L.fix_group[2], jb[1], wave, lane, live, bad, i, r0, rows, row, st,
                          sbase);
    flat_dec_fixed<2, NW>(L, fix, L.fix_group[2], L.fix_group[3], jb[2], wave, lane, live, bad, i, r0, rows, row, st,
                          sbase);
    flat_dec_fixed<1, NW>(L, fix, L.fix_group[3], L.fix_group[4], jb[3], wave, lane, live, bad, i, r0, rows, row, st,
                          sbase);
  }
  if (WRITE && L.prof) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  DEC_STAMP(3);
  // var fields: one per wave at a time, output span staged in LDS
  uint8_t* stg = lds + cap + wave * stg_bytes;
  const bool ivs = NW >= 2 && L.iv_split;  // wave 1 assembles field 0's item validity
  uint32_t* ivw = reinterpret_cast<uint32_t*>(sbase + (L.num_struct ? (1 + L.num_struct) * 64 : 0));
  for (int v = wave; v < L.num_var; v += NW) {
    const VarFieldDev& f = vf[v];
    const bool islist = f.is_list;
    const int w = f.w;
    const int iflags = f.iflags;
    int64_t rel = 0, n = 0;
    bool nul = true;
    if (!bad) nul = flat_var_slot(L, f, st, sbase, lane, row, row_len, &rel, &n, false, status);
    if (f.out_validity) {
      const uint64_t m = __ballot(live && !nul);
      if (lane == 0) write_validity64(f.out_validity, r0, rows, m);
    }
    // Arrow offsets of this tile: base (tile prefix written by decode_sizes) + in-wave prefix
    const int64_t O0 = __shfl(obase, v);
    const int64_t incl = wave_incl_scan64(n, lane);
    const int64_t O1 = O0 + __shfl(incl, 63);
    const int64_t e0 = O0 + incl - n;
    if (live) *gp(f.out_offsets + i) = (int32_t)e0;
    const int64_t S = (O1 - O0) * w;
    const uint8_t* src = row + rel + (islist ? 8 + bitmap_bytes(n) : 0);
    // this lane's payload into the staging at d (BinaryArray.toXArray; null items,
    // BinaryArray.isNullAt, read as 0)
    auto stage_lane = [&](uint8_t* d) {
      if (!islist) {
        lds_copy_any(d, src, (int)n);
        return;
      }
      const uint8_t* abm = row + rel + 8;
      if (w == 8 || w == 4) {  // src 4-byte aligned (8-padded row offsets), d w-aligned
        // a bitmap byte (8 items) at a time: items of a null-free byte move as up to
        // 16 dwords, all loads before the stores; bytes with nulls item by item
        for (int64_t j = 0; j < n; j += 8) {
          const int take = n - j < 8 ? (int)(n - j) : 8;
          const uint32_t nb = abm[j >> 3] & ((1u << take) - 1u);
          const uint8_t* sp = src + j * w;
          uint8_t* dp = d + j * w;
          if (!nb) {
            const int nd = take * w / 4;
            for (int h = 0; h < nd; h += 8) {
              uint32_t t[8];
#pragma unroll
              for (int u = 0; u < 8; ++u) t[u] = h + u < nd ? ld32(sp + 4 * (h + u)) : 0u;
#pragma unroll
              for (int u = 0; u < 8; ++u)
                if (h + u < nd) st32(dp + 4 * (h + u), t[u]);
            }
          } else {
            for (int t = 0; t < take; ++t) {
              const bool en = (nb >> t) & 1;
              st32(dp + t * w, en ? 0u : ld32(sp + t * w));
              if (w == 8) st32(dp + t * w + 4, en ? 0u : ld32(sp + t * w + 4));
            }
          }
        }
      } else {
        for (int64_t j = 0; j < n; ++j) {
          const bool en = (abm[j >> 3] >> (j & 7)) & 1;
          for (int b = 0; b < w; ++b) d[j * w + b] = en ? 0 : src[j * w + b];
        }
      }
    };
    // this lane's payload straight to the column (bool items, records beyond the staging)
    auto lane_global = [&]() {
      if (!islist) {
        copy_out(f.out_values + e0, src, n);
        return;
      }
      const uint8_t* arr = row + rel;
      for (int64_t j = 0; j < n; ++j) {
        const bool en = (arr[8 + (j >> 3)] >> (j & 7)) & 1;
        uint64_t x = 0;
        if (!en) {
          const uint8_t* pp = src + j * w;
          switch (w) {
            case 8: x = (uint64_t)ld32(pp) | ((uint64_t)ld32(pp + 4) << 32); break;
            case 4: x = ld32(pp); break;
            case 2: x = (uint64_t)pp[0] | ((uint64_t)pp[1] << 8); break;
            default: x = pp[0]; break;
          }
        }
        if (iflags & 2) x = (x & 0xff) ? 1 : 0;
        store_elem(f.out_values, w, e0 + j, x);
        if (f.out_item_validity) {
          const int64_t q = e0 + j;
          const uint32_t bit = 1u << (q & 31);
          uint32_t* word = reinterpret_cast<uint32_t*>(f.out_item_validity) + (q >> 5);
          if (en) g_and(word, ~bit);
          else g_or(word, bit);
        }
      }
    };
    const bool fits_all = S >= 0 && S + 32 <= stg_bytes;
    if ((iflags & 2) == 0 && S >= 0) {
      // record groups whose output span fits the staging: the whole tile when it does,
      // else the longest runs of records from lo (a span beyond the staging once took
      // the per-item global path for the whole tile: Nested frame streams, whose bigger
      // image leaves a staging the mean tile span just exceeds, wrote 1.36x the columns)
      for (int lo = 0; lo < rows;) {
        int hi = rows;
        if (!fits_all) {
          const int64_t base = __shfl(e0, lo);
          const int64_t ph = (int64_t)(reinterpret_cast<uintptr_t>(f.out_values + base * w) & 15);
          const bool ok = lane >= lo && lane < rows && ph + (e0 + n - base) * w + 32 <= stg_bytes;
          const uint64_t m = __ballot(ok) >> lo;  // a prefix of the lanes from lo (e0 + n nondecreasing)
          hi = lo + (~m == 0 ? 64 - lo : (int)__builtin_ctzll(~m));
        }
        if (hi == lo) {  // record lo alone exceeds the staging
          if (lane == lo && live && n > 0) lane_global();
          lo = lo + 1;
          continue;
        }
        const bool mine = lane >= lo && lane < hi;
        const int64_t G0 = __shfl(e0, lo), G1 = __shfl(e0 + n, hi - 1);
        const int64_t GS = (G1 - G0) * w;
        uint8_t* gdst = f.out_values + G0 * w;
        const int phase = (int)(reinterpret_cast<uintptr_t>(gdst) & 15);
        if (mine && live && n > 0) stage_lane(stg + phase + (e0 - G0) * w);
        wave_lds_sync();
        uint8_t* g = gdst - phase;
        const int tot = (int)(phase + GS);
        const int nch = (tot + 15) >> 4;
        for (int cc = lane; cc < nch; cc += 64) {
          const int lo16 = cc * 16;
          const u32x4 c = *reinterpret_cast<const u32x4*>(stg + lo16);
          if (lo16 >= phase && lo16 + 16 <= tot) {
            *gp(reinterpret_cast<u32x4*>(g + lo16)) = c;
          } else {  // an edge chunk: its bytes from registers (no LDS read per byte), stores back to back
#pragma unroll
            for (int d = 0; d < 4; ++d) {
              const int o = lo16 + 4 * d;
              if (o >= phase && o + 4 <= tot) {
                *gp(reinterpret_cast<uint32_t*>(g + o)) = c[d];
              } else {
#pragma unroll
                for (int b = 0; b < 4; ++b)
                  if (o + b >= phase && o + b < tot) store_byte(g + o + b, (uint8_t)(c[d] >> (8 * b)));
              }
            }
          }
        }
        wave_lds_sync();
        // the group's item validity, assembled in LDS (staging reused); with one var field,
        // a whole-tile span and an idle second wave, that wave does it (below) while this
        // one copies
        if (islist && f.out_item_validity && !(ivs && fits_all))
          dec_item_validity(f, G0, G1, e0, n, row + rel + 8, live && mine, lane, reinterpret_cast<uint32_t*>(stg));
        lo = hi;
      }
    } else if (live && n > 0) {
      lane_global();
    }
  }
  if (ivs && wave == 1) {  // field 0's item validity (the staged span of wave 0's pass)
    const VarFieldDev& f = vf[0];
    int64_t rel = 0, n = 0;
    if (!bad) flat_var_slot(L, f, st, sbase, lane, row, row_len, &rel, &n, false, status);
    const int64_t O0 = __shfl(obase, 0);
    const int64_t incl = wave_incl_scan64(n, lane);
    const int64_t O1 = O0 + __shfl(incl, 63);
    const int64_t S = (O1 - O0) * f.w;
    if ((f.iflags & 2) == 0 && S >= 0 && S + 32 <= stg_bytes)
      dec_item_validity(f, O0, O1, O0 + incl - n, n, row + rel + 8, live, lane, ivw);
  }
  if (WRITE && L.prof) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    DEC_STAMP(4);
    __syncthreads();
    DEC_STAMP(5);
    DEC_STAMP(6);
    DEC_STAMP(7);
  }
  };
  if (!SPILL) {
    body(var_tile(blockIdx.x, gridDim.x, L.kn.var_xcd));
    return;
  }
  const int64_t count = *sp.count;  // tiles the main launch spilled
  for (int64_t k = blockIdx.x; k < count; k += gridDim.x) {
    body(sp.list[k]);
    __syncthreads();
  }
#undef DEC_STAMP
}

}  // namespace

hipError_t launch_var_sizes(const VarLaunch& L, int64_t* d_row_offsets, hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  const int64_t blocks = (L.num_rows + kWG - 1) / kWG;
  if (L.flat && !L.kn.sizes_program)  // (A/B knob of the plan)
    hipLaunchKernelGGL(var_sizes_flat_kernel, dim3((unsigned)((L.num_rows + kWG * kSizeRows - 1) / (kWG * kSizeRows))),
                       dim3(kWG), 0, s, L, L.vf, L.st, d_row_offsets);
  else
    hipLaunchKernelGGL(var_sizes_kernel, dim3((unsigned)blocks), dim3(kWG), 0, s, L, L.prog, L.cols, d_row_offsets);
  return hipGetLastError();
}

namespace {

// Test knobs: the plan's LaunchKnobs (plan.h), read from the environment once at
// plan creation. They force the fallback engines and LDS budgets so the parity
// suite exercises every path; none selects a rejected variant.
bool var_tiles(const VarLaunch& L) { return !L.kn.no_tiles; }

int var_cap(const VarLaunch& L) {
  const int cap = L.kn.var_cap ? L.kn.var_cap : L.tile_cap;
  return cap < 1024 ? 1024 : (cap > 160 * 1024 ? 160 * 1024 : cap);
}

// Tile image of the cooperative kernels from the batch's mean row (bytes per row or
// frame): 64 rows + 4 % + the 16-B phase, 256-B granular, in [4, 64] KiB. Tiles
// above it go to the spill launch; the image is the largest LDS item, so sizing it
// to the data instead of the plan's static estimate is what sets the resident
// workgroups per CU (Mixed: 37 KiB static -> 32 KiB, 3 -> 4 workgroups per CU).
int fit_cap(const VarLaunch& L, int64_t mean_row) {
  if (L.kn.var_cap || L.kn.var_fit || mean_row <= 0 || L.num_rows < 64)
    return var_cap(L);
  int64_t need = (64 * mean_row * 104 / 100 + 16 + 255) & ~int64_t(255);
  need = need < 4096 ? 4096 : (need > 64 * 1024 ? 64 * 1024 : need);
  return (int)need;
}

// Debug timeline of the cooperative kernels (the plan's FORY_ROWFMT_VARPROF=1): one
// process-wide buffer, 8 stamps per tile.
std::mutex g_prof_mu;
uint64_t* g_prof = nullptr;
int64_t g_prof_words = 0;

}  // namespace

uint64_t* var_prof_buffer(int64_t tiles, bool on) {
  if (!on) return nullptr;
  std::lock_guard<std::mutex> lock(g_prof_mu);
  if (tiles * 8 > g_prof_words) {
    if (g_prof) (void)hipFree(g_prof);
    g_prof = nullptr;
    g_prof_words = 0;
    if (hipMalloc(&g_prof, (size_t)tiles * 8 * sizeof(uint64_t)) != hipSuccess) return nullptr;
    g_prof_words = tiles * 8;
  }
  return g_prof;
}

int64_t var_prof_copy(uint64_t* host, int64_t max_words) {
  std::lock_guard<std::mutex> lock(g_prof_mu);
  if (!g_prof) return 0;
  const int64_t n = max_words < g_prof_words ? max_words : g_prof_words;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(host, g_prof, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return n;
}

namespace {

bool var_flat(const VarLaunch& L) { return L.flat && !L.kn.no_flat; }

constexpr int kNW = 4;  // waves per 64-record tile of the cooperative kernels (8 was slower at every occupancy)

// Waves per tile: 4, or 2 for plans with at most two var fields, whose small tiles
// leave waves idle (the layout is wave 0's; two waves per tile double the tiles in
// flight per CU). bench A/B on one box (profiles/r02/nw/): Nested encode 1.215 ->
// 0.896 ms, decode 1.043 -> 0.766 ms (1 wave: 1.47 ms); Mixed (8 strings) is best at
// 4 (2 waves: encode 4.60 -> 6.64 ms, decode 4.08 -> 5.90 ms).
// FORY_ROWFMT_VARNW=2|4 forces one (tests).
int flat_waves(const VarLaunch& L) {
  if (L.kn.var_nw == 2 || L.kn.var_nw == 4) return L.kn.var_nw;
  return L.num_var <= 2 ? 2 : 4;
}

size_t sbase_lds(const VarLaunch& L) {
  return L.num_struct ? (size_t)(1 + L.num_struct) * 64 * sizeof(int32_t) : 0;
}

// Encode LDS: row image, staging for the min(NW, num_var) waves that place var
// fields, payload offsets and child-row offsets (nested plans).
size_t flat_lds_enc(const VarLaunch& L, int cap, int nw) {
  const int np = var_placers(L.num_var, nw, 1);
  const int nslot = L.num_var < np ? L.num_var : np;
  return (size_t)cap + (size_t)nslot * L.stg_bytes + (size_t)L.num_var * 64 * sizeof(int32_t) + sbase_lds(L);
}

// The largest slot (up to b) that keeps the most resident workgroups any slot in
// [1, 2] KiB reaches (occupancy with the kernel's registers and LDS).
template <typename K, typename F>
int fit_slot(K* k, int threads, int b, F lds_of) {
  int want = -1;
  for (int t = 2048; t >= 1024; t -= 256) {
    const int o = occupancy_of(k, threads, lds_of(t));
    want = o > want ? o : want;
  }
  int r = 1024;
  if (want > 0) {
    r = b;
    while (r > 1024 && occupancy_of(k, threads, lds_of(r)) < want) r -= 256;
  }
  return r;
}

// Encode staging per slot sized from the caller's capacity (normally the exact
// encoded size): 1.5x the mean per-field span of a 64-record tile, in [2, 16] KiB,
// so most tiles stage each field in one record group -- but never at the cost of
// resident workgroups. FORY_ROWFMT_VARSTG overrides.
template <typename K>
int enc_stg_bytes(K* k, const VarLaunch& L, int64_t capacity, int cap, int nw) {
  if (L.kn.var_stg || L.num_rows < 64 || L.num_var == 0) return L.stg_bytes;
  const int64_t var_row = capacity / L.num_rows - L.fixed_size - frame_header_bytes(L.frame) - L.nested_fixed;
  const int64_t per = var_row > 0 ? 64 * var_row / L.num_var : 0;
  int b = (int)((per * 3 / 2 + 512 + 255) & ~int64_t(255));
  b = b < 2048 ? 2048 : (b > 16384 ? 16384 : b);
  return fit_slot(k, 64 * nw, b, [&](int stg) {
    VarLaunch T = L;
    T.stg_bytes = stg;
    return flat_lds_enc(T, cap, nw);
  });
}

// LDS image of the spill launches: 3x the main image, in [32, 96] KiB
// (FORY_ROWFMT_SPILLCAP overrides, for tests).
int spill_cap(const VarLaunch& L, int cap) {
  int c = L.kn.spill_cap ? L.kn.spill_cap : 3 * cap;
  if (!L.kn.spill_cap) c = c < 32 * 1024 ? 32 * 1024 : (c > 96 * 1024 ? 96 * 1024 : c);
  return c < 1024 ? 1024 : (c > 128 * 1024 ? 128 * 1024 : c);
}

SpillArgs spill_args(const VarLaunch& L, int cap) { return SpillArgs{L.spill, L.spill_count, spill_cap(L, cap), 0}; }

// Persistent spill grid: resident workgroups at the spill image size.
template <typename K>
unsigned spill_grid(K* k, const VarLaunch& L, size_t lds, int wg) {
  return (unsigned)persistent_grid(k, lds, (L.num_rows + 63) / 64, wg);
}

// Decode values pass: staging only for the waves that own var fields.
size_t flat_lds_dec(const VarLaunch& L, int cap, int nw) {
  const int nslot = L.num_var < nw ? L.num_var : nw;
  // wave 1's item-validity words: a staged span holds <= stg_bytes items
  const size_t ivw = nw >= 2 && L.iv_split ? (size_t)((L.stg_bytes / 8 + 16 + 15) & ~15) : 0;
  return (size_t)cap + (size_t)nslot * L.stg_bytes + sbase_lds(L) + ivw;
}

// Decode staging per slot: the output span of a 64-record tile of the widest
// var field at the plan's static estimate (var_est_row: ~32 B per string,
// 16 items per list, +25 %), in [2, 16] KiB, under the same occupancy guard as
// the encode slots (FORY_ROWFMT_VARSTG overrides). Spans that still do not fit
// take the per-lane path.
template <typename K>
int dec_stg_bytes(K* k, const VarLaunch& L, int cap, int nw) {
  if (L.kn.var_stg || L.num_var == 0) return L.stg_bytes;
  int b = (int)(((int64_t)64 * L.var_est_row * 5 / 4 + 512 + 255) & ~int64_t(255));
  b = b < 2048 ? 2048 : (b > 16384 ? 16384 : b);
  return fit_slot(k, 64 * nw, b, [&](int stg) {
    VarLaunch T = L;
    T.stg_bytes = stg;
    return flat_lds_dec(T, cap, nw);
  });
}

// Grows a data-fitted tile image (fit_cap) in 256-B steps, up to +20 %, while the
// resident workgroups per CU stay the same: spill margin that costs no occupancy.
template <typename K, typename F>
int grow_cap(const VarLaunch& L, K* k, int threads, int cap, F lds_of) {
  if (L.kn.var_cap || L.kn.var_fit) return cap;
  const int b0 = occupancy_of(k, threads, lds_of(cap));
  int c = cap;
  const int limit = cap * 6 / 5 < 64 * 1024 ? cap * 6 / 5 : 64 * 1024;
  if (b0 > 0)
    while (c + 256 <= limit && occupancy_of(k, threads, lds_of(c + 256)) >= b0) c += 256;
  return c;
}

// FORY_ROWFMT_VARDIAG=1: the tile kernels' LDS sizing and resulting residency, to stderr.
template <typename K>
void var_diag(const VarLaunch& L, const char* what, K* k, int threads, int cap, int stg, size_t lds) {
  if (!L.kn.diag) return;
  fprintf(stderr, "[fory_rowfmt] %s tile kernel: image %d B, staging %d B/slot, LDS %zu B, %d workgroups/CU\n", what,
          cap, stg, lds, occupancy_of(k, threads, lds));
}

// Encode: default or lean kernel (5 waves per SIMD register budget), whichever keeps
// more workgroups per CU resident with its own staging / image sizing (ties: default).
template <int HDR, int NW, bool NEST>
void launch_flat_enc_t(const VarLaunch& L0, const int64_t* offs, uint8_t* out, int64_t capacity, int32_t* status,
                       int cap, hipStream_t s) {
  VarLaunch L = L0;
  L.pl_all = 1;
  auto* kd = &var_encode_flat_kernel<HDR, NW, NEST, false>;
  auto* kl = &var_encode_flat_lean_kernel<HDR, NW, NEST, false>;
  // Staging first, then the image grown while the residency holds. When that leaves the
  // staging >= 4 KiB per slot (small rows: staging is plentiful), the image is grown
  // first instead (<= +12 %, at the same residency) and the staging takes the rest:
  // fewer tiles spill to the big-image launch (Nested encode 0.79 -> 0.73 ms in
  // alternating runs; Mixed keeps its sizing, its staging is the scarce part).
  auto size_for = [&](decltype(kd) kk, int* stg, int* c) {
    VarLaunch T = L;
    *stg = enc_stg_bytes(kk, T, capacity, cap, NW);
    T.stg_bytes = *stg;
    *c = grow_cap(T, kk, 64 * NW, cap, [&](int x) { return flat_lds_enc(T, x, NW); });
    const int occ = occupancy_of(kk, 64 * NW, flat_lds_enc(T, *c, NW));
    if (*stg < 4096 || occ <= 0 || L.kn.var_cap || L.kn.var_fit || L.kn.var_stg) return occ;
    VarLaunch U = L;
    U.stg_bytes = 1024;
    int cc = cap;
    const int lim = cap * 112 / 100 < 64 * 1024 ? cap * 112 / 100 : 64 * 1024;
    while (cc + 256 <= lim && occupancy_of(kk, 64 * NW, flat_lds_enc(U, cc + 256, NW)) >= occ) cc += 256;
    U.stg_bytes = L.stg_bytes;
    const int s2 = enc_stg_bytes(kk, U, capacity, cc, NW);
    U.stg_bytes = s2;
    if (cc <= *c || occupancy_of(kk, 64 * NW, flat_lds_enc(U, cc, NW)) < occ) return occ;
    *stg = s2;
    *c = cc;
    return occ;
  };
  int stg_d = 0, cap_d = cap, stg_l = 0, cap_l = cap;
  const int occ_d = size_for(kd, &stg_d, &cap_d);
  const int occ_l = size_for(kl, &stg_l, &cap_l);
  const bool lean = occ_l > occ_d;
  auto* k = lean ? kl : kd;
  L.stg_bytes = lean ? stg_l : stg_d;
  cap = lean ? cap_l : cap_d;
  raise_lds_cap(k);
  const SpillArgs sp = spill_args(L, cap);
  (void)hipMemsetAsync(L.spill_count, 0, sizeof(int32_t), s);
  var_diag(L, lean ? "encode (lean)" : "encode", k, 64 * NW, cap, L.stg_bytes, flat_lds_enc(L, cap, NW));
  hipLaunchKernelGGL(k, dim3((unsigned)((L.num_rows + 63) / 64)), dim3(64 * NW), flat_lds_enc(L, cap, NW), s, L, L.prog,
                     L.cols, L.fix, L.vf, L.st, offs, out, capacity, status, cap, sp);
  auto* k2 = lean ? &var_encode_flat_lean_kernel<HDR, NW, NEST, true> : &var_encode_flat_kernel<HDR, NW, NEST, true>;
  raise_lds_cap(k2);
  hipLaunchKernelGGL(k2, dim3(spill_grid(k2, L, flat_lds_enc(L, sp.cap, NW), 64 * NW)), dim3(64 * NW),
                     flat_lds_enc(L, sp.cap, NW), s, L, L.prog, L.cols, L.fix, L.vf, L.st, offs, out, capacity, status, sp.cap,
                     sp);
}

// Encode v7 LDS: row image, NW staging slots, the payload-size table (NEST: positions),
// then the null-bit table (flat) or the child-row starts (NEST).
size_t flat7_lds(const VarLaunch& L, int cap, int slot, int nw) {
  const size_t tail = L.num_struct ? (size_t)(1 + L.num_struct) * 64 * sizeof(int32_t)
                                   : (size_t)64 * (L.bitmap_bytes >> 2) * sizeof(uint32_t);
  int nslot = 0;  // waves that own a list field
  for (int w = 0; w < nw; ++w) nslot += flat7_wave_lists(L.list_mask, w, nw) != 0;
  return (size_t)cap + (size_t)nslot * slot + (size_t)L.num_var * 64 * sizeof(int32_t) + tail;
}

// List staging slot of a wave in encode v7 (strings need none: they go through
// registers): the tile spans of the list fields it owns at 1.25x the batch's mean bytes
// per var field (the caller's capacity, normally encoded_size's total, gives the mean row)
// + slack; 256-B granular, [1, 32] KiB; 0 for plans without list fields. A span that does
// not fit is copied per lane from global (correct, slower).
int flat7_slot(const VarLaunch& L, int64_t capacity, int nw) {
  if (!L.num_list) return 0;
  if (L.kn.var_stg) return L.kn.var_stg;
  int own = 0;  // list fields of the wave that owns the most
  for (int w = 0; w < nw; ++w) {
    const int c = __builtin_popcount(flat7_wave_lists(L.list_mask, w, nw));
    own = own > c ? own : c;
  }
  int64_t var_row =
      L.num_rows > 0 ? capacity / L.num_rows - L.fixed_size - frame_header_bytes(L.frame) - L.nested_fixed : 0;
  if (var_row < 0) var_row = 0;
  const int64_t per = L.num_var > 0 ? 64 * var_row / L.num_var : 0;
  int64_t b = own * (per * 5 / 4 + 64);
  b = (b + 255) & ~int64_t(255);
  return (int)(b < 1024 ? 1024 : (b > 32768 ? 32768 : b));
}

template <int HDR, int NW, bool NEST, int OWN>
void launch_flat_enc7(const VarLaunch& L0, const int64_t* offs, uint8_t* out, int64_t capacity, int32_t* status,
                      int cap, hipStream_t s) {
  VarLaunch L = L0;
  L.pl_all = 1;
  auto* k = &var_encode_flat7_kernel<HDR, NW, NEST, OWN>;
  const int slot = flat7_slot(L, capacity, NW);
  const size_t lds = flat7_lds(L, cap, slot, NW);
  raise_lds_cap(k);
  // tiles beyond the image: the tile kernel's big-image spill launch (its own staging)
  auto* k2 = &var_encode_flat_kernel<HDR, NW, NEST, true>;
  L.stg_bytes = enc_stg_bytes(k2, L, capacity, cap, NW);
  const SpillArgs sp = spill_args(L, cap);
  (void)hipMemsetAsync(L.spill_count, 0, sizeof(int32_t), s);
  var_diag(L, "encode v7", k, 64 * NW, cap, slot, lds);
  hipLaunchKernelGGL(k, dim3((unsigned)((L.num_rows + 63) / 64)), dim3(64 * NW), lds, s, L, L.prog, L.cols, L.fix,
                     L.vf, L.st, offs, out, capacity, status, cap, slot, sp);
  raise_lds_cap(k2);
  hipLaunchKernelGGL(k2, dim3(spill_grid(k2, L, flat_lds_enc(L, sp.cap, NW), 64 * NW)), dim3(64 * NW),
                     flat_lds_enc(L, sp.cap, NW), s, L, L.prog, L.cols, L.fix, L.vf, L.st, offs, out, capacity, status,
                     sp.cap, sp);
}

// Encode v9 LDS: row image, the payload-size table, the partial null-bit words, two tile flags.
size_t flat9_lds(const VarLaunch& L, int cap, int nw) {
  return (size_t)cap + (size_t)L.num_var * 64 * sizeof(int32_t) + (size_t)nw * 64 * (L.bitmap_bytes >> 2) * 4 + 8;
}

// Plans encode v9 takes: fixed fields and strings / binary only, one fixed batch per wave.
bool flat9_fits(const VarLaunch& L, int nw) {
  return !L.num_struct && !L.num_list && L.num_var >= 1 && L.num_var <= 2 * nw && L.fix_group[4] >= 1 &&
         L.fix_group[4] <= kFixBatch * nw &&
         L.bitmap_bytes <= 4 * kV9Bmw;
}

template <int HDR, int NW>
void launch_flat_enc9(const VarLaunch& L0, const int64_t* offs, uint8_t* out, int64_t capacity, int32_t* status,
                      int cap, hipStream_t s) {
  VarLaunch L = L0;
  L.pl_all = 1;
  // 2 tiles per workgroup; one instantiation per column nullability (NUL bit 0 fixed, bit 1 var)
  using KFn = decltype(&var_encode_flat9_kernel<HDR, NW, 2, 2, 3>);
  KFn k;
  switch (L.nullable & 3) {
    case 0: k = &var_encode_flat9_kernel<HDR, NW, 2, 2, 0>; break;
    case 1: k = &var_encode_flat9_kernel<HDR, NW, 2, 2, 1>; break;
    case 2: k = &var_encode_flat9_kernel<HDR, NW, 2, 2, 2>; break;
    default: k = &var_encode_flat9_kernel<HDR, NW, 2, 2, 3>;
  }
  const int K = 2;
  const size_t lds = flat9_lds(L, cap, NW);
  raise_lds_cap(k);
  auto* k2 = &var_encode_flat_kernel<HDR, NW, false, true>;  // tiles beyond the image
  L.stg_bytes = enc_stg_bytes(k2, L, capacity, cap, NW);
  const SpillArgs sp = spill_args(L, cap);
  (void)hipMemsetAsync(L.spill_count, 0, sizeof(int32_t), s);
  var_diag(L, "encode v9", k, 64 * NW, cap, 0, lds);
  const unsigned grid = (unsigned)(((L.num_rows + 63) / 64 + K - 1) / K);
  hipLaunchKernelGGL(k, dim3(grid), dim3(64 * NW), lds, s, L, L.prog, L.cols, L.fix, L.vf, offs, out, capacity,
                     status, cap, sp);
  raise_lds_cap(k2);
  hipLaunchKernelGGL(k2, dim3(spill_grid(k2, L, flat_lds_enc(L, sp.cap, NW), 64 * NW)), dim3(64 * NW),
                     flat_lds_enc(L, sp.cap, NW), s, L, L.prog, L.cols, L.fix, L.vf, L.st, offs, out, capacity, status,
                     sp.cap, sp);
}

template <int HDR, int NW, bool NEST>
void launch_flat_enc7_own(const VarLaunch& L, const int64_t* offs, uint8_t* out, int64_t capacity, int32_t* status,
                          int cap, hipStream_t s) {
  if (L.num_var <= 2 * NW) launch_flat_enc7<HDR, NW, NEST, 2>(L, offs, out, capacity, status, cap, s);
  else launch_flat_enc7<HDR, NW, NEST, kOwnVar>(L, offs, out, capacity, status, cap, s);
}

template <int HDR, int NW>
void launch_flat_enc(const VarLaunch& L, const int64_t* offs, uint8_t* out, int64_t capacity, int32_t* status,
                     int cap, hipStream_t s) {
  // plans with nested struct fields and flat ones get their own instantiations: each
  // carries only its layout path (the other one's registers would count against it)
  // defaults (measured): plans with nested structs -> the round-3 tile kernel
  // (Nested 0.74 vs v7 0.79 ms); flat plans of fixed fields + strings -> v9 (Mixed 3.2 vs
  // v7 3.6, round 3 4.5 ms); other flat plans (lists) -> v7. FORY_ROWFMT_VARENC=1 / 7 / 9
  // force round 3 / v7 / v9 where they apply (the parity suite runs every one).
  const int e = L.kn.var_enc;
  const bool v7 = e != 1 && L.num_var <= kOwnVar * NW;
  if (L.num_struct) {
    if (v7 && e == 7) launch_flat_enc7_own<HDR, NW, true>(L, offs, out, capacity, status, cap, s);
    else launch_flat_enc_t<HDR, NW, true>(L, offs, out, capacity, status, cap, s);
  } else if ((e == 0 || e == 9) && flat9_fits(L, NW)) {
    launch_flat_enc9<HDR, NW>(L, offs, out, capacity, status, cap, s);
  } else {
    if (v7) launch_flat_enc7_own<HDR, NW, false>(L, offs, out, capacity, status, cap, s);
    else launch_flat_enc_t<HDR, NW, false>(L, offs, out, capacity, status, cap, s);
  }
}

template <int HDR, bool WRITE, int NW>
void launch_flat_dec(const VarLaunch& L0, const uint8_t* rows, const int64_t* offs, int64_t* tile_tot,
                     int32_t* status, int cap, hipStream_t s) {
  auto* k = &var_decode_flat_kernel<HDR, WRITE, NW, false>;
  raise_lds_cap(k);
  VarLaunch L = L0;
  L.fr_bytes = 0;
  if (!WRITE && FORY_DEC_FR && !L.num_struct && !L.num_list && !L.level2) {
    // totals pass of a string-only flat plan: a tile image of each record's fixed part (tiles
    // with a shorter record keep the whole-row image, or spill)
    const int frb = HDR + L.fixed_size;
    const int img = ((frb + 15) / 16 + 1) * 16 * 64;
    if (img < cap) {
      L.fr_bytes = frb;
      cap = img;
    }
  }
  if (WRITE) L.stg_bytes = dec_stg_bytes(k, L0, cap, NW);
  if (WRITE && L.mean_row > 0) cap = grow_cap(L, k, 64 * NW, cap, [&](int c) { return flat_lds_dec(L, c, NW); });
  const SpillArgs sp = spill_args(L, cap);
  (void)hipMemsetAsync(L.spill_count, 0, sizeof(int32_t), s);
  const size_t lds = WRITE ? flat_lds_dec(L, cap, NW) : (size_t)cap + sbase_lds(L);  // pass 1: row image (+ struct offsets)
  var_diag(L, WRITE ? "decode" : "decode lengths", k, 64 * NW, cap, L.stg_bytes, lds);
  hipLaunchKernelGGL(k, dim3((unsigned)((L.num_rows + 63) / 64)), dim3(64 * NW), lds, s, L, L.prog, L.cols, L.fix,
                     L.vf, L.st, rows, offs, tile_tot, status, cap, sp);
  auto* k2 = &var_decode_flat_kernel<HDR, WRITE, NW, true>;
  raise_lds_cap(k2);
  const size_t lds2 = WRITE ? flat_lds_dec(L, sp.cap, NW) : (size_t)sp.cap + sbase_lds(L);
  hipLaunchKernelGGL(k2, dim3(spill_grid(k2, L, lds2, 64 * NW)), dim3(64 * NW), lds2, s, L, L.prog, L.cols, L.fix,
                     L.vf, L.st, rows, offs, tile_tot, status, sp.cap, sp);
}

// Encode: the caller's capacity (normally encoded_size's total) gives the mean
// row size for free (fit_cap).
int enc_cap(const VarLaunch& L, int64_t capacity) {
  if (L.num_rows < 64) return var_cap(L);
  return fit_cap(L, capacity / L.num_rows);
}

template <bool WRITE>
hipError_t launch_var_decode_pass(const VarLaunch& L, const uint8_t* rows, const int64_t* offs, int64_t* tile_tot,
                                  int32_t* status, hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  if (var_tiles(L) && var_flat(L)) {
    const int cap = fit_cap(L, L.mean_row);
    if (flat_waves(L) == 2) {
      switch (frame_header_bytes(L.frame)) {
        case 12: launch_flat_dec<12, WRITE, 2>(L, rows, offs, tile_tot, status, cap, s); break;
        case 8: launch_flat_dec<8, WRITE, 2>(L, rows, offs, tile_tot, status, cap, s); break;
        default: launch_flat_dec<0, WRITE, 2>(L, rows, offs, tile_tot, status, cap, s); break;
      }
      return hipGetLastError();
    }
    switch (frame_header_bytes(L.frame)) {
      case 12: launch_flat_dec<12, WRITE, kNW>(L, rows, offs, tile_tot, status, cap, s); break;
      case 8: launch_flat_dec<8, WRITE, kNW>(L, rows, offs, tile_tot, status, cap, s); break;
      default: launch_flat_dec<0, WRITE, kNW>(L, rows, offs, tile_tot, status, cap, s); break;
    }
    return hipGetLastError();
  }
  if (var_tiles(L)) {
    const int cap = var_cap(L);
    const SpillArgs sp = spill_args(L, cap);
    (void)hipMemsetAsync(L.spill_count, 0, sizeof(int32_t), s);
    raise_lds_cap(&var_decode_tile_kernel<WRITE, false>);
    hipLaunchKernelGGL((var_decode_tile_kernel<WRITE, false>), dim3((unsigned)((L.num_rows + 63) / 64)), dim3(64),
                       (size_t)cap, s, L, L.prog, L.cols, rows, offs, status, cap, sp);
    raise_lds_cap(&var_decode_tile_kernel<WRITE, true>);
    hipLaunchKernelGGL((var_decode_tile_kernel<WRITE, true>),
                       dim3(spill_grid(&var_decode_tile_kernel<WRITE, true>, L, (size_t)sp.cap, 64)), dim3(64),
                       (size_t)sp.cap, s, L, L.prog, L.cols, rows, offs, status, sp.cap, sp);
    return hipGetLastError();
  }
  const int64_t blocks = (L.num_rows + kWG - 1) / kWG;
  hipLaunchKernelGGL(var_decode_kernel<WRITE>, dim3((unsigned)blocks), dim3(kWG), 0, s, L, L.prog, L.cols, rows, offs,
                     status);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_var_encode(const VarLaunch& L, const int64_t* offs, uint8_t* out, int64_t capacity,
                             int32_t* status, hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  if (var_tiles(L) && var_flat(L)) {
    const int cap = enc_cap(L, capacity);
    if (flat_waves(L) == 2) {
      switch (frame_header_bytes(L.frame)) {
        case 12: launch_flat_enc<12, 2>(L, offs, out, capacity, status, cap, s); break;
        case 8: launch_flat_enc<8, 2>(L, offs, out, capacity, status, cap, s); break;
        default: launch_flat_enc<0, 2>(L, offs, out, capacity, status, cap, s); break;
      }
      return hipGetLastError();
    }
    switch (frame_header_bytes(L.frame)) {
      case 12: launch_flat_enc<12, kNW>(L, offs, out, capacity, status, cap, s); break;
      case 8: launch_flat_enc<8, kNW>(L, offs, out, capacity, status, cap, s); break;
      default: launch_flat_enc<0, kNW>(L, offs, out, capacity, status, cap, s); break;
    }
    return hipGetLastError();
  }
  if (var_tiles(L)) {
    const int cap = enc_cap(L, capacity);
    const SpillArgs sp = spill_args(L, cap);
    (void)hipMemsetAsync(L.spill_count, 0, sizeof(int32_t), s);
    raise_lds_cap(&var_encode_tile_kernel<false>);
    hipLaunchKernelGGL(var_encode_tile_kernel<false>, dim3((unsigned)((L.num_rows + 63) / 64)), dim3(64),
                       (size_t)cap, s, L, L.prog, L.cols, offs, out, capacity, status, cap, sp);
    raise_lds_cap(&var_encode_tile_kernel<true>);
    hipLaunchKernelGGL(var_encode_tile_kernel<true>,
                       dim3(spill_grid(&var_encode_tile_kernel<true>, L, (size_t)sp.cap, 64)), dim3(64),
                       (size_t)sp.cap, s, L, L.prog, L.cols, offs, out, capacity, status, sp.cap, sp);
    return hipGetLastError();
  }
  const int64_t blocks = (L.num_rows + kWG - 1) / kWG;
  hipLaunchKernelGGL(var_encode_kernel, dim3((unsigned)blocks), dim3(kWG), 0, s, L, L.prog, L.cols, offs, out,
                     capacity, status);
  return hipGetLastError();
}

bool var_decode_tiled_offsets(const VarLaunch& L) { return L.num_rows > 0 && var_tiles(L) && var_flat(L); }

int64_t var_tile_totals_words(int64_t num_var, int64_t n) { return num_var * ((n + 63) / 64 + 1); }

int64_t var_spill_words(int64_t n) { return (n + 63) / 64 + 4; }

hipError_t launch_var_decode_lengths(const VarLaunch& L, const uint8_t* rows, const int64_t* offs,
                                     int64_t* tile_tot, int64_t* partials, int32_t* status, hipStream_t s) {
  hipError_t e = launch_var_decode_pass<false>(L, rows, offs, tile_tot, status, s);
  if (e != hipSuccess || !var_decode_tiled_offsets(L)) return e;
  const int64_t tiles = (L.num_rows + 63) / 64;
  e = launch_scan_i64_multi(tile_tot, tiles, tiles + 1, L.num_var, partials, s);  // each field's tile totals
  if (e != hipSuccess) return e;
  const int64_t words = (int64_t)L.num_var * (tiles + 1);
  hipLaunchKernelGGL(flat_tile_bases_kernel, dim3((unsigned)((words + kWG - 1) / kWG)), dim3(kWG), 0, s, L.vf,
                     L.num_var, tile_tot, L.num_rows, status);
  return hipGetLastError();
}

hipError_t launch_var_decode(const VarLaunch& L, const uint8_t* rows, const int64_t* offs, int32_t* status,
                             hipStream_t s) {
  return launch_var_decode_pass<true>(L, rows, offs, nullptr, status, s);
}

}  // namespace fory_amd
