// generic.hip — the tree engine: any nesting of struct / list / map fields.
//
// The op-program engines (varlen.hip) cover the shapes of the benchmark configs
// and most beans: scalars, strings, nested structs, list<scalar | string>,
// List<Bean of fixed fields>, maps of scalars / strings. Everything else —
// list<list<...>>, List<Bean with strings / lists / maps>, Map<K, Bean>,
// Map<Bean, List<Bean>> (the reference's own ArrayEncoderTest / MapEncoderTest /
// BeanA shapes) — runs here: one lane per record walks the schema tree exactly as
// the generated codec does (BaseBinaryEncoderBuilder.serializeFor, :149-490):
//   struct : child row inline at the writerIndex, slot = (rel, size)      :436-490
//   list   : BinaryArrayWriter.reset(n) + per-element serializeFor       :293-351
//            [i64 n][bitmap][n x elemSize padded to 8][element var data]   BinaryArrayWriter.java:93-118
//   map    : [i64 keyArrayBytes][key array][value array]                 :370-427, BinaryMap.java:62-77
//   string : bytes at the writerIndex, zero-padded to 8, slot = (rel, n) BinaryWriter.java:162-194
//   decimal: 32 bytes at the writerIndex (decimal128 sign-extended), slot = (rel, 32)
//            BinaryWriter.writeDecimal :214-230, DecimalUtils.DECIMAL_BYTE_LENGTH = 32
//   BigInteger: toByteArray() as bytes (writeUnaligned), slot = (rel, len)  :192-194, :559-560
// Offsets in slots are relative to the enclosing row's / array's start. Rows are
// written straight to global memory (the output is not zeroed by the caller, so
// every fixed part is zeroed first: the bytes Java writes into a fresh buffer).
// Decode walks the same tree level by level: the lengths pass of container depth L
// (list / map nesting) writes the counts of the columns at depth L, their Arrow
// offsets are scanned, then depth L+1 can be positioned (decode_sizes); the values
// pass writes every column.
//
// No device recursion: each lane keeps an explicit stack of D frames (one per open
// struct / array / map, D = schema depth + 1, a template parameter), so the kernels
// have a static scratch size.
#include "gen_device.h"

namespace fory_amd {

namespace {

template <int D, bool TAB>
__global__ __launch_bounds__(kWG) void gen_sizes_kernel(GenLaunch L0, int64_t* sizes) {
  __shared__ GenTables tabs;
  const GenLaunch L = gen_tables<TAB>(L0, &tabs);
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i >= L.num_rows) return;
  bool overflow = false;
  const int64_t s = g_sizes<D>(L, i, &overflow);
  sizes[i] = overflow ? 0 : s;  // overflow: the encode pass reports it
}

template <int D, bool TAB>
__global__ __launch_bounds__(kWG) void gen_encode_kernel(GenLaunch L0, const int64_t* __restrict__ offs,
                                                         uint8_t* __restrict__ out, int64_t capacity,
                                                         int32_t* status) {
  __shared__ GenTables tabs;
  const GenLaunch L = gen_tables<TAB>(L0, &tabs);
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i >= L.num_rows) return;
  gen_encode_one<D>(L, offs, out, capacity, status, i);
}

// ---------------------------------------------------------------------------
// decode
// ---------------------------------------------------------------------------
// Validity of position pos (1 = valid), words shared between lanes.
__device__ __forceinline__ void g_valid_bit(uint8_t* validity, int64_t pos, bool valid) {
  uint32_t* word = reinterpret_cast<uint32_t*>(validity) + (pos >> 5);
  const uint32_t bit = 1u << (pos & 31);
  if (valid) atomicOr(word, bit);
  else atomicAnd(word, ~bit);
}

// Array header at `at` bounded by `lim`: numElements, or -1 (corrupt).
__device__ __forceinline__ int64_t g_array_n(const GenLaunch& L, const uint8_t* row, int item, int64_t at,
                                             int64_t lim) {
  if (at < 0 || at + 8 > lim) return -1;
  const int64_t n = (int64_t)gget(row + at, 8);
  if (n < 0 || n > 0x7fffffffLL || at + 8 + gbm(n) + n * elem_size(L.nodes[item]) > lim) return -1;
  return n;
}

// A container (LIST / MAP) payload at [at, at + size): its element count, or -1;
// *kat / *vat: the (key) array and the value array.
__device__ int64_t g_container_n(const GenLaunch& L, const uint8_t* row, int node, int64_t at, int64_t size,
                                 int64_t* kat, int64_t* vat) {
  if (L.nodes[node].kind == KIND_LIST) {
    *kat = at;
    return g_array_n(L, row, node + 1, at, at + size);
  }
  // BinaryMap.pointTo (BinaryMap.java:62-77): [i64 keyArrayBytes][keys][values]
  if (size < 8) return -1;
  const int64_t kb = (int64_t)gget(row + at, 8);
  const int key = node + 1, val = L.nodes[key].end;
  *kat = at + 8;
  *vat = at + 8 + kb;
  if (kb < 8 || *vat + 8 > at + size) return -1;
  const int64_t nk = g_array_n(L, row, key, *kat, *vat);
  const int64_t nv = g_array_n(L, row, val, *vat, at + size);
  return nk < 0 || nk != nv ? -1 : nk;  // keys.numElements() == values.numElements()
}

// Decodes record i of `row` (row_len bytes) for L.fill_level: >= 0 the counts of
// the columns at that container depth (Arrow offsets[pos + 1]), -1 every value.
// present = false: the record is broken (its values read as null).
template <int D>
__device__ void g_decode(const GenLaunch& L, const uint8_t* row, int64_t row_len, int64_t i, bool present,
                         int32_t* status) {
  GFrame st[D];
  int sp = 0;
  const bool values = L.fill_level < 0;
  auto corrupt = [&]() { set_status(status, FORY_ERR_CORRUPT); };
  // A container's elements: positions out_offsets[pos] .. + n (checked against the sizes pass).
  auto open_container = [&](int node, int64_t at, int64_t size, int64_t pos) {
    const ColumnDev& c = L.cols[node];
    int64_t kat = 0, vat = 0;
    const int64_t n = g_container_n(L, row, node, at, size, &kat, &vat);
    if (n < 0) { corrupt(); return; }
    const int64_t p0 = c.out_offsets[pos];
    if ((int64_t)c.out_offsets[pos + 1] - p0 != n) { corrupt(); return; }  // the rows changed since
    if (n == 0) return;
    if (sp == D) { corrupt(); return; }
    const bool map = L.nodes[node].kind == KIND_MAP;
    GFrame& f = st[sp++];
    f.type = map ? F_MAP_KEYS : F_ARRAY;
    f.node = node;
    f.ch = node + 1;
    f.k = 0;
    f.n = (int32_t)n;
    f.pos = p0;
    f.start = (int32_t)kat;
    f.header = 8 + gbm(n);
    f.elem = elem_size(L.nodes[node + 1]);
    f.off = (int32_t)vat;
    f.rel = 1;
  };
  // The value of `node` read through frame r's slot k, at position pos.
  auto visit = [&](int node, const GFrame& r, int32_t k, int64_t pos) {
    const GNode& nd = L.nodes[node];
    const ColumnDev& c = L.cols[node];
    const int32_t bm = r.type == F_STRUCT ? 0 : 8;
    const bool isnull = !r.rel || ((row[r.start + bm + (k >> 3)] >> (k & 7)) & 1);  // isNullAt
    const uint8_t* slot = row + r.start + r.header + (int64_t)k * r.elem;
    if (values && (nd.flags & 1) && c.out_validity) g_valid_bit(c.out_validity, pos, !isnull);
    if (is_scalar(nd.kind)) {
      if (!values) return;
      uint64_t v = isnull ? 0 : gget(slot, nd.width);  // UnsafeTrait.getX: the low bytes of the slot
      if (nd.kind == KIND_BOOL) v = (v & 0xff) ? 1 : 0;
      store_elem(c.out_values, nd.width, pos, v);
      return;
    }
    if (nd.kind == KIND_STRUCT) {
      if (!values && nd.cdepth > L.fill_level) return;  // nothing at this level below
      if (sp == D) { corrupt(); return; }
      GFrame& f = st[sp++];
      f.type = F_STRUCT;
      f.ch = node + 1;
      f.end = nd.end;
      f.k = 0;
      f.pos = pos;
      f.start = 0;
      f.header = gbm(nd.nchild);
      f.elem = 8;
      f.rel = 0;
      if (!isnull) {  // BinaryRow.getStruct: the child row at the slot's offset
        const int64_t rel = (int32_t)(gget(slot, 8) >> 32);
        const int64_t start = r.start + rel;
        if (rel < 0 || start + f.header + 8LL * nd.nchild > row_len) corrupt();
        else f.start = (int32_t)start, f.rel = 1;
      }
      return;
    }
    if (nd.kind == KIND_DECIMAL) {  // UnsafeTrait.getDecimal (UnsafeTrait.java:139-150): 32 bytes
      if (!values) return;
      uint32_t w[4] = {0u, 0u, 0u, 0u};  // null: zeros
      if (!isnull && g_bigint(nd)) {  // new BigInteger(getBinary(ordinal)): sign-extended big-endian bytes
        const uint64_t os = gget(slot, 8);
        const int64_t rel = (int64_t)(int32_t)(os >> 32), at = r.start + rel, len = (int64_t)(int32_t)(uint32_t)os;
        if (rel < 0 || len < 0 || at + len > row_len || !g_get_bigint(row + at, len, w)) {
          corrupt();
          return;
        }
      } else if (!isnull) {
        const uint64_t os = gget(slot, 8);
        const int64_t rel = (int64_t)(int32_t)(os >> 32), at = r.start + rel;
        if (rel < 0 || (uint32_t)os != 32u || at + 32 > row_len || (at & 3)) {
          corrupt();
          return;
        }
        for (int q = 0; q < 4; ++q) w[q] = ld32(row + at + 4 * q);
        const uint32_t ext = (w[3] >> 31) ? 0xffffffffu : 0u;
        bool fits = true;  // a decimal128 output holds it: bytes 16..31 are the sign extension
        for (int q = 4; q < 8; ++q) fits = fits && ld32(row + at + 4 * q) == ext;
        if (!fits) {
          corrupt();
          return;
        }
      }
      for (int q = 0; q < 4; ++q) st32(c.out_values + 16 * pos + 4 * q, w[q]);
      return;
    }
    // BYTES / LIST / MAP: (offset, size) relative to the enclosing row / array
    int64_t at = 0, size = 0;
    if (!isnull) {
      const uint64_t os = gget(slot, 8);
      at = r.start + (int64_t)(int32_t)(os >> 32);
      size = (int64_t)(int32_t)(uint32_t)os;
      if ((int32_t)(os >> 32) < 0 || size < 0 || at + size > row_len) {
        corrupt();
        return;
      }
    }
    if (!values) {
      if (nd.cdepth == L.fill_level) {  // this level's counts
        if (!c.out_offsets) return;
        int64_t cnt = 0;
        if (!isnull) {
          if (nd.kind == KIND_BYTES) {
            cnt = size;
          } else {
            int64_t kat, vat;
            cnt = g_container_n(L, row, node, at, size, &kat, &vat);
            if (cnt < 0) {
              corrupt();
              cnt = 0;
            }
          }
        }
        c.out_offsets[pos + 1] = (int32_t)cnt;
        return;
      }
      if (nd.kind == KIND_BYTES || isnull || nd.cdepth > L.fill_level) return;
      open_container(node, at, size, pos);  // a deeper level's counts
      return;
    }
    if (isnull) return;
    if (nd.kind == KIND_BYTES) {
      const int64_t o0 = c.out_offsets[pos];
      if ((int64_t)c.out_offsets[pos + 1] - o0 != size) {  // differs from the sizes pass
        corrupt();
        return;
      }
      g_get_bytes(c.out_values + o0, row + at, size);
      return;
    }
    open_container(node, at, size, pos);
  };
  if (L.frame == FORY_FRAME_COLLECTION) {
    const ColumnDev& c = L.cols[0];
    if (values && (L.nodes[0].flags & 1) && c.out_validity) g_valid_bit(c.out_validity, i, present);
    if (!present) return;
    if (L.fill_level == 0) {
      int64_t kat, vat;
      const int64_t n = g_container_n(L, row, 0, 0, row_len, &kat, &vat);
      if (n < 0) corrupt();
      if (c.out_offsets) c.out_offsets[i + 1] = (int32_t)(n < 0 ? 0 : n);
      return;
    }
    open_container(0, 0, row_len, i);
  } else {
    GFrame& f = st[sp++];
    f.type = F_STRUCT;
    f.ch = 0;
    f.end = L.num_nodes;
    f.k = 0;
    f.pos = i;
    f.start = 0;
    f.header = L.bitmap_bytes;
    f.elem = 8;
    f.rel = present ? 1 : 0;
  }
  while (sp > 0) {
    GFrame& f = st[sp - 1];
    const bool more = f.type == F_STRUCT ? f.ch < f.end : f.k < f.n;
    if (more) {
      int node;
      int64_t pos;
      const int32_t k = f.k++;
      if (f.type == F_STRUCT) {
        node = f.ch;
        f.ch = L.nodes[node].end;
        pos = f.pos;
      } else {
        node = f.ch;
        pos = f.pos + k;
      }
      const GFrame r = f;
      visit(node, r, k, pos);
      continue;
    }
    if (f.type == F_MAP_KEYS) {  // keys done: the value array (same count, same positions)
      f.type = F_MAP_VALS;
      f.ch = L.nodes[f.ch].end;
      f.k = 0;
      f.start = f.off;
      f.elem = elem_size(L.nodes[f.ch]);
      continue;
    }
    --sp;
  }
}

template <int D, bool TAB>
__global__ __launch_bounds__(kWG) void gen_decode_kernel(GenLaunch L0, const uint8_t* __restrict__ in,
                                                         const int64_t* __restrict__ offs, int32_t* status) {
  __shared__ GenTables tabs;
  const GenLaunch L = gen_tables<TAB>(L0, &tabs);
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i >= L.num_rows) return;
  const int64_t beg = offs[i], end = offs[i + 1];
  const uint8_t* frame = in + beg;
  int64_t len = end - beg;
  bool bad = end < beg || len > 0x7fffffffLL + 12;
  const bool report = L.fill_level <= 0;  // each error once: the first lengths pass, or the values pass
  auto fail = [&](int32_t code) {
    if (report) set_status(status, code);
    bad = true;
  };
  if (bad) fail(FORY_ERR_CORRUPT);
  const int hdr = L.frame == FORY_FRAME_COLLECTION ? 4 : frame_header_bytes(L.frame);
  if (!bad && L.frame == FORY_FRAME_COLLECTION) {  // [i32 size][payload] (Encoders.java:394-404)
    const int64_t size = len >= 4 ? (int64_t)ld32(frame) : -1;
    if (size < 8 || size + 4 != len) fail(FORY_ERR_CORRUPT);
  } else if (!bad && hdr == 12) {  // Encoders.decode(MemoryBuffer): size, then the schema hash (:177-193)
    if (len < 12) fail(FORY_ERR_CORRUPT);
    else if (gget(frame + 4, 8) != (uint64_t)L.schema_hash) fail(FORY_ERR_SCHEMA_MISMATCH);
    else if ((int64_t)ld32(frame) + 4 != len || len < 12 + L.fixed_size) fail(FORY_ERR_CORRUPT);
  } else if (!bad && hdr == 8) {  // decode(byte[]) (Encoders.java:195-197)
    if (len < 8) fail(FORY_ERR_CORRUPT);
    else if (gget(frame, 8) != (uint64_t)L.schema_hash) fail(FORY_ERR_SCHEMA_MISMATCH);
    else if (len < 8 + L.fixed_size) fail(FORY_ERR_CORRUPT);
  } else if (!bad && len < L.fixed_size) {  // a raw row shorter than its fixed part
    fail(FORY_ERR_CORRUPT);
  }
  g_decode<D>(L, frame + hdr, bad ? 0 : len - hdr, i, !bad, status);
}

template <int D, bool TAB>
hipError_t launch_gen_t(const GenLaunch& L, int what, int64_t* sizes, const int64_t* offs, uint8_t* out,
                        int64_t capacity, const uint8_t* rows, int32_t* status, hipStream_t s) {
  const dim3 grid((unsigned)((L.num_rows + kWG - 1) / kWG));
  if (what == 0) hipLaunchKernelGGL((gen_sizes_kernel<D, TAB>), grid, dim3(kWG), 0, s, L, sizes);
  else if (what == 1)
    hipLaunchKernelGGL((gen_encode_kernel<D, TAB>), grid, dim3(kWG), 0, s, L, offs, out, capacity, status);
  else hipLaunchKernelGGL((gen_decode_kernel<D, TAB>), grid, dim3(kWG), 0, s, L, rows, offs, status);
  return hipGetLastError();
}

template <int D>
hipError_t launch_gen_d(const GenLaunch& L, int what, int64_t* sizes, const int64_t* offs, uint8_t* out,
                        int64_t capacity, const uint8_t* rows, int32_t* status, hipStream_t s) {
  if (L.num_nodes <= kGenLdsNodes) return launch_gen_t<D, true>(L, what, sizes, offs, out, capacity, rows, status, s);
  return launch_gen_t<D, false>(L, what, sizes, offs, out, capacity, rows, status, s);
}

// Frames = open containers + the row: schema depth + 1 (plan depth <= 17).
hipError_t launch_gen(const GenLaunch& L, int what, int64_t* sizes, const int64_t* offs, uint8_t* out,
                      int64_t capacity, const uint8_t* rows, int32_t* status, hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  if (L.max_depth + 1 <= 4) return launch_gen_d<4>(L, what, sizes, offs, out, capacity, rows, status, s);
  if (L.max_depth + 1 <= 8) return launch_gen_d<8>(L, what, sizes, offs, out, capacity, rows, status, s);
  return launch_gen_d<18>(L, what, sizes, offs, out, capacity, rows, status, s);
}

}  // namespace

hipError_t launch_gen_sizes(const GenLaunch& L, int64_t* sizes, hipStream_t s) {
  return launch_gen(L, 0, sizes, nullptr, nullptr, 0, nullptr, nullptr, s);
}

hipError_t launch_gen_encode(const GenLaunch& L, const int64_t* offs, uint8_t* out, int64_t capacity,
                             int32_t* status, hipStream_t s) {
  return launch_gen(L, 1, nullptr, offs, out, capacity, nullptr, status, s);
}

hipError_t launch_gen_decode(const GenLaunch& L, const uint8_t* rows, const int64_t* offs, int32_t* status,
                             hipStream_t s) {
  return launch_gen(L, 2, nullptr, offs, nullptr, 0, rows, status, s);
}

}  // namespace fory_amd
