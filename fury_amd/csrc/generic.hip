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
#include "kcommon.h"

namespace fory_amd {

namespace {

__device__ __forceinline__ int32_t gbm(int64_t n) { return (int32_t)(((n + 63) >> 6) << 3); }
__device__ __forceinline__ int64_t gr8(int64_t n) { return (n + 7) & ~int64_t(7); }

__device__ __forceinline__ bool gvalid(const uint8_t* validity, int64_t i) {
  return !validity || ((validity[i >> 3] >> (i & 7)) & 1);
}

// Row bytes at p: 8-byte values are 4-byte aligned at least (frame rows start 12
// bytes into the frame), narrower ones naturally aligned relative to the row start.
__device__ __forceinline__ void gput(uint8_t* p, uint64_t v, int w) {
  switch (w) {
    case 8:
      st32(p, (uint32_t)v);
      st32(p + 4, (uint32_t)(v >> 32));
      break;
    case 4: st32(p, (uint32_t)v); break;
    case 2: *reinterpret_cast<uint16_t*>(p) = (uint16_t)v; break;
    default: *p = (uint8_t)v; break;
  }
}

__device__ __forceinline__ uint64_t gget(const uint8_t* p, int w) {
  switch (w) {
    case 8: return (uint64_t)ld32(p) | ((uint64_t)ld32(p + 4) << 32);
    case 4: return ld32(p);
    case 2: return *reinterpret_cast<const uint16_t*>(p);
    default: return *p;
  }
}

__device__ __forceinline__ void gzero(uint8_t* p, int64_t n) {  // p 4-byte aligned, n multiple of 4
  for (int64_t k = 0; k < n; k += 4) st32(p + k, 0u);
}

// writeUnaligned's bytes (+ zero padding to 8) at a 4-byte aligned row position from a
// source of any alignment: aligned source dwords, each holding at least one byte of
// the string (never outside the mapped buffer), funnel-shifted into dword stores.
__device__ __forceinline__ void g_put_bytes(uint8_t* dst, const uint8_t* src, int64_t n) {
  const int sh = (int)(reinterpret_cast<uintptr_t>(src) & 3);
  const uint32_t* s = reinterpret_cast<const uint32_t*>(src - sh);
  const int64_t nw = (n + 3) >> 2;
  uint32_t lo = nw > 0 ? s[0] : 0u;
  for (int64_t k = 0; k < nw; ++k) {
    uint32_t w = lo;
    if (sh) {
      const uint32_t hi = 4 * (k + 1) - sh < n ? s[k + 1] : 0u;
      w = (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sh));
      lo = hi;
    } else if (k + 1 < nw) {
      lo = s[k + 1];
    }
    const int64_t left = n - 4 * k;
    if (left < 4) w &= (1u << (8 * left)) - 1u;
    st32(dst + 4 * k, w);
  }
  if (gr8(n) > 4 * nw) st32(dst + 4 * nw, 0u);  // zeroOutPaddingBytes
}

// Row bytes (4-byte aligned source) to an Arrow values buffer of any alignment:
// byte head to a 4-byte boundary, dword body (funnel-shifted source), byte tail.
__device__ __forceinline__ void g_get_bytes(uint8_t* dst, const uint8_t* src, int64_t n) {
  int64_t b = 0;
  for (; b < n && (reinterpret_cast<uintptr_t>(dst + b) & 3); ++b) dst[b] = src[b];
  const int ph = (int)(b & 3);  // src + b phase (src aligned)
  const uint32_t* s = reinterpret_cast<const uint32_t*>(src + b - ph);
  for (int64_t k = 0; b + 4 <= n; b += 4, ++k) {
    uint32_t w = s[k];
    if (ph) w = (uint32_t)((((uint64_t)s[k + 1] << 32) | w) >> (8 * ph));
    st32(dst + b, w);
  }
  for (; b < n; ++b) dst[b] = src[b];
}

__device__ __forceinline__ bool is_scalar(int kind) { return kind == KIND_FIXED || kind == KIND_BOOL; }

// DecimalUtility.checkPrecisionAndScale: the unscaled value (decimal128 dwords w, little-
// endian two's complement) has at most `prec` digits, |v| <= 10^prec - 1.
__device__ __forceinline__ bool g_dec_fits(const uint32_t w[4], int prec) {
  const unsigned __int128 u = (unsigned __int128)w[0] | ((unsigned __int128)w[1] << 32) |
                              ((unsigned __int128)w[2] << 64) | ((unsigned __int128)w[3] << 96);
  const bool neg = (w[3] >> 31) != 0;
  const unsigned __int128 mag = neg ? ~u + 1 : u;
  unsigned __int128 lim = 1;
  for (int k = 0; k < prec; ++k) lim *= 10;
  return mag <= lim - 1;
}
__device__ __forceinline__ int elem_size(const GNode& it) { return is_scalar(it.kind) ? it.width : 8; }

// Frame of an open container. STRUCT: children [ch, end) at position pos, the
// child row at `start`. ARRAY: elements k..n-1 of node `item` at positions pos + k,
// the array at `start`. MAP_KEYS / MAP_VALS: the key / value array of map `node`.
enum : int32_t { F_STRUCT = 0, F_ARRAY = 1, F_MAP_KEYS = 2, F_MAP_VALS = 3 };

struct GFrame {
  int32_t type;
  int32_t node;     // STRUCT: the struct node (-1 = the row); ARRAY: unused; MAP_*: the map node
  int32_t ch, end;  // STRUCT: next child, children end; ARRAY / MAP_*: item node, -
  int32_t k, n;     // next ordinal / element, element count (arrays)
  int64_t pos;      // STRUCT: position; arrays: position of element 0
  int32_t start;    // row / array start (record-row relative)
  int32_t header;   // bitmap end (row) or 8 + bitmap (array)
  int32_t elem;     // slot / element bytes
  int32_t off;      // encode: where the value began; decode maps: the value array start
  int32_t slot;     // encode: record-row relative slot to fill when the frame closes (-1: none)
  int32_t rel;      // encode: the slot's relative offset; decode: 1 = present (structs)
};

// ---------------------------------------------------------------------------
// sizes
// ---------------------------------------------------------------------------
template <int D>
__device__ int64_t g_sizes(const GenLaunch& L, int64_t i, bool* overflow) {
  GFrame st[D];
  int sp = 0;
  int64_t total = 0;
  // an array's fixed part; pushes its elements when they may carry var data
  auto array = [&](int item, int64_t e0, int64_t n) {
    const GNode& it = L.nodes[item];
    total += 8 + gbm(n) + gr8(n * elem_size(it));
    if (is_scalar(it.kind) || n == 0) return;
    if (sp == D) { *overflow = true; return; }
    GFrame& f = st[sp++];
    f.type = F_ARRAY;
    f.ch = item;
    f.k = 0;
    f.n = (int32_t)n;
    f.pos = e0;
  };
  auto visit = [&](int node, int64_t pos) {
    const GNode& nd = L.nodes[node];
    const ColumnDev& c = L.cols[node];
    if ((nd.flags & 1) && !gvalid(c.validity, pos)) return;
    if (nd.kind == KIND_BYTES) {
      total += gr8((int64_t)c.offsets[pos + 1] - c.offsets[pos]);
    } else if (nd.kind == KIND_DECIMAL) {
      total += 32;
    } else if (nd.kind == KIND_STRUCT) {
      total += gbm(nd.nchild) + 8LL * nd.nchild;
      if (sp == D) { *overflow = true; return; }
      GFrame& f = st[sp++];
      f.type = F_STRUCT;
      f.ch = node + 1;
      f.end = nd.end;
      f.pos = pos;
    } else if (nd.kind == KIND_LIST || nd.kind == KIND_MAP) {
      const int64_t e0 = c.offsets[pos], n = (int64_t)c.offsets[pos + 1] - e0;
      if (nd.kind == KIND_LIST) {
        array(node + 1, e0, n);
      } else {
        total += 8;
        const int key = node + 1;
        array(key, e0, n);
        array(L.nodes[key].end, e0, n);
      }
    }
  };
  if (L.frame == FORY_FRAME_COLLECTION) {  // [i32 size][the single field's BinaryArray / BinaryMap]
    const ColumnDev& c = L.cols[0];
    const int64_t e0 = c.offsets[i], n = (int64_t)c.offsets[i + 1] - e0;
    total = 4;
    if (L.nodes[0].kind == KIND_LIST) {
      array(1, e0, n);
    } else {
      total += 8;
      array(1, e0, n);
      array(L.nodes[1].end, e0, n);
    }
  } else {
    total = frame_header_bytes(L.frame) + L.fixed_size;
    GFrame& f = st[sp++];
    f.type = F_STRUCT;
    f.ch = 0;
    f.end = L.num_nodes;
    f.pos = i;
  }
  while (sp > 0 && !*overflow) {
    GFrame& f = st[sp - 1];
    if (f.type == F_STRUCT) {
      if (f.ch >= f.end) { --sp; continue; }
      const int ch = f.ch;
      f.ch = L.nodes[ch].end;
      visit(ch, f.pos);
    } else {
      if (f.k >= f.n) { --sp; continue; }
      const int64_t p = f.pos + f.k++;
      visit(f.ch, p);
    }
  }
  return total;
}

// The node table and column views in LDS (every visit reads them; from global they
// add two dependent loads per visit). Plans with more nodes read them from global.
constexpr int kGenLdsNodes = 128;

struct GenTables {
  GNode nodes[kGenLdsNodes];
  ColumnDev cols[kGenLdsNodes];
};

template <bool TAB>
__device__ __forceinline__ GenLaunch gen_tables(const GenLaunch& L, GenTables* t) {
  if (!TAB) return L;
  for (int k = threadIdx.x; k < L.num_nodes; k += kWG) {
    t->nodes[k] = L.nodes[k];
    t->cols[k] = L.cols[k];
  }
  __syncthreads();
  GenLaunch LL = L;
  LL.nodes = t->nodes;
  LL.cols = t->cols;
  return LL;
}

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

// ---------------------------------------------------------------------------
// encode
// ---------------------------------------------------------------------------
template <int D>
__device__ int32_t g_encode(const GenLaunch& L, uint8_t* row, int64_t i) {
  GFrame st[D];
  int sp = 0;
  int32_t wi = 0;
  bool ok = true;
  bool prec_ok = true;  // every decimal within its precision
  // BinaryArrayWriter.reset(n) at wi (+ the zeroed bitmap / elements of a fresh buffer)
  auto open_array = [&](int type, int node, int item, int64_t e0, int64_t n, int32_t slot, int32_t rel, int32_t off) {
    if (sp == D) { ok = false; return; }
    const int es = elem_size(L.nodes[item]);
    GFrame& f = st[sp++];
    f.type = type;
    f.node = node;
    f.ch = item;
    f.k = 0;
    f.n = (int32_t)n;
    f.pos = e0;
    f.start = wi;
    f.header = 8 + gbm(n);
    f.elem = es;
    f.off = off;
    f.slot = slot;
    f.rel = rel;
    const int64_t data = gr8(n * es);
    gput(row + wi, (uint64_t)n, 8);
    gzero(row + wi + 8, f.header - 8 + data);
    wi += (int32_t)(f.header + data);
  };
  // serializeFor of node at (writer frame w, ordinal k, position pos)
  auto visit = [&](int node, const GFrame& w, int32_t k, int64_t pos) {
    const GNode& nd = L.nodes[node];
    const ColumnDev& c = L.cols[node];
    const int32_t bm = w.type == F_STRUCT ? 0 : 8;
    if ((nd.flags & 1) && !gvalid(c.validity, pos)) {  // setNullAt: bit set, slot left zero
      uint8_t* b = row + w.start + bm + (k >> 3);
      *b = (uint8_t)(*b | (1u << (k & 7)));
      return;
    }
    const int32_t slot = w.start + w.header + k * w.elem;
    const int32_t rel = wi - w.start;
    switch (nd.kind) {
      case KIND_FIXED:
      case KIND_BOOL: {
        uint64_t v = load_elem(c.values, nd.width, pos);
        if (nd.kind == KIND_BOOL) v = v ? 1 : 0;  // MemoryBuffer.putBoolean
        // rows: putInt64(slot, 0) then the value (zero-extended); arrays: the element only
        gput(row + slot, v, bm ? nd.width : 8);
        return;
      }
      case KIND_BYTES: {
        const int64_t s0 = c.offsets[pos], n = (int64_t)c.offsets[pos + 1] - s0;
        g_put_bytes(row + wi, c.values + s0, n);
        gput(row + slot, ((uint64_t)rel << 32) | (uint32_t)n, 8);
        wi += (int32_t)gr8(n);
        return;
      }
      case KIND_DECIMAL: {  // BinaryWriter.writeDecimal: checkPrecisionAndScale, 32 LE bytes, (rel, 32)
        const uint8_t* v = c.values + 16 * pos;
        const uint32_t w[4] = {ld32(v), ld32(v + 4), ld32(v + 8), ld32(v + 12)};
        if (!g_dec_fits(w, nd.prec)) {
          prec_ok = false;
          return;
        }
        const uint32_t ext = (w[3] >> 31) ? 0xffffffffu : 0u;  // sign extension to DECIMAL_BYTE_LENGTH
        for (int q = 0; q < 4; ++q) st32(row + wi + 4 * q, w[q]);
        for (int q = 4; q < 8; ++q) st32(row + wi + 4 * q, ext);
        gput(row + slot, ((uint64_t)rel << 32) | 32u, 8);
        wi += 32;
        return;
      }
      case KIND_STRUCT: {  // BinaryRowWriter.reset (+ slots of a fresh buffer)
        if (sp == D) { ok = false; return; }
        GFrame& f = st[sp++];
        f.type = F_STRUCT;
        f.node = node;
        f.ch = node + 1;
        f.end = nd.end;
        f.k = 0;
        f.pos = pos;
        f.start = wi;
        f.header = gbm(nd.nchild);
        f.elem = 8;
        f.off = wi;
        f.slot = slot;
        f.rel = rel;
        gzero(row + wi, f.header + 8LL * nd.nchild);
        wi += f.header + 8 * nd.nchild;
        return;
      }
      case KIND_LIST: {
        const int64_t e0 = c.offsets[pos], n = (int64_t)c.offsets[pos + 1] - e0;
        open_array(F_ARRAY, node, node + 1, e0, n, slot, rel, wi);
        return;
      }
      case KIND_MAP: {  // serializeForMap: reserve 8 bytes, key array, back-patch, value array
        const int64_t e0 = c.offsets[pos], n = (int64_t)c.offsets[pos + 1] - e0;
        const int32_t off = wi;
        wi += 8;
        open_array(F_MAP_KEYS, node, node + 1, e0, n, slot, rel, off);
        return;
      }
      default: return;
    }
  };
  if (L.frame == FORY_FRAME_COLLECTION) {  // ArrayEncoder / MapEncoder.encode(MemoryBuffer, T)
    const ColumnDev& c = L.cols[0];
    const int64_t e0 = c.offsets[i], n = (int64_t)c.offsets[i + 1] - e0;
    if (L.nodes[0].kind == KIND_LIST) {
      open_array(F_ARRAY, 0, 1, e0, n, -1, 0, 0);
    } else {
      wi = 8;
      open_array(F_MAP_KEYS, 0, 1, e0, n, -1, 0, 0);
    }
  } else {  // BinaryRowWriter.reset
    GFrame& f = st[sp++];
    f.type = F_STRUCT;
    f.node = -1;
    f.ch = 0;
    f.end = L.num_nodes;
    f.k = 0;
    f.pos = i;
    f.start = 0;
    f.header = L.bitmap_bytes;
    f.elem = 8;
    f.slot = -1;
    gzero(row, L.fixed_size);
    wi = L.fixed_size;
  }
  while (sp > 0 && ok) {
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
      const GFrame w = f;  // visit may push (the stack slot above f)
      visit(node, w, k, pos);
      continue;
    }
    if (f.type == F_MAP_KEYS) {  // keys done: back-patch their size, then the value array
      gput(row + f.off, (uint64_t)(wi - f.start), 8);
      const GFrame m = f;
      --sp;
      open_array(F_MAP_VALS, m.node, L.nodes[m.ch].end, m.pos, m.n, m.slot, m.rel, m.off);
      continue;
    }
    if (f.slot >= 0) gput(row + f.slot, ((uint64_t)(uint32_t)f.rel << 32) | (uint32_t)(wi - f.off), 8);
    --sp;
  }
  return !ok ? FORY_ERR_ENCODER : (prec_ok ? 0 : FORY_ERR_UNSUPPORTED);
}

template <int D, bool TAB>
__global__ __launch_bounds__(kWG) void gen_encode_kernel(GenLaunch L0, const int64_t* __restrict__ offs,
                                                         uint8_t* __restrict__ out, int64_t capacity,
                                                         int32_t* status) {
  __shared__ GenTables tabs;
  const GenLaunch L = gen_tables<TAB>(L0, &tabs);
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i >= L.num_rows) return;
  const int64_t beg = offs[i], end = offs[i + 1];
  if (end > capacity || beg < 0 || end < beg) {
    set_status(status, FORY_ERR_CAPACITY);
    return;
  }
  const int64_t size = end - beg;
  const int hdr = L.frame == FORY_FRAME_COLLECTION ? 4 : frame_header_bytes(L.frame);
  if (size - hdr > 0x7fffffffLL || size < hdr) {  // rows index with int (MemoryBuffer), or sizes overflowed
    set_status(status, FORY_ERR_CAPACITY);
    return;
  }
  uint8_t* frame = out + beg;
  if (hdr == 12 || hdr == 4) st32(frame, (uint32_t)(size - 4));  // Encoders.encode(MemoryBuffer, T) size field
  if (hdr == 12) gput(frame + 4, (uint64_t)L.schema_hash, 8);    // [i32 8+rowSize][i64 hash]
  if (hdr == 8) gput(frame, (uint64_t)L.schema_hash, 8);         // Encoder.encode(T): [i64 hash]
  const int32_t err = g_encode<D>(L, frame + hdr, i);
  if (err) set_status(status, err);
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
      if (!isnull) {
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
