// gen_device.h — device side of the tree engine shared by the per-lane kernels
// (generic.hip) and the columnar engine (treecol.hip): row-byte helpers, the per-lane
// sizes / encode walks (g_sizes, g_encode) and their LDS node tables.
#pragma once

#include "kcommon.h"

namespace fory_amd {
namespace {

__device__ __forceinline__ int32_t gbm(int64_t n) { return (int32_t)(((n + 63) >> 6) << 3); }
__device__ __forceinline__ int64_t gr8(int64_t n) { return (n + 7) & ~int64_t(7); }

__device__ __forceinline__ bool gvalid(const uint8_t* validity, int64_t i) {
  return !validity || ((gp(validity)[i >> 3] >> (i & 7)) & 1);
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
  const GAS uint32_t* s = gp(reinterpret_cast<const uint32_t*>(src - sh));  // (an Arrow column)
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
__device__ __forceinline__ void g_get_bytes(uint8_t* dst0, const uint8_t* src, int64_t n) {
  GAS uint8_t* dst = gp(dst0);  // (an Arrow values buffer)
  int64_t b = 0;
  for (; b < n && (reinterpret_cast<uintptr_t>(dst0 + b) & 3); ++b) dst[b] = src[b];
  const int ph = (int)(b & 3);  // src + b phase (src aligned)
  const uint32_t* s = reinterpret_cast<const uint32_t*>(src + b - ph);
  for (int64_t k = 0; b + 4 <= n; b += 4, ++k) {
    uint32_t w = s[k];
    if (ph) w = (uint32_t)((((uint64_t)s[k + 1] << 32) | w) >> (8 * ph));
    *reinterpret_cast<GAS uint32_t*>(dst + b) = w;
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

// A decimal node that holds a java.math.BigInteger field (descriptor FORY_DECIMAL_BIGINTEGER).
__device__ __forceinline__ bool g_bigint(const GNode& nd) { return nd.kind == KIND_DECIMAL && nd.prec == 0; }

__device__ __forceinline__ void g_load_dec(const uint8_t* values, int64_t k, uint32_t w[4]) {
  const GAS uint32_t* x = gp(reinterpret_cast<const uint32_t*>(values + 16 * k));  // (an Arrow decimal column)
  w[0] = x[0];
  w[1] = x[1];
  w[2] = x[2];
  w[3] = x[3];
}

// BigInteger.toByteArray().length of a decimal128 value: bitLength() / 8 + 1, where bitLength
// counts the bits of the minimal two's complement without the sign (of ~v for negatives):
// 0 -> 1 (00), -1 -> 1 (ff), 128 -> 2 (00 80), -129 -> 2 (ff 7f), +-2^127 -> 16.
__device__ __forceinline__ int g_bigint_len(const uint32_t w[4]) {
  const uint32_t s = (w[3] >> 31) ? 0xffffffffu : 0u;
  int bits = 0;
  for (int q = 3; q >= 0; --q) {
    const uint32_t x = w[q] ^ s;
    if (x) {
      bits = 32 * q + 32 - __clz(x);
      break;
    }
  }
  return bits / 8 + 1;
}
// Row bytes a BigInteger value takes: writeUnaligned's round8(len).
__device__ __forceinline__ int64_t g_bigint_bytes(const uint32_t w[4]) { return gr8(g_bigint_len(w)); }

// toByteArray()'s len bytes (big-endian, most significant first) + zero padding to 8 at a
// 4-byte aligned dst (BinaryWriter.writeUnaligned + zeroOutPaddingBytes).
__device__ __forceinline__ void g_put_bigint(uint8_t* dst, const uint32_t w[4], int len) {
  // the value's 16 bytes big-endian in memory order, shifted so the last len of them lead
  unsigned __int128 b = (unsigned __int128)__builtin_bswap32(w[3]) |
                        ((unsigned __int128)__builtin_bswap32(w[2]) << 32) |
                        ((unsigned __int128)__builtin_bswap32(w[1]) << 64) |
                        ((unsigned __int128)__builtin_bswap32(w[0]) << 96);
  b >>= 8 * (16 - len);
  const int nw = (int)(gr8(len) >> 2);
  for (int q = 0; q < nw; ++q) st32(dst + 4 * q, (uint32_t)(b >> (32 * q)));
}

// new BigInteger(bytes) of the len row bytes at src into decimal128 dwords: sign-extended
// big-endian. len outside 1..16 does not fit a decimal128 (0: Java's "Zero length
// BigInteger"): returns false.
__device__ __forceinline__ bool g_get_bigint(const uint8_t* src, int64_t len, uint32_t w[4]) {
  if (len < 1 || len > 16) return false;
  unsigned __int128 v = (src[0] & 0x80) ? ~(unsigned __int128)0 : 0;
  for (int j = 0; j < (int)len; ++j) v = (v << 8) | src[j];
  for (int q = 0; q < 4; ++q) w[q] = (uint32_t)(v >> (32 * q));
  return true;
}

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
      total += gr8((int64_t)gp(c.offsets)[pos + 1] - gp(c.offsets)[pos]);
    } else if (nd.kind == KIND_DECIMAL) {
      if (g_bigint(nd)) {
        uint32_t w[4];
        g_load_dec(c.values, pos, w);
        total += g_bigint_bytes(w);
      } else {
        total += 32;
      }
    } else if (nd.kind == KIND_STRUCT) {
      total += gbm(nd.nchild) + 8LL * nd.nchild;
      if (sp == D) { *overflow = true; return; }
      GFrame& f = st[sp++];
      f.type = F_STRUCT;
      f.ch = node + 1;
      f.end = nd.end;
      f.pos = pos;
    } else if (nd.kind == KIND_LIST || nd.kind == KIND_MAP) {
      const int64_t e0 = gp(c.offsets)[pos], n = (int64_t)gp(c.offsets)[pos + 1] - e0;
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
    const int64_t e0 = gp(c.offsets)[i], n = (int64_t)gp(c.offsets)[i + 1] - e0;
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
        const int64_t s0 = gp(c.offsets)[pos], n = (int64_t)gp(c.offsets)[pos + 1] - s0;
        g_put_bytes(row + wi, c.values + s0, n);
        gput(row + slot, ((uint64_t)rel << 32) | (uint32_t)n, 8);
        wi += (int32_t)gr8(n);
        return;
      }
      case KIND_DECIMAL: {  // BinaryWriter.writeDecimal: checkPrecisionAndScale, 32 LE bytes, (rel, 32)
        const uint8_t* v = c.values + 16 * pos;
        const uint32_t w[4] = {ld32(v), ld32(v + 4), ld32(v + 8), ld32(v + 12)};
        if (g_bigint(nd)) {  // BigInteger: write(ordinal, value.toByteArray()) -> writeUnaligned
          const int len = g_bigint_len(w);
          g_put_bigint(row + wi, w, len);
          gput(row + slot, ((uint64_t)rel << 32) | (uint32_t)len, 8);
          wi += (int32_t)gr8(len);
          return;
        }
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
        const int64_t e0 = gp(c.offsets)[pos], n = (int64_t)gp(c.offsets)[pos + 1] - e0;
        open_array(F_ARRAY, node, node + 1, e0, n, slot, rel, wi);
        return;
      }
      case KIND_MAP: {  // serializeForMap: reserve 8 bytes, key array, back-patch, value array
        const int64_t e0 = gp(c.offsets)[pos], n = (int64_t)gp(c.offsets)[pos + 1] - e0;
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
    const int64_t e0 = gp(c.offsets)[i], n = (int64_t)gp(c.offsets)[i + 1] - e0;
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

// One record of the per-lane encoder at offs[i] (frame header + row): gen_encode_kernel's
// body, also the columnar writer's path for tiles too large for its LDS image.
template <int D>
__device__ void gen_encode_one(const GenLaunch& L, const int64_t* __restrict__ offs, uint8_t* __restrict__ out,
                               int64_t capacity, int32_t* status, int64_t i) {
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

}  // namespace
}  // namespace fory_amd
