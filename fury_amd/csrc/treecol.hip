// treecol.hip — the columnar tree engine: encode of any nesting as per-node passes.
//
// The per-lane engine (generic.hip) walks one record per lane, serially through a
// frame stack, so a wave runs as long as its deepest record and every column access is
// a lane-private gather. Here the same bytes (BaseBinaryEncoderBuilder.serializeFor,
// :236-351 arrays, :370-427 maps, :436-490 beans) come from three kinds of passes over
// instance columns (one instance = one element of a schema node's column):
//   sizes   bottom-up, one launch per var node (children first), lane per instance:
//           A[c][j] = the bytes instance j adds to its parent — strings round8(len),
//           decimals 32, beans bitmap + 8 x fields + their var children, arrays
//           8 + bitmap + round8(n x elemSize) + their var items (a difference of the
//           items' scanned sizes), maps 8 + key array + value array. Item nodes (list
//           items, map keys / values) are scanned in place: A[x][k] = bytes of the
//           items before k, A[x][m] = all of them.
//   rows    row / frame size = header + fixed part + the top-level var fields' sizes;
//           scanned into the row offsets (encoded_size's output).
//   write   one workgroup per tile of rows: the tile's bytes [offs[r0], offs[r1]) are
//           assembled in an LDS image and stored once, coalesced. Phase 0 writes the
//           rows' frame headers and fixed parts; phase d the instances of depth-d var
//           nodes: each reads its position (handed down by its parent in phase d-1),
//           writes its own fixed part (bean slots, array header / bitmap / elements,
//           map key-array size, string bytes, decimal) and hands its var children their
//           positions. Tiles too large for the image (a row bigger than the tile
//           budget) are encoded by the per-lane engine instead, row by row.
// The instance ranges of a tile follow from the row range: a struct child has its
// parent's range, items the parent's offsets at the range ends.
#include "gen_device.h"

namespace fory_amd {
namespace {

constexpr int kTcWG = 256;

__device__ __forceinline__ bool tc_is_var(int kind) { return !is_scalar(kind); }

__device__ __forceinline__ int64_t tc_clamp(int64_t k, int64_t m) { return k < 0 ? 0 : (k > m ? m : k); }

// Bytes of the array of items x in [o0, o1): BinaryArrayWriter.reset(n) fixed part + var items.
__device__ __forceinline__ int64_t tc_array_bytes(const GenLaunch& L, const TcTables* T, int x, int64_t o0,
                                                  int64_t o1) {
  const GNode it = L.nodes[x];
  const int64_t n = o1 - o0;
  int64_t b = 8 + gbm(n) + gr8(n * elem_size(it));
  if (tc_is_var(it.kind)) b += T->A[x][o1] - T->A[x][o0];
  return b;
}

// Item range [o0, o1) of container instance j of node c (offsets clamped to the items' column).
__device__ __forceinline__ void tc_items(const GenLaunch& L, const TcTables* T, int c, int64_t j, int64_t* o0,
                                         int64_t* o1) {
  const int32_t* off = L.cols[c].offsets;
  const int64_t mx = T->m[c + 1];
  const int64_t a = tc_clamp(off[j], mx), b = tc_clamp(off[j + 1], mx);
  *o0 = a;
  *o1 = b < a ? a : b;
}

// ---------------------------------------------------------------------------
// sizes
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kTcWG) void tc_sizes_kernel(GenLaunch L, const TcTables* __restrict__ T, int c,
                                                         int64_t m, int root_coll) {
  const int64_t j = (int64_t)blockIdx.x * kTcWG + threadIdx.x;
  if (j >= m) return;
  const GNode nd = L.nodes[c];
  const ColumnDev col = L.cols[c];
  int64_t s = 0;
  if (root_coll || !(nd.flags & 1) || gvalid(col.validity, j)) {
    switch (nd.kind) {
      case KIND_BYTES: s = gr8((int64_t)col.offsets[j + 1] - col.offsets[j]); break;
      case KIND_DECIMAL: s = 32; break;
      case KIND_STRUCT:
        s = gbm(nd.nchild) + 8LL * nd.nchild;
        for (int ch = c + 1; ch < nd.end; ch = L.nodes[ch].end)
          if (tc_is_var(L.nodes[ch].kind)) s += T->A[ch][j];
        break;
      case KIND_LIST:
      case KIND_MAP: {
        int64_t o0, o1;
        tc_items(L, T, c, j, &o0, &o1);
        if (nd.kind == KIND_LIST) s = tc_array_bytes(L, T, c + 1, o0, o1);
        else s = 8 + tc_array_bytes(L, T, c + 1, o0, o1) + tc_array_bytes(L, T, L.nodes[c + 1].end, o0, o1);
        break;
      }
      default: break;
    }
  }
  T->A[c][j] = s;
}

__global__ __launch_bounds__(kTcWG) void tc_rows_kernel(GenLaunch L, const TcTables* __restrict__ T,
                                                        int64_t* __restrict__ sizes) {
  const int64_t i = (int64_t)blockIdx.x * kTcWG + threadIdx.x;
  if (i >= L.num_rows) return;
  int64_t s;
  if (L.frame == FORY_FRAME_COLLECTION) {
    s = 4 + T->A[0][i];
  } else {
    s = frame_header_bytes(L.frame) + L.fixed_size;
    for (int t = 0; t < L.num_nodes; t = L.nodes[t].end)
      if (tc_is_var(L.nodes[t].kind)) s += T->A[t][i];
  }
  sizes[i] = s;
}

// ---------------------------------------------------------------------------
// write
// ---------------------------------------------------------------------------
// One tile's LDS state: the image (I = the byte of the tile's first position, 16-byte
// phase of the output kept), per entry its instance range [lo, lo + cnt), per var entry
// the start of its position entries in pl (image-relative, -1 = absent / null) and, for
// lists / maps, aux: each instance's first item relative to the items' range start.
struct TcTile {
  uint8_t* I;
  int32_t* pl;
  int32_t* aux;
  const int64_t* lo;
  const int32_t* cnt;
  const int32_t* pb;
  int32_t len;  // image bytes
};

// The `w` low bytes of v at p (4-byte aligned for w = 8; naturally aligned otherwise).
__device__ __forceinline__ void tc_put(uint8_t* p, uint64_t v, int w) {
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

// Hands var child / item instance k of node `node` its position `at` (if in the tile).
__device__ __forceinline__ void tc_hand(const TcTables* T, const TcTile& t, int node, int64_t k, int32_t at) {
  const int v = T->vidx[node];
  const int64_t e = k - t.lo[v];
  if (e >= 0 && e < t.cnt[v]) t.pl[t.pb[v] + e] = at;
}

// Slot size field of a var value: a string's byte length, else its bytes (decimals 32).
__device__ __forceinline__ uint32_t tc_slot_size(const GNode& nd, const ColumnDev& col, int64_t k, int64_t bytes) {
  if (nd.kind == KIND_BYTES) return (uint32_t)(col.offsets[k + 1] - col.offsets[k]);
  return (uint32_t)bytes;
}

// A bean's (or the row's) fixed part at P: null bits, scalar slots (the value's bytes,
// zero-extended: the image is zeroed), var slots (rel, size) + their children's positions.
// Fields [first, end) of the schema, instance k. Returns false when they do not fit.
__device__ __forceinline__ bool tc_fields(const GenLaunch& L, const TcTables* T, const TcTile& t, int first,
                                          int end, int nf, int bm, int64_t k, int32_t P) {
  int32_t at = P + bm + 8 * nf;
  if (at > t.len) return false;
  int q = 0;
  for (int ch = first; ch < end; ch = L.nodes[ch].end, ++q) {
    const GNode nd = L.nodes[ch];
    const ColumnDev col = L.cols[ch];
    uint8_t* slot = t.I + P + bm + 8 * q;
    if ((nd.flags & 1) && !gvalid(col.validity, k)) {  // setNullAt: bit, slot zero
      t.I[P + (q >> 3)] |= (uint8_t)(1u << (q & 7));
      continue;
    }
    if (is_scalar(nd.kind)) {
      uint64_t v = load_elem(col.values, nd.width, k);
      if (nd.kind == KIND_BOOL) v = v ? 1 : 0;
      tc_put(slot, v, nd.width);
      continue;
    }
    const int64_t S = T->A[ch][k];
    if (S < 0 || at + S > t.len) return false;
    st32(slot, tc_slot_size(nd, col, k, S));
    st32(slot + 4, (uint32_t)(at - P));
    tc_hand(T, t, ch, k, at);
    at += (int32_t)S;
  }
  return true;
}

// aux of list / map instance g (entry v, node c): its first item relative to the tile's items.
__device__ __forceinline__ int64_t tc_aux(const GenLaunch& L, const TcTables* T, const TcTile& t, int v, int c,
                                          int g, int64_t k, int64_t* o1 = nullptr) {
  int64_t o0, e1;
  tc_items(L, T, c, k, &o0, &e1);
  t.aux[t.pb[v] + g] = (int32_t)(o0 - t.lo[T->vidx[c + 1]]);
  if (o1) *o1 = e1;
  return o0;
}

// A var instance's own bytes (step A of a depth): string bytes, a decimal, a bean's fixed
// part, an array's / map's headers (their elements are step B's). g: the instance's
// index in the tile, v its entry.
__device__ __forceinline__ int32_t tc_head(const GenLaunch& L, const TcTables* T, const TcTile& t, int v, int c,
                                           int g, int64_t k, int32_t P) {
  const GNode nd = L.nodes[c];
  const ColumnDev col = L.cols[c];
  switch (nd.kind) {
    case KIND_BYTES: {  // writeUnaligned + zeroOutPaddingBytes
      const int64_t s0 = col.offsets[k], n = (int64_t)col.offsets[k + 1] - s0;
      if (n < 0 || P + gr8(n) > t.len) return FORY_ERR_ENCODER;
      g_put_bytes(t.I + P, col.values + s0, n);
      return 0;
    }
    case KIND_DECIMAL: {  // BinaryWriter.writeDecimal
      if (P + 32 > t.len) return FORY_ERR_ENCODER;
      const uint8_t* x = col.values + 16 * k;
      const uint32_t w[4] = {ld32(x), ld32(x + 4), ld32(x + 8), ld32(x + 12)};
      if (!g_dec_fits(w, nd.prec)) return FORY_ERR_UNSUPPORTED;
      const uint32_t ext = (w[3] >> 31) ? 0xffffffffu : 0u;
      for (int q = 0; q < 4; ++q) st32(t.I + P + 4 * q, w[q]);
      for (int q = 4; q < 8; ++q) st32(t.I + P + 4 * q, ext);
      return 0;
    }
    case KIND_STRUCT:
      return tc_fields(L, T, t, c + 1, nd.end, nd.nchild, gbm(nd.nchild), k, P) ? 0 : FORY_ERR_ENCODER;
    case KIND_LIST:
    case KIND_MAP: {  // [i64 n] | [i64 key array bytes][i64 n ...keys][i64 n ...values]
      int64_t o1;
      const int64_t o0 = tc_aux(L, T, t, v, c, g, k, &o1);
      const int64_t n = o1 - o0;
      const int key = c + 1;
      if (nd.kind == KIND_LIST) {
        if (P + 8 + gbm(n) + gr8(n * elem_size(L.nodes[key])) > t.len) return FORY_ERR_ENCODER;
        tc_put(t.I + P, (uint64_t)n, 8);
        return 0;
      }
      const int val = L.nodes[key].end;
      const int64_t kb = tc_array_bytes(L, T, key, o0, o1);
      if (kb < 0 || P + 8 + kb + 8 + gbm(n) + gr8(n * elem_size(L.nodes[val])) > t.len) return FORY_ERR_ENCODER;
      tc_put(t.I + P, (uint64_t)kb, 8);
      tc_put(t.I + P + 8, (uint64_t)n, 8);
      tc_put(t.I + P + 8 + kb, (uint64_t)n, 8);
      return 0;
    }
    default: return 0;
  }
}

// Item i (tile-relative) of entry xe under list / map entry v (step B): its element —
// a null bit, a scalar, or a var item's slot + position. which: 0 list items, 1 keys,
// 2 values.
__device__ __forceinline__ int32_t tc_item(const GenLaunch& L, const TcTables* T, const TcTile& t, int v, int xe,
                                           int x, int which, int i) {
  const int cv = t.cnt[v];
  const int32_t* aux = t.aux + t.pb[v];
  int a = 0, b = cv - 1;  // the last instance whose items start at or before i
  while (a < b) {
    const int mid = (a + b + 1) >> 1;
    if (aux[mid] <= i) a = mid;
    else b = mid - 1;
  }
  const int32_t P = t.pl[t.pb[v] + a];
  if (P < 0) return 0;  // a null / absent container
  const int32_t o0 = aux[a], o1 = a + 1 < cv ? aux[a + 1] : t.cnt[xe];
  const int64_t n = o1 - o0;
  const int64_t q = i - o0;
  const int32_t Pa = which == 0 ? P : (which == 1 ? P + 8 : P + 8 + (int32_t)ld32(t.I + P));
  const GNode it = L.nodes[x];
  const ColumnDev col = L.cols[x];
  const int es = elem_size(it);
  const int32_t hb = 8 + gbm(n);
  if (q < 0 || q >= n || Pa + hb + gr8(n * es) > t.len) return FORY_ERR_ENCODER;
  const int64_t e = t.lo[xe] + i;
  if ((it.flags & 1) && !gvalid(col.validity, e)) {  // setNullAt: the element bit
    atomicOr(reinterpret_cast<uint32_t*>(t.I + Pa + 8) + (q >> 5), 1u << (q & 31));
    return 0;
  }
  if (is_scalar(it.kind)) {
    uint64_t val = load_elem(col.values, es, e);
    if (it.kind == KIND_BOOL) val = val ? 1 : 0;
    tc_put(t.I + Pa + hb + q * es, val, es);
    return 0;
  }
  const int64_t* A = T->A[x];
  const int64_t S = A[e + 1] - A[e];
  const int64_t at = Pa + hb + gr8(n * 8) + (A[e] - A[t.lo[xe] + o0]);
  if (S < 0 || at < 0 || at + S > t.len) return FORY_ERR_ENCODER;
  uint8_t* slot = t.I + Pa + hb + 8 * q;
  st32(slot, tc_slot_size(it, col, e, S));
  st32(slot + 4, (uint32_t)(at - Pa));
  tc_hand(T, t, x, e, (int32_t)at);
  return 0;
}

// Row / frame i: header, then the row's fixed part (or the collection's position).
__device__ __forceinline__ void tc_row(const GenLaunch& L, const TcTables* T, const TcTile& t,
                                       const int64_t* offs, int64_t base, int64_t i, int32_t* status) {
  const int64_t fb = offs[i] - base, fe = offs[i + 1] - base;
  const int coll = L.frame == FORY_FRAME_COLLECTION;
  const int hdr = coll ? 4 : frame_header_bytes(L.frame);
  const int64_t size = fe - fb;
  if (fb < 0 || fe > t.len || size < hdr || size - hdr > 0x7fffffffLL) {
    set_status(status, FORY_ERR_CAPACITY);
    return;
  }
  uint8_t* f = t.I + fb;
  if (coll) {
    if (4 + T->A[0][i] > size) {  // offsets not from these columns' sizes
      set_status(status, FORY_ERR_CAPACITY);
      return;
    }
    st32(f, (uint32_t)(size - 4));
    tc_hand(T, t, 0, i, (int32_t)fb + 4);
    return;
  }
  int64_t need = hdr + L.fixed_size;
  for (int c = 0; c < L.num_nodes; c = L.nodes[c].end)
    if (tc_is_var(L.nodes[c].kind)) need += T->A[c][i];
  if (need > size) {
    set_status(status, FORY_ERR_CAPACITY);
    return;
  }
  if (hdr == 12) {  // Encoders.encode(MemoryBuffer, T): [i32 8 + rowSize][i64 hash]
    st32(f, (uint32_t)(size - 4));
    tc_put(f + 4, (uint64_t)L.schema_hash, 8);
  } else if (hdr == 8) {  // Encoder.encode(T): [i64 hash]
    tc_put(f, (uint64_t)L.schema_hash, 8);
  }
  const int nf = (L.fixed_size - L.bitmap_bytes) / 8;
  if (!tc_fields(L, T, t, 0, L.num_nodes, nf, L.bitmap_bytes, i, (int32_t)(fb + hdr)))
    set_status(status, FORY_ERR_ENCODER);
}

__global__ __launch_bounds__(kTcWG) void tc_tiles_kernel(TcLaunch W, const int64_t* __restrict__ offs) {
  const int64_t i = (int64_t)blockIdx.x * kTcWG + threadIdx.x;
  const int64_t n = W.g.num_rows;
  if (i > n) return;
  const int64_t B = W.tile_bytes;
  const int64_t prev = i == 0 ? -1 : offs[i - 1];
  int64_t t0 = prev < 0 ? 0 : prev / B + 1;  // tiles t with prev < t x B <= offs[i]
  int64_t t1 = i == n ? W.ntiles : offs[i] / B;
  if (t1 > W.ntiles) t1 = W.ntiles;
  for (int64_t t = t0; t <= t1; ++t) W.tiles[t] = i;
}

template <int D>
__global__ __launch_bounds__(kTcWG) void tc_encode_kernel(TcLaunch W, const int64_t* __restrict__ offs,
                                                          uint8_t* __restrict__ out, int64_t capacity,
                                                          int32_t* status) {
  __shared__ __attribute__((aligned(16))) uint8_t s_img[kTcImg + 16];
  __shared__ int32_t s_pl[kTcPl], s_aux[kTcPl];
  __shared__ int64_t s_lo[kTcMaxNodes];
  __shared__ int32_t s_cnt[kTcMaxNodes], s_pb[kTcMaxNodes];
  __shared__ int64_t s_base, s_end;
  __shared__ int32_t s_mode, s_tot;
  const GenLaunch& L = W.g;
  const TcTables* T = W.T;
  const int tid = threadIdx.x;
  const int64_t r0 = W.tiles[blockIdx.x], r1 = W.tiles[blockIdx.x + 1];
  if (r0 >= r1) return;  // no row starts in this tile's bytes
  if (r0 < 0 || r1 > L.num_rows) {  // offsets not ascending
    if (tid == 0) set_status(status, FORY_ERR_CAPACITY);
    return;
  }
  if (tid == 0) {
    s_base = offs[r0];
    s_end = offs[r1];
  }
  // instance ranges, depth by depth (an item range reads the parent's offsets)
  const int depths = T->depths;
  for (int d = 1; d <= depths; ++d) {
    for (int v = T->phase[d - 1] + tid; v < T->phase[d]; v += kTcWG) {
      const TcVar tv = T->var[v];
      int64_t lo, hi;
      if (tv.parent < 0) {
        lo = r0;
        hi = r1;
      } else if (!tv.items) {
        lo = s_lo[tv.parent];
        hi = lo + s_cnt[tv.parent];
      } else {
        const int32_t* po = L.cols[T->var[tv.parent].node].offsets;
        const int64_t mx = T->m[tv.node], a = s_lo[tv.parent];
        lo = tc_clamp(po[a], mx);
        hi = tc_clamp(po[a + s_cnt[tv.parent]], mx);
        if (hi < lo) hi = lo;
      }
      s_lo[v] = lo;
      s_cnt[v] = hi - lo > (1 << 30) ? (1 << 30) : (int32_t)(hi - lo);
    }
    __syncthreads();
  }
  if (tid == 0) {
    int32_t tot = 0;
    bool fit = true;
    for (int v = 0; v < T->nvar; ++v) {
      s_pb[v] = tot;
      if (T->var[v].var) tot += s_cnt[v];
      if (s_cnt[v] == (1 << 30) || tot > kTcPl) {
        fit = false;
        tot = kTcPl;
      }
    }
    const int64_t base = s_base, end = s_end;
    int mode = 0;
    if (base < 0 || end < base || end > capacity) {
      set_status(status, FORY_ERR_CAPACITY);
      mode = 2;
    } else if (!fit || ((base | end) & 3) ||
               end - base + (int64_t)((reinterpret_cast<uintptr_t>(out) + base) & 15) > kTcImg) {
      mode = 1;
    }
    s_mode = mode;
    s_tot = tot;
  }
  __syncthreads();
  const int mode = s_mode;
  if (mode == 2) return;
  if (mode == 1) {  // too large for the image: the per-lane engine, row by row
    for (int64_t i = r0 + tid; i < r1; i += kTcWG) gen_encode_one<D>(L, offs, out, capacity, status, i);
    return;
  }
  const int64_t base = s_base;
  const int mis = (int)((reinterpret_cast<uintptr_t>(out) + base) & 15);
  const int32_t len = (int32_t)(s_end - base);
  const int zn = (mis + len + 15) >> 4;
  for (int q = tid; q < zn; q += kTcWG) reinterpret_cast<u32x4*>(s_img)[q] = u32x4{0u, 0u, 0u, 0u};
  for (int q = tid; q < s_tot; q += kTcWG) s_pl[q] = -1;
  __syncthreads();
  TcTile t;
  t.I = s_img + mis;
  t.pl = s_pl;
  t.aux = s_aux;
  t.lo = s_lo;
  t.cnt = s_cnt;
  t.pb = s_pb;
  t.len = len;
  for (int64_t i = r0 + tid; i < r1; i += kTcWG) tc_row(L, T, t, offs, base, i, status);
  __syncthreads();
  for (int d = 1; d <= depths; ++d) {
    const int v0 = T->phase[d - 1], v1 = T->phase[d];
    // A: the depth's var instances (rot spreads the nodes over the waves)
    int rot = 0;
    for (int v = v0; v < v1; ++v) {
      const TcVar tv = T->var[v];
      if (!tv.var) continue;
      const int cnt = s_cnt[v];
      const int32_t* pl = s_pl + s_pb[v];
      const int kind = L.nodes[tv.node].kind;
      const bool cont = kind == KIND_LIST || kind == KIND_MAP;
      for (int g = (tid - rot) & (kTcWG - 1); g < cnt; g += kTcWG) {
        const int32_t P = pl[g];
        if (P < 0) {  // a null / absent container still delimits the items' search
          if (cont) tc_aux(L, T, t, v, tv.node, g, s_lo[v] + g);
          continue;
        }
        const int32_t err = tc_head(L, T, t, v, tv.node, g, s_lo[v] + g, P);
        if (err) set_status(status, err);
      }
      rot = (rot + cnt) & (kTcWG - 1);
    }
    __syncthreads();
    // B: the elements of the depth's arrays and maps, item-parallel
    bool any = false;
    for (int v = v0; v < v1; ++v) {
      const TcVar tv = T->var[v];
      if (!tv.var) continue;
      const int kind = L.nodes[tv.node].kind;
      if (kind != KIND_LIST && kind != KIND_MAP) continue;
      any = true;
      for (int which = kind == KIND_LIST ? 0 : 1; which <= (kind == KIND_LIST ? 0 : 2); ++which) {
        const int x = which == 2 ? L.nodes[tv.node + 1].end : tv.node + 1;
        const int xe = T->vidx[x];
        const int cnt = s_cnt[xe];
        for (int i = (tid - rot) & (kTcWG - 1); i < cnt; i += kTcWG) {
          const int32_t err = tc_item(L, T, t, v, xe, x, which, i);
          if (err) set_status(status, err);
        }
        rot = (rot + cnt) & (kTcWG - 1);
      }
    }
    if (any) __syncthreads();
  }
  // the image to [base, end): 16-byte stores between dword head / tail
  uint8_t* o = out + base;
  const int head = (16 - mis) & 15;  // bytes before the first 16-byte boundary
  const int h = head < len ? head : len;
  if (tid < (h >> 2)) st32(o + 4 * tid, ld32(t.I + 4 * tid));
  const int body = (len - h) >> 4;
  for (int q = tid; q < body; q += kTcWG)
    *gp(reinterpret_cast<u32x4*>(o + h) + q) = reinterpret_cast<const u32x4*>(t.I + h)[q];
  const int tail0 = h + 16 * body;
  const int tw = (len - tail0) >> 2;
  if (tid < tw) st32(o + tail0 + 4 * tid, ld32(t.I + tail0 + 4 * tid));
}

template <int D>
hipError_t launch_tc_encode_d(const TcLaunch& W, const int64_t* offs, uint8_t* out, int64_t capacity,
                              int32_t* status, hipStream_t s) {
  hipLaunchKernelGGL(tc_encode_kernel<D>, dim3((unsigned)W.ntiles), dim3(kTcWG), 0, s, W, offs, out, capacity,
                     status);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_tc_sizes(const GenLaunch& L, const TcTables* T, int node, int64_t m, bool root_coll,
                           hipStream_t s) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(tc_sizes_kernel, dim3((unsigned)((m + kTcWG - 1) / kTcWG)), dim3(kTcWG), 0, s, L, T, node, m,
                     root_coll ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_tc_rows(const GenLaunch& L, const TcTables* T, int64_t* sizes, hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(tc_rows_kernel, dim3((unsigned)((L.num_rows + kTcWG - 1) / kTcWG)), dim3(kTcWG), 0, s, L, T,
                     sizes);
  return hipGetLastError();
}

hipError_t launch_tc_tiles(const TcLaunch& W, const int64_t* offs, hipStream_t s) {
  const int64_t n = W.g.num_rows + 1;
  hipLaunchKernelGGL(tc_tiles_kernel, dim3((unsigned)((n + kTcWG - 1) / kTcWG)), dim3(kTcWG), 0, s, W, offs);
  return hipGetLastError();
}

hipError_t launch_tc_encode(const TcLaunch& W, const int64_t* offs, uint8_t* out, int64_t capacity,
                            int32_t* status, hipStream_t s) {
  if (W.g.num_rows <= 0 || W.ntiles <= 0) return hipSuccess;
  if (W.g.max_depth + 1 <= 4) return launch_tc_encode_d<4>(W, offs, out, capacity, status, s);
  if (W.g.max_depth + 1 <= 8) return launch_tc_encode_d<8>(W, offs, out, capacity, status, s);
  return launch_tc_encode_d<18>(W, offs, out, capacity, status, s);
}

}  // namespace fory_amd
