// treecol.hip — the columnar tree engine: encode of any nesting as per-node passes.
//
// The per-lane engine (generic.hip) walks one record per lane, serially through a
// frame stack, so a wave runs as long as its deepest record and every column access is
// a lane-private gather. Here the same bytes (BaseBinaryEncoderBuilder.serializeFor,
// :236-351 arrays, :370-427 maps, :436-490 beans) come from passes over instance columns
// (one instance = one element of a schema node's column), each a full-occupancy grid:
//   sizes   bottom-up, one launch per var node (children first), lane per instance:
//           A[c][j] = the bytes instance j adds to its parent — strings round8(len),
//           decimals 32 (BigIntegers round8 of their toByteArray() length), beans bitmap + 8 x fields + their var children, arrays
//           8 + bitmap + round8(n x elemSize) + their var items (a difference of the
//           items' scanned sizes), maps 8 + key array + value array. Item nodes (list
//           items, map keys / values) are scanned in place: A[x][k] = bytes of the
//           items before k, A[x][m] = all of them.
//   rows    row / frame size = header + fixed part + the top-level var fields' sizes;
//           scanned into the row offsets (encoded_size's output).
//   write   top-down, one launch per bean / list / map node (parents first). Lane per
//           row: frame header, null bits, slots, strings and decimals in place, and the
//           positions of the top-level beans / lists / maps. Lane per bean instance at its
//           position: the same for its fields. Lists / maps: a workgroup per 256
//           containers writes their headers (count, null bitmap from the items'
//           validity, element padding), then their elements item-parallel — each item
//           finds its container by a binary search over the workgroup's item starts in
//           LDS, writes its element (value, zero, or var slot) and a var item's position
//           (the container's data start + the items' scanned sizes before it), a
//           string / decimal item in place.
// Every byte of a record is written once (fixed parts whole, zero slots included), so
// the output needs no clearing. Absent instances (under a null parent) get position -1
// and write nothing.
#include "gen_device.h"

namespace fory_amd {
namespace {

constexpr int kTcWG = 256;

__device__ __forceinline__ bool tc_is_var(int kind) { return !is_scalar(kind); }
// Strings and decimals are leaves: their parent writes them in place (no positions) and
// sizes them from their own column unless they are items (whose sizes are scanned).
__device__ __forceinline__ bool tc_leaf(int kind) { return kind == KIND_BYTES || kind == KIND_DECIMAL; }
__device__ __forceinline__ bool tc_has_pos(int kind) { return tc_is_var(kind) && !tc_leaf(kind); }

// Row bytes of decimal value k: 32 (writeDecimal), or a BigInteger's round8(toByteArray().length).
__device__ __forceinline__ int64_t tc_dec_bytes(const GNode& nd, const ColumnDev& col, int64_t k) {
  if (!g_bigint(nd)) return 32;
  uint32_t w[4];
  g_load_dec(col.values, k, w);
  return g_bigint_bytes(w);
}

// Bytes var value k of (non-item) node c adds to its parent; 0 when null.
__device__ __forceinline__ int64_t tc_size(const TcTables* T, int c, const GNode& nd, const ColumnDev& col,
                                           int64_t k) {
  if (nd.kind == KIND_BYTES || nd.kind == KIND_DECIMAL) {
    if ((nd.flags & 1) && !gvalid(col.validity, k)) return 0;
    return nd.kind == KIND_DECIMAL ? tc_dec_bytes(nd, col, k) : gr8((int64_t)gp(col.offsets)[k + 1] - gp(col.offsets)[k]);
  }
  return gp(T->A[c])[k];
}

__device__ __forceinline__ int64_t tc_clamp(int64_t k, int64_t m) { return k < 0 ? 0 : (k > m ? m : k); }

// Bytes of the array of items x in [o0, o1): BinaryArrayWriter.reset(n) fixed part + var items.
__device__ __forceinline__ int64_t tc_array_bytes(const GenLaunch& L, const TcTables* T, int x, int64_t o0,
                                                  int64_t o1) {
  const GNode it = L.nodes[x];
  const int64_t n = o1 - o0;
  int64_t b = 8 + gbm(n) + gr8(n * elem_size(it));
  if (tc_is_var(it.kind)) b += gp(T->A[x])[o1] - gp(T->A[x])[o0];
  return b;
}

// Item range [o0, o1) of container instance j of node c (offsets clamped to the items' column,
// so no pass reads or writes past it). Returns false when the offsets did not fit the items'
// column length the caller passed (or decrease): the write pass reports that as
// FORY_ERR_INVALID_ARGUMENT instead of dropping the items silently.
__device__ __forceinline__ bool tc_items(const GenLaunch& L, const TcTables* T, int c, int64_t j, int64_t* o0,
                                         int64_t* o1) {
  const int32_t* off = L.cols[c].offsets;
  const int64_t mx = T->m[c + 1];
  const int64_t ra = gp(off)[j], rb = gp(off)[j + 1];
  const int64_t a = tc_clamp(ra, mx), b = tc_clamp(rb, mx);
  *o0 = a;
  *o1 = b < a ? a : b;
  return ra >= 0 && rb >= ra && rb <= mx;
}

// ---------------------------------------------------------------------------
// sizes
// ---------------------------------------------------------------------------
// Bytes instance j of var node c adds to its parent (root_coll: node 0 of a collection
// frame, present whatever its validity).
__device__ __forceinline__ int64_t tc_node_size(const GenLaunch& L, const TcTables* T, int c, int64_t j,
                                                int root_coll) {
  const GNode nd = L.nodes[c];
  const ColumnDev col = L.cols[c];
  if (!root_coll && (nd.flags & 1) && !gvalid(col.validity, j)) return 0;
  switch (nd.kind) {
    case KIND_BYTES: return gr8((int64_t)gp(col.offsets)[j + 1] - gp(col.offsets)[j]);
    case KIND_DECIMAL: return tc_dec_bytes(nd, col, j);
    case KIND_STRUCT: {
      int64_t s = gbm(nd.nchild) + 8LL * nd.nchild;
      for (int ch = c + 1; ch < nd.end; ch = L.nodes[ch].end) {
        const GNode cn = L.nodes[ch];
        if (tc_is_var(cn.kind)) s += tc_size(T, ch, cn, L.cols[ch], j);
      }
      return s;
    }
    case KIND_LIST:
    case KIND_MAP: {
      int64_t o0, o1;
      tc_items(L, T, c, j, &o0, &o1);
      if (nd.kind == KIND_LIST) return tc_array_bytes(L, T, c + 1, o0, o1);
      return 8 + tc_array_bytes(L, T, c + 1, o0, o1) + tc_array_bytes(L, T, L.nodes[c + 1].end, o0, o1);
    }
    default: return 0;
  }
}

// Row / frame i's bytes.
__device__ __forceinline__ int64_t tc_row_size(const GenLaunch& L, const TcTables* T, int64_t i) {
  if (L.frame == FORY_FRAME_COLLECTION) return 4 + gp(T->A[0])[i];
  int64_t s = frame_header_bytes(L.frame) + L.fixed_size;
  for (int t = 0; t < L.num_nodes; t = L.nodes[t].end) {
    const GNode tn = L.nodes[t];
    if (tc_is_var(tn.kind)) s += tc_size(T, t, tn, L.cols[t], i);
  }
  return s;
}

__global__ __launch_bounds__(kTcWG) void tc_sizes_kernel(GenLaunch L, const TcTables* __restrict__ T, int c,
                                                         int64_t m, int root_coll) {
  const int64_t j = (int64_t)blockIdx.x * kTcWG + threadIdx.x;
  if (j >= m) return;
  gp(T->A[c])[j] = tc_node_size(L, T, c, j, root_coll);
}

// Sizes + exclusive scan, reduce-then-scan in three launches (no cross-workgroup waits:
// the L2s are per XCD, so a look-back chain pays a memory round trip per hop):
// sums    tiles of kTcScanTile: each value's size into out[j], the tile's sum into part[t]
// part    one workgroup scans the tile sums (exclusive, part[tiles] = total)
// down    each tile scans its values in place from its base; out[m] = the total.
// node >= 0: that node's instance sizes; node < 0: the rows' sizes.
constexpr int kTcScanPer = 8;
constexpr int kTcScanTile = kTcWG * kTcScanPer;

__device__ __forceinline__ int64_t tc_block_excl(int64_t x, int64_t* s_wave, int64_t* total) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int64_t inc = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(inc, d, 64);
    if (lane >= d) inc += y;
  }
  if (lane == 63) s_wave[wv] = inc;
  __syncthreads();
  int64_t wbase = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kTcWG / 64; ++w) {
    if (w < wv) wbase += s_wave[w];
    tot += s_wave[w];
  }
  __syncthreads();
  *total = tot;
  return wbase + inc - x;
}

__global__ __launch_bounds__(kTcWG) void tc_size_sums_kernel(GenLaunch L, const TcTables* __restrict__ T, int c,
                                                             int64_t m, int root_coll, int64_t* __restrict__ out,
                                                             int64_t* __restrict__ part) {
  __shared__ int64_t s_wave[kTcWG / 64];
  const int64_t j0 = (int64_t)blockIdx.x * kTcScanTile + threadIdx.x;  // lanes in instance order (coalesced)
  int64_t sum = 0;
#pragma unroll
  for (int u = 0; u < kTcScanPer; ++u) {
    const int64_t j = j0 + u * kTcWG;
    if (j < m) {
      const int64_t v = c >= 0 ? tc_node_size(L, T, c, j, root_coll) : tc_row_size(L, T, j);
      out[j] = v;
      sum += v;
    }
  }
  int64_t tot;
  tc_block_excl(sum, s_wave, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kTcWG) void tc_part_scan_kernel(int64_t* __restrict__ part, int64_t nb) {
  __shared__ int64_t s_wave[kTcWG / 64];
  int64_t carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += kTcWG) {
    const int64_t b = b0 + threadIdx.x;
    const int64_t x = b < nb ? part[b] : 0;
    int64_t tot;
    const int64_t ex = tc_block_excl(x, s_wave, &tot);
    if (b < nb) part[b] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) part[nb] = carry;
}

__global__ __launch_bounds__(kTcWG) void tc_scan_down_kernel(int64_t* __restrict__ out, int64_t m,
                                                             const int64_t* __restrict__ part) {
  __shared__ int64_t s_wave[kTcWG / 64];
  __shared__ int64_t tile[kTcWG * (kTcScanPer + 1)];  // runs of kTcScanPer, padded: lanes read / write in order
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * kTcScanTile;
  auto pos = [](int e) { return (e / kTcScanPer) * (kTcScanPer + 1) + e % kTcScanPer; };
#pragma unroll
  for (int u = 0; u < kTcScanPer; ++u) {
    const int e = u * kTcWG + tid;
    tile[pos(e)] = b0 + e < m ? out[b0 + e] : 0;
  }
  __syncthreads();
  int64_t v[kTcScanPer];
  int64_t sum = 0;
#pragma unroll
  for (int u = 0; u < kTcScanPer; ++u) {
    v[u] = tile[tid * (kTcScanPer + 1) + u];
    sum += v[u];
  }
  int64_t tot;
  int64_t at = part[blockIdx.x] + tc_block_excl(sum, s_wave, &tot);
#pragma unroll
  for (int u = 0; u < kTcScanPer; ++u) {
    tile[tid * (kTcScanPer + 1) + u] = at;
    at += v[u];
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kTcScanPer; ++u) {
    const int e = u * kTcWG + tid;
    if (b0 + e < m) out[b0 + e] = tile[pos(e)];
  }
  if (blockIdx.x == gridDim.x - 1 && tid == 0) out[m] = part[gridDim.x];  // the total
}

__global__ __launch_bounds__(kTcWG) void tc_rows_kernel(GenLaunch L, const TcTables* __restrict__ T,
                                                        int64_t* __restrict__ sizes) {
  const int64_t i = (int64_t)blockIdx.x * kTcWG + threadIdx.x;
  if (i < L.num_rows) sizes[i] = tc_row_size(L, T, i);
}

// ---------------------------------------------------------------------------
// write
// ---------------------------------------------------------------------------
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

// Slot size field of a var value: a string's byte length, a BigInteger's toByteArray()
// length, else its bytes (decimals 32).
__device__ __forceinline__ uint32_t tc_slot_size(const GNode& nd, const ColumnDev& col, int64_t k, int64_t bytes) {
  if (nd.kind == KIND_BYTES) return (uint32_t)(gp(col.offsets)[k + 1] - gp(col.offsets)[k]);
  if (g_bigint(nd)) {
    uint32_t w[4];
    g_load_dec(col.values, k, w);
    return (uint32_t)g_bigint_len(w);
  }
  return (uint32_t)bytes;
}

// g_put_bytes (n bytes + zero padding to 8 at a 4-byte aligned dst) with a short string's
// source dwords all loaded before any store: one memory latency, not one per dword.
__device__ __forceinline__ void tc_copy(uint8_t* dst, const uint8_t* src, int64_t n) {
  constexpr int kW = 16;  // n <= 60: <= 16 source dwords, <= 16 output dwords with the padding
  if (n > 60) {
    g_put_bytes(dst, src, n);
    return;
  }
  const int sh = (int)(reinterpret_cast<uintptr_t>(src) & 3);
  const GAS uint32_t* s = gp(reinterpret_cast<const uint32_t*>(src - sh));  // (an Arrow column)
  const int nin = (sh + (int)n + 3) >> 2;  // source dwords holding string bytes
  const int nout = (int)(gr8(n) >> 2);     // output dwords (string + padding)
  uint32_t w[kW + 1];
#pragma unroll
  for (int k = 0; k < kW; ++k) w[k] = k < nin ? s[k] : 0u;
  w[kW] = 0u;
#pragma unroll
  for (int k = 0; k < kW; ++k) {
    if (k >= nout) break;
    uint32_t v = sh ? (uint32_t)((((uint64_t)w[k + 1] << 32) | w[k]) >> (8 * sh)) : w[k];
    const int left = (int)n - 4 * k;
    if (left <= 0) v = 0u;
    else if (left < 4) v &= (1u << (8 * left)) - 1u;
    st32(dst + 4 * k, v);
  }
}

// A leaf value at `at`, S bytes allotted (room for S checked by the caller):
// writeUnaligned + zeroOutPaddingBytes (strings, BigInteger.toByteArray()), or
// BinaryWriter.writeDecimal (checkPrecisionAndScale: FORY_ERR_UNSUPPORTED). A string whose padded length is not S
// (sizes from an encoded_size call over other contents) is not written: FORY_ERR_ENCODER.
__device__ __forceinline__ int32_t tc_leaf_write(uint8_t* out, const GNode& nd, const ColumnDev& col, int64_t k,
                                                 int64_t at, int64_t S) {
  if (nd.kind == KIND_BYTES) {
    const int64_t s0 = gp(col.offsets)[k], n = (int64_t)gp(col.offsets)[k + 1] - s0;
    if (n < 0 || gr8(n) != S) return FORY_ERR_ENCODER;
    tc_copy(out + at, col.values + s0, n);
    return 0;
  }
  uint32_t w[4];
  g_load_dec(col.values, k, w);
  if (g_bigint(nd)) {  // BigInteger: write(ordinal, value.toByteArray()) -> writeUnaligned
    const int len = g_bigint_len(w);
    if (gr8(len) != S) return FORY_ERR_ENCODER;
    g_put_bigint(out + at, w, len);
    return 0;
  }
  if (S != 32) return FORY_ERR_ENCODER;
  if (!g_dec_fits(w, nd.prec)) return FORY_ERR_UNSUPPORTED;
  const uint32_t ext = (w[3] >> 31) ? 0xffffffffu : 0u;
  for (int q = 0; q < 4; ++q) st32(out + at + 4 * q, w[q]);
  for (int q = 4; q < 8; ++q) st32(out + at + 4 * q, ext);
  return 0;
}

// Rows and beans, field-parallel: one lane per (instance k, field q) writes the field's
// slot — scalar zero-extended (putInt64(slot, 0) then the value), null zero, var
// (rel, size) — and a string / decimal in place at its position (the fixed part's end +
// the sizes of the var fields before it), or hands a bean / list / map field its
// position. Lane q = 0 writes the null bitmap (and for rows the frame header, after the
// row's size is checked against its offsets). Adjacent lanes write adjacent slots.
// ROWS: instances are the rows (c unused); else bean node c at T->P[c] (-1: absent, its
// bean / list / map fields get -1).
template <bool ROWS>
__global__ __launch_bounds__(kTcWG) void tc_write_fields_kernel(GenLaunch L, const TcTables* __restrict__ T, int c,
                                                                int64_t m, const int64_t* __restrict__ offs,
                                                                uint8_t* __restrict__ out, int64_t cap,
                                                                int32_t* status) {
  __shared__ GNode s_nd[kTcMaxNodes];
  __shared__ ColumnDev s_col[kTcMaxNodes];
  __shared__ int32_t s_kid[kTcMaxNodes];
  const int tid = threadIdx.x;
  const int nf = ROWS ? T->nroot : L.nodes[c].nchild;
  const int bm = ROWS ? L.bitmap_bytes : gbm(nf);
  const int k0 = ROWS ? 0 : T->kid0[c];
  for (int q = tid; q < nf; q += kTcWG) {
    const int kid = T->kids[k0 + q];
    s_kid[q] = kid;
    s_nd[q] = L.nodes[kid];
    s_col[q] = L.cols[kid];
  }
  __syncthreads();
  // An instance's fields are a group of NP = pow2(nf) <= 64 adjacent lanes inside one
  // wave: the bytes of the var fields before a field are a prefix sum over the group and
  // the null bitmap a ballot of it (one size load per lane). Wider beans: NP = nf, each
  // lane sums its predecessors' sizes itself.
  int lg = 0;
  while ((1 << lg) < nf) ++lg;
  const bool grp = lg <= 6;
  const int np = grp ? 1 << lg : nf;
  const uint64_t w = (uint64_t)blockIdx.x * kTcWG + tid;
  if (!grp && w >= (uint64_t)m * (uint64_t)nf) return;
  const int64_t k = grp ? (int64_t)(w >> lg) : (int64_t)(w / (uint64_t)nf);
  const int q = grp ? (int)(w & (uint64_t)(np - 1)) : (int)(w - (uint64_t)k * (uint64_t)nf);
  const bool live = k < m && q < nf;  // (grouped lanes past the fields / instances only shuffle)
  const int qq = live ? q : 0;
  const GNode nd = s_nd[qq];
  const ColumnDev col = s_col[qq];
  const int kid = s_kid[qq];
  const int64_t kk = live ? k : 0;
  const bool has_pos = tc_has_pos(nd.kind), var = tc_is_var(nd.kind);
  // Everything that does not depend on the instance's position is loaded first, so the
  // lane waits one memory latency for all of it (the position is one more load):
  // null bit, value or this var field's bytes (and the group's prefix of them), and the
  // bitmap words (and, for rows, the row's var bytes to check its size).
  const bool isnull = live && (nd.flags & 1) && !gvalid(col.validity, kk);
  uint64_t v = 0;
  int64_t rel = 0, S = 0;
  if (!var) {
    v = load_elem(col.values, nd.width, kk);
    if (nd.kind == KIND_BOOL) v = v ? 1 : 0;
  } else {
    S = tc_size(T, kid, nd, col, kk);
  }
  uint32_t bw[kTcMaxNodes / 32] = {0u, 0u, 0u, 0u};  // lane q = 0: setNullAt bits of every field
  int64_t need = 0;
  if (grp) {
    const int64_t mine = live && var ? S : 0;
    int64_t x = mine;
    for (int d = 1; d < np; d <<= 1) {
      const int64_t y = __shfl_up(x, d, np);
      if (q >= d) x += y;
    }
    rel = x - mine;
    need = __shfl(x, np - 1, np);
    const uint64_t nb = __ballot(isnull);
    const int g0 = (threadIdx.x & 63) & ~(np - 1);  // the group's first lane in the wave
    const uint64_t bits = np == 64 ? nb : (nb >> g0) & ((1ull << np) - 1);
    bw[0] = (uint32_t)bits;
    bw[1] = (uint32_t)(bits >> 32);
    if (!live) return;
  } else {
    if (var)
      for (int f = 0; f < q; ++f)
        if (tc_is_var(s_nd[f].kind)) rel += tc_size(T, s_kid[f], s_nd[f], s_col[f], k);
    if (q == 0) {
      for (int f = 0; f < nf; ++f) {
        if ((s_nd[f].flags & 1) && !gvalid(s_col[f].validity, k)) bw[f >> 5] |= 1u << (f & 31);
        if (ROWS && tc_is_var(s_nd[f].kind)) need += tc_size(T, s_kid[f], s_nd[f], s_col[f], k);
      }
    }
  }
  int64_t P;
  int hdr = 0;
  int64_t beg = 0, size = 0;
  if (ROWS) {
    beg = offs[k];
    const int64_t end = offs[k + 1];
    hdr = frame_header_bytes(L.frame);
    size = end - beg;
    const bool bad = beg < 0 || end > cap || size < hdr + L.fixed_size || size - hdr > 0x7fffffffLL || (beg & 3);
    if (bad && q == 0) set_status(status, FORY_ERR_CAPACITY);
    P = bad ? -1 : beg + hdr;
  } else {
    P = gp(T->P[c])[k];
    if (P >= 0 && P + bm + 8LL * nf > cap) {
      if (q == 0) set_status(status, FORY_ERR_ENCODER);
      P = -1;
    }
  }
  if (P < 0) {
    if (has_pos) gp(T->P[kid])[k] = -1;
    return;
  }
  const int64_t fixed_end = P + bm + 8LL * nf;
  if (q == 0) {
    if (ROWS) {  // the row's size against its offsets, then the frame header
      if (hdr + L.fixed_size + need > size) set_status(status, FORY_ERR_CAPACITY);  // offsets not from these columns
      if (hdr == 12) {  // Encoders.encode(MemoryBuffer, T): [i32 8 + rowSize][i64 hash]
        st32(out + beg, (uint32_t)(size - 4));
        tc_put(out + beg + 4, (uint64_t)L.schema_hash, 8);
      } else if (hdr == 8) {  // Encoder.encode(T): [i64 hash]
        tc_put(out + beg, (uint64_t)L.schema_hash, 8);
      }
    }
#pragma unroll
    for (int wq = 0; wq < kTcMaxNodes / 32; ++wq)
      if (wq < bm / 4) st32(out + P + 4 * wq, bw[wq]);
  }
  uint8_t* slot = out + P + bm + 8 * q;
  if (isnull) {  // BinaryWriter.setNullAt: slot zero
    tc_put(slot, 0, 8);
    if (has_pos) gp(T->P[kid])[k] = -1;
    return;
  }
  if (!var) {
    tc_put(slot, v, 8);
    return;
  }
  const int64_t at = fixed_end + rel;
  if (S < 0 || at + S > cap) {
    set_status(status, FORY_ERR_ENCODER);
    tc_put(slot, 0, 8);
    if (has_pos) gp(T->P[kid])[k] = -1;
    return;
  }
  tc_put(slot, ((uint64_t)(at - P) << 32) | tc_slot_size(nd, col, k, S), 8);
  if (has_pos) {
    gp(T->P[kid])[k] = at;
  } else {
    const int32_t r = tc_leaf_write(out, nd, col, k, at, S);
    if (r) set_status(status, r);
  }
}

// Rows and beans, a lane per instance (the column loads of a wave are consecutive
// elements), fields in batches of kTcBatch whose loads are issued together: each lane
// builds its instance's frame header, null bitmap and slots in an LDS image (FS bytes
// per lane), hands its bean / list / map fields their positions (consecutive per wave)
// and writes its strings / decimals in place; then each wave stores its 64 images as
// consecutive dwords of each instance (coalesced). Same bytes as tc_write_fields_kernel,
// which stays for images beyond kTcStageMax.
constexpr int kTcBatch = 4;
constexpr int kTcStageMax = 280;  // frame header + bitmap + slots of up to 32 fields

template <bool ROWS>
__global__ __launch_bounds__(kTcWG) void tc_write_fields_lds_kernel(GenLaunch L, const TcTables* __restrict__ T,
                                                                    int c, int64_t m,
                                                                    const int64_t* __restrict__ offs,
                                                                    uint8_t* __restrict__ out, int64_t cap,
                                                                    int32_t* status, int FS) {
  extern __shared__ __attribute__((aligned(16))) uint8_t tc_stage[];
  __shared__ GNode s_nd[kTcMaxNodes];
  __shared__ ColumnDev s_col[kTcMaxNodes];
  __shared__ int32_t s_kid[kTcMaxNodes];
  const int tid = threadIdx.x, lane = tid & 63;
  const int nf = ROWS ? T->nroot : L.nodes[c].nchild;
  const int bm = ROWS ? L.bitmap_bytes : gbm(nf);
  const int k0 = ROWS ? 0 : T->kid0[c];
  for (int q = tid; q < nf; q += kTcWG) {
    const int kid = T->kids[k0 + q];
    s_kid[q] = kid;
    s_nd[q] = L.nodes[kid];
    s_col[q] = L.cols[kid];
  }
  __syncthreads();
  const int64_t k = (int64_t)blockIdx.x * kTcWG + tid;
  const bool inb = k < m;
  const int64_t kk = inb ? k : 0;
  const int hdr = ROWS ? frame_header_bytes(L.frame) : 0;
  uint8_t* img = tc_stage + (size_t)tid * FS;  // [frame header][bitmap][slots]
  int64_t P = -1, beg = 0, size = 0;
  if (inb) {
    if (ROWS) {
      beg = offs[k];
      const int64_t end = offs[k + 1];
      size = end - beg;
      const bool bad = beg < 0 || end > cap || size < hdr + L.fixed_size || size - hdr > 0x7fffffffLL || (beg & 3);
      if (bad) set_status(status, FORY_ERR_CAPACITY);
      else P = beg + hdr;
    } else {
      P = gp(T->P[c])[k];
      if (P >= 0 && P + bm + 8LL * nf > cap) {
        set_status(status, FORY_ERR_ENCODER);
        P = -1;
      }
    }
  }
  const int64_t fixed_end = P + bm + 8LL * nf;
  int64_t rel = 0;  // bytes of the var fields so far
  for (int w = 0; w < bm / 4; ++w) st32(img + hdr + 4 * w, 0u);
  for (int q0 = 0; q0 < nf; q0 += kTcBatch) {
    bool nul[kTcBatch];
    uint64_t v[kTcBatch];
    int64_t S[kTcBatch];
#pragma unroll
    for (int u = 0; u < kTcBatch; ++u) {  // the batch's loads, issued together
      const int q = q0 + u < nf ? q0 + u : nf - 1;
      const GNode nd = s_nd[q];
      const ColumnDev col = s_col[q];
      nul[u] = (nd.flags & 1) && !gvalid(col.validity, kk);
      v[u] = 0;
      S[u] = 0;
      if (!tc_is_var(nd.kind)) v[u] = load_elem(col.values, nd.width, kk);
      else S[u] = tc_size(T, s_kid[q], nd, col, kk);
    }
#pragma unroll 1
    for (int u = 0; u < kTcBatch; ++u) {  // rolled: one copy of the field body
      const int q = q0 + u;
      if (q >= nf) break;
      bool nu = nul[0];
      uint64_t vu = v[0];
      int64_t Su = S[0];
#pragma unroll
      for (int t = 1; t < kTcBatch; ++t) {
        nu = u == t ? nul[t] : nu;
        vu = u == t ? v[t] : vu;
        Su = u == t ? S[t] : Su;
      }
      const GNode nd = s_nd[q];
      const int kid = s_kid[q];
      const bool has_pos = tc_has_pos(nd.kind);
      uint8_t* slot = img + hdr + bm + 8 * q;
      if (P < 0 || nu) {  // BinaryWriter.setNullAt: bit set, slot zero (absent: no position)
        if (nu) img[hdr + (q >> 3)] |= (uint8_t)(1u << (q & 7));
        st32(slot, 0u);
        st32(slot + 4, 0u);
        if (inb && has_pos) gp(T->P[kid])[k] = -1;
        continue;
      }
      if (!tc_is_var(nd.kind)) {
        const uint64_t x = nd.kind == KIND_BOOL ? (vu ? 1 : 0) : vu;
        st32(slot, (uint32_t)x);
        st32(slot + 4, (uint32_t)(x >> 32));
        continue;
      }
      const int64_t at = fixed_end + rel;
      if (Su < 0 || at + Su > cap) {
        set_status(status, FORY_ERR_ENCODER);
        st32(slot, 0u);
        st32(slot + 4, 0u);
        if (has_pos) gp(T->P[kid])[k] = -1;
        continue;
      }
      const uint64_t sw = ((uint64_t)(at - P) << 32) | tc_slot_size(nd, s_col[q], kk, Su);
      st32(slot, (uint32_t)sw);
      st32(slot + 4, (uint32_t)(sw >> 32));
      rel += Su;
      if (has_pos) {
        gp(T->P[kid])[k] = at;
      } else {
        const int32_t r = tc_leaf_write(out, nd, s_col[q], kk, at, Su);
        if (r) set_status(status, r);
      }
    }
  }
  if (ROWS && P >= 0) {  // the row's size against its offsets, then the frame header
    if (hdr + L.fixed_size + rel > size) set_status(status, FORY_ERR_CAPACITY);  // offsets not from these columns
    if (hdr == 12) {  // Encoders.encode(MemoryBuffer, T): [i32 8 + rowSize][i64 hash]
      st32(img, (uint32_t)(size - 4));
      st32(img + 4, (uint32_t)(uint64_t)L.schema_hash);
      st32(img + 8, (uint32_t)((uint64_t)L.schema_hash >> 32));
    } else if (hdr == 8) {  // Encoder.encode(T): [i64 hash]
      st32(img, (uint32_t)(uint64_t)L.schema_hash);
      st32(img + 4, (uint32_t)((uint64_t)L.schema_hash >> 32));
    }
  }
  // this wave's images out: consecutive dwords of each instance (its start: P - hdr)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int nd4 = (hdr + bm + 8 * nf) >> 2;  // dwords per image
  const uint8_t* wimg = tc_stage + (size_t)(tid - lane) * FS;
  for (int t = lane; t < 64 * nd4; t += 64) {  // (every lane the same trip count: shuffles are uniform)
    const int r = t / nd4, j = t - r * nd4;
    const int64_t pr = __shfl(P, r);
    if (pr >= 0) st32(out + pr - hdr + 4 * j, ld32(wimg + (size_t)r * FS + 4 * j));
  }
}

// Collection frames: [i32 size] and the collection's position.
__global__ __launch_bounds__(kTcWG) void tc_write_coll_kernel(GenLaunch L, const TcTables* __restrict__ T,
                                                              const int64_t* __restrict__ offs,
                                                              uint8_t* __restrict__ out, int64_t cap,
                                                              int32_t* status) {
  const int64_t i = (int64_t)blockIdx.x * kTcWG + threadIdx.x;
  if (i >= L.num_rows) return;
  const int64_t beg = offs[i], end = offs[i + 1], size = end - beg;
  const bool bad = beg < 0 || end > cap || size < 4 || size - 4 > 0x7fffffffLL || (beg & 3) ||
                   4 + gp(T->A[0])[i] > size;
  if (bad) set_status(status, FORY_ERR_CAPACITY);
  else st32(out + beg, (uint32_t)(size - 4));
  gp(T->P[0])[i] = bad ? -1 : beg + 4;
}

// The null bitmap of items [o0, o0 + n) (1 = null, BinaryArrayWriter.setNullAt) from their
// Arrow validity (1 = valid, none = all valid) at dst: gbm(n) bytes.
__device__ __forceinline__ void tc_bitmap(uint8_t* dst, const uint8_t* validity, int64_t o0, int64_t n) {
  const int nw = gbm(n) / 4;
  for (int w = 0; w < nw; ++w) {
    const int64_t rem = n - 32LL * w;
    uint32_t bits = 0;
    if (rem > 0 && validity) {  // the 32 bits from bit b: one or two aligned dwords (Arrow pads to 8 bytes)
      const int64_t b = o0 + 32LL * w;
      const GAS uint32_t* v = gp(reinterpret_cast<const uint32_t*>(validity)) + (b >> 5);
      const int sh = (int)(b & 31);
      const int take = rem < 32 ? (int)rem : 32;
      uint64_t win = v[0];
      if (sh + take > 32) win |= (uint64_t)v[1] << 32;
      const uint32_t mask = take == 32 ? 0xffffffffu : ((1u << take) - 1u);
      bits = ~(uint32_t)(win >> sh) & mask;
    }
    st32(dst + 4 * w, bits);
  }
}

// The validity dwords of items [o0, o1) from o0's dword: up to three, those the range
// reaches (a bitmap of <= 64 items needs no more), loaded with the container's sizes.
struct TcVwin {
  uint32_t w[3];
};
__device__ __forceinline__ TcVwin tc_vwin(const uint8_t* validity, int64_t o0, int64_t o1) {
  TcVwin r{{0u, 0u, 0u}};
  if (!validity) return r;
  const GAS uint32_t* v = gp(reinterpret_cast<const uint32_t*>(validity)) + (o0 >> 5);
#pragma unroll
  for (int t = 0; t < 3; ++t)
    if (((o0 >> 5) + t) * 32 < o1) r.w[t] = v[t];
  return r;
}

// An array header at Pa: [i64 n][null bitmap][element padding]; returns its fixed bytes.
// vw: the items' validity window (tc_vwin) when n <= 64.
__device__ __forceinline__ int64_t tc_array_head(const GenLaunch& L, uint8_t* out, int x, int64_t o0, int64_t n,
                                                 int64_t Pa, const TcVwin& vw) {
  const GNode it = L.nodes[x];
  const int es = elem_size(it);
  const int64_t hb = 8 + gbm(n), data = n * es, fixed = hb + gr8(data);
  tc_put(out + Pa, (uint64_t)n, 8);
  if (n > 64) {
    tc_bitmap(out + Pa + 8, (it.flags & 1) ? L.cols[x].validity : nullptr, o0, n);
  } else if (n > 0) {  // [8, 16) bytes of bitmap: two words from the window
    const int sh = (int)(o0 & 31);
    const uint64_t lo = (uint64_t)vw.w[0] | ((uint64_t)vw.w[1] << 32);
    const uint32_t b0 = (uint32_t)(lo >> sh);
    const uint32_t b1 = (uint32_t)((((uint64_t)vw.w[1] | ((uint64_t)vw.w[2] << 32)) >> sh));
    const bool nul = (it.flags & 1) && L.cols[x].validity;
    const uint32_t m0 = n >= 32 ? 0xffffffffu : ((1u << n) - 1u);
    const uint32_t m1 = n <= 32 ? 0u : (n >= 64 ? 0xffffffffu : ((1u << (n - 32)) - 1u));
    st32(out + Pa + 8, nul ? ~b0 & m0 : 0u);
    st32(out + Pa + 12, nul ? ~b1 & m1 : 0u);
  }
  for (int64_t b = data; b < gr8(data); ++b) out[Pa + hb + b] = 0;  // zeroOutPaddingBytes
  return fixed;
}

// Element q of the array at Pa (n items from o0) of item node x: item e = o0 + q.
__device__ __forceinline__ int32_t tc_element(const GenLaunch& L, const TcTables* T, uint8_t* out, int64_t cap,
                                              int x, int64_t o0, int64_t n, int64_t Pa, int64_t e) {
  const GNode it = L.nodes[x];
  const ColumnDev col = L.cols[x];
  const int es = elem_size(it);
  const int64_t q = e - o0;
  const int64_t hb = 8 + gbm(n);
  uint8_t* el = out + Pa + hb + q * es;
  const bool var = tc_is_var(it.kind), leaf = tc_leaf(it.kind);
  // the validity bit, the value or the item's scanned sizes: loaded together, then used
  const bool isnull = (it.flags & 1) && !gvalid(col.validity, e);
  uint64_t v = 0;
  int64_t a0 = 0, a1 = 0, ab = 0;
  if (!var) {
    v = load_elem(col.values, es, e);
  } else {
    const int64_t* A = T->A[x];
    a0 = A[e];
    a1 = A[e + 1];
    ab = A[o0];
  }
  if (isnull) {  // null: zero element (the header set the bit)
    tc_put(el, 0, es);
    if (var && !leaf) gp(T->P[x])[e] = -1;
    return 0;
  }
  if (!var) {
    if (it.kind == KIND_BOOL) v = v ? 1 : 0;
    tc_put(el, v, es);
    return 0;
  }
  const int64_t S = a1 - a0;
  const int64_t at = Pa + hb + gr8(n * 8) + (a0 - ab);
  if (S < 0 || at + S > cap) {
    tc_put(el, 0, 8);
    if (!leaf) gp(T->P[x])[e] = -1;
    return FORY_ERR_ENCODER;
  }
  tc_put(el, ((uint64_t)(at - Pa) << 32) | tc_slot_size(it, col, e, S), 8);
  if (leaf) return tc_leaf_write(out, it, col, e, at, S);
  gp(T->P[x])[e] = at;
  return 0;
}

// Item classes of a container node's items / keys / values (the plan's, from the host):
// scalars, strings, beans / lists / maps (positioned: their own pass writes them), and
// decimals (the generic element path).
constexpr int kTcScalar = 0, kTcStr = 1, kTcPos = 2, kTcOther = 3;
constexpr int kTcU = 4;  // items per lane whose inputs are in flight together

// One element's inputs, loaded before any is used. The loads are unconditional (an
// absent validity reads a dummy byte), so the compiler's counted waits stay exact and
// kTcU items' loads overlap.
struct TcIn {
  uint32_t vb;     // the validity byte holding the item's bit
  uint64_t v;      // scalar: the value
  int64_t a0, a1;  // string / positioned: the items' scanned sizes A[e], A[e + 1]
  int32_t s0, s1;  // string: its Arrow offsets
};

template <int CLS>
__device__ __forceinline__ void tc_in_load(const GNode& it, const ColumnDev& col, const int64_t* A, int64_t e,
                                           const uint8_t* dummy, TcIn& in) {
  in.vb = *gp((it.flags & 1) && col.validity ? col.validity + (e >> 3) : dummy);
  if (CLS == kTcScalar) {
    in.v = load_elem(col.values, elem_size(it), e);
  } else if (CLS == kTcStr || CLS == kTcPos) {
    in.a0 = gp(A)[e];
    in.a1 = gp(A)[e + 1];
    if (CLS == kTcStr) {
      in.s0 = gp(col.offsets)[e];
      in.s1 = gp(col.offsets)[e + 1];
    }
  }
}

// Element e (item q = e - o0 of n) of the array at Pa from its loaded inputs: the
// same bytes as tc_element. ab: A[x][o0] of the container (string / positioned items).
template <int CLS>
__device__ __forceinline__ int32_t tc_el_store(const GenLaunch& L, const TcTables* T, uint8_t* out, int64_t cap,
                                               int x, const GNode& it, const ColumnDev& col, int64_t o0, int64_t n,
                                               int64_t Pa, int64_t ab, int64_t e, const TcIn& in) {
  if (CLS == kTcOther) return tc_element(L, T, out, cap, x, o0, n, Pa, e);
  const int es = elem_size(it);
  const int64_t hb = 8 + gbm(n);
  uint8_t* el = out + Pa + hb + (e - o0) * es;
  const bool isnull = (it.flags & 1) && col.validity && !((in.vb >> (e & 7)) & 1);
  if (isnull) {  // null: zero element (the header set the bit)
    tc_put(el, 0, es);
    if (CLS == kTcPos) gp(T->P[x])[e] = -1;
    return 0;
  }
  if (CLS == kTcScalar) {
    tc_put(el, it.kind == KIND_BOOL ? (in.v ? 1 : 0) : in.v, es);
    return 0;
  }
  const int64_t S = in.a1 - in.a0;
  const int64_t at = Pa + hb + gr8(n * 8) + (in.a0 - ab);
  if (S < 0 || at + S > cap) {
    tc_put(el, 0, 8);
    if (CLS == kTcPos) gp(T->P[x])[e] = -1;
    return FORY_ERR_ENCODER;
  }
  if (CLS == kTcPos) {
    tc_put(el, ((uint64_t)(at - Pa) << 32) | (uint32_t)S, 8);
    gp(T->P[x])[e] = at;
    return 0;
  }
  const int64_t len = (int64_t)in.s1 - in.s0;  // writeUnaligned + zeroOutPaddingBytes
  tc_put(el, ((uint64_t)(at - Pa) << 32) | (uint32_t)len, 8);
  if (len < 0 || gr8(len) != S) return FORY_ERR_ENCODER;
  tc_copy(out + at, col.values + in.s0, len);
  return 0;
}

// Lists / maps: a workgroup per kTcWG containers. (1) lane per container: its position and
// item range; (2) the first kTcU items of every lane issue their inputs' loads together with
// the container headers' (array sizes, validity windows), and the headers are written; (3)
// the elements item-parallel, kTcU per lane per round, each finding its container by a
// binary search over the workgroup's item starts in LDS. KC / VC: the item (key) / value
// classes, so each instantiation carries only its items' paths.
template <bool MAP, int KC, int VC>
__global__ __launch_bounds__(kTcWG) void tc_write_cont_kernel(GenLaunch L, const TcTables* __restrict__ T, int c,
                                                              int64_t m, uint8_t* __restrict__ out, int64_t cap,
                                                              int32_t* status) {
  __shared__ int64_t sP[kTcWG];      // container position (-1: absent / null / does not fit)
  __shared__ int32_t sO[kTcWG + 1];  // first item of each container (+ the end)
  __shared__ int32_t sK[kTcWG];      // maps: key array bytes
  __shared__ int64_t sAk[kTcWG], sAv[kTcWG];  // A[key][o0], A[val][o0]: the items' sizes before the container's
  const int tid = threadIdx.x;
  const int64_t j0 = (int64_t)blockIdx.x * kTcWG;
  const int cnt = m - j0 < kTcWG ? (int)(m - j0) : kTcWG;
  constexpr bool map = MAP;
  const int key = c + 1, val = map ? L.nodes[key].end : key;  // (val: maps only)
  const GNode kit = L.nodes[key], vit = L.nodes[val];
  const ColumnDev kcol = L.cols[key], vcol = L.cols[val];
  const int64_t* Ak = T->A[key];
  const int64_t* Av = T->A[val];
  const uint8_t* dummy = reinterpret_cast<const uint8_t*>(T);
  constexpr bool kvar = KC != kTcScalar, vvar = MAP && VC != kTcScalar;
  const int64_t mx = T->m[key];
  int32_t err = 0;
  int64_t P = -1, o0 = 0, o1 = 0;
  if (tid < cnt) {
    const int64_t j = j0 + tid;
    P = gp(T->P[c])[j];
    // offsets past the items' column length (a short fory_column.length): an error, not a
    // silently shorter array (present containers only: absent ones read no items)
    if (!tc_items(L, T, c, j, &o0, &o1) && P >= 0) err = FORY_ERR_INVALID_ARGUMENT;
    sO[tid] = (int32_t)o0;
    if (tid == cnt - 1) sO[cnt] = (int32_t)o1;
  }
  __syncthreads();
  const int64_t e0 = sO[0], e1 = sO[cnt];
  TcIn ki[kTcU], vi[kTcU];
  auto load_round = [&](int64_t r0) {
#pragma unroll
    for (int u = 0; u < kTcU; ++u) {
      const int64_t e = r0 + tid + u * kTcWG;
      const int64_t ee = e < e1 ? e : e0;  // (past the end: a readable item, unused)
      tc_in_load<KC>(kit, kcol, Ak, ee, dummy, ki[u]);
      if (map) tc_in_load<VC>(vit, vcol, Av, ee, dummy, vi[u]);
    }
  };
  if (e1 > e0) load_round(e0);
  if (tid < cnt) {
    const int64_t n = o1 - o0;
    // the header's inputs: the items' validity windows and scanned sizes
    const TcVwin vk = tc_vwin((kit.flags & 1) ? kcol.validity : nullptr, o0, o1);
    const TcVwin vv = map ? tc_vwin((vit.flags & 1) ? vcol.validity : nullptr, o0, o1) : TcVwin{};
    int64_t ak0 = 0, ak1 = 0, av0 = 0, av1 = 0;
    if (kvar) {
      ak0 = gp(Ak)[o0];
      ak1 = gp(Ak)[o1];
    }
    if (vvar) {
      av0 = gp(Av)[o0];
      av1 = gp(Av)[o1];
    }
    const int64_t kb = 8 + gbm(n) + gr8(n * elem_size(kit)) + (ak1 - ak0);  // tc_array_bytes
    const int64_t vb = map ? 8 + gbm(n) + gr8(n * elem_size(vit)) + (av1 - av0) : 0;
    if (P >= 0 && P + (map ? 8 + kb + vb : kb) > cap) {
      err = FORY_ERR_ENCODER;
      P = -1;
    }
    if (P >= 0) {
      if (map) {  // [i64 key array bytes][key array][value array]
        tc_put(out + P, (uint64_t)kb, 8);
        tc_array_head(L, out, key, o0, n, P + 8, vk);
        tc_array_head(L, out, val, o0, n, P + 8 + kb, vv);
      } else {
        tc_array_head(L, out, key, o0, n, P, vk);
      }
    }
    sP[tid] = P;
    sK[tid] = (int32_t)kb;
    sAk[tid] = ak0;
    sAv[tid] = av0;
  }
  __syncthreads();
  for (int64_t r0 = e0; r0 < e1; r0 += kTcU * kTcWG) {
    if (r0 != e0) load_round(r0);
#pragma unroll
    for (int u = 0; u < kTcU; ++u) {
      const int64_t e = r0 + tid + u * kTcWG;
      if (e >= e1) break;
      int a = 0, b = cnt - 1;  // the last container whose items start at or before e
      while (a < b) {
        const int mid = (a + b + 1) >> 1;
        if (sO[mid] <= e) a = mid;
        else b = mid - 1;
      }
      const int64_t Pa = sP[a];
      const int64_t ao = sO[a], n = sO[a + 1] - ao;
      if (Pa < 0 || e >= ao + n) {  // absent container (or items between non-adjacent ranges)
        if (KC == kTcPos) gp(T->P[key])[e] = -1;
        if (map && VC == kTcPos) gp(T->P[val])[e] = -1;
        continue;
      }
      int32_t r = tc_el_store<KC>(L, T, out, cap, key, kit, kcol, ao, n, map ? Pa + 8 : Pa, sAk[a], e, ki[u]);
      if (map) {
        const int32_t r2 = tc_el_store<VC>(L, T, out, cap, val, vit, vcol, ao, n, Pa + 8 + sK[a], sAv[a], e, vi[u]);
        if (!r) r = r2;
      }
      if (r) err = r;
    }
  }
  // items no container of the call references: no position
  constexpr bool kpos = KC == kTcPos, vpos = MAP && VC == kTcPos;
  if (blockIdx.x == 0 && (kpos || vpos))
    for (int64_t e = tid; e < e0; e += kTcWG) {
      if (kpos) gp(T->P[key])[e] = -1;
      if (vpos) gp(T->P[val])[e] = -1;
    }
  if (j0 + cnt == m && (kpos || vpos))
    for (int64_t e = e1 + tid; e < mx; e += kTcWG) {
      if (kpos) gp(T->P[key])[e] = -1;
      if (vpos) gp(T->P[val])[e] = -1;
    }
  if (err) set_status(status, err);
}

// Lanes per instance of tc_write_fields_kernel: the fields rounded up to a power of two
// (<= 64, a group inside one wave), or the fields themselves beyond 64.
int64_t tc_group_lanes(int nf) {
  int np = 1;
  while (np < nf) np <<= 1;
  return np <= 64 ? np : nf;
}

}  // namespace

hipError_t launch_tc_sizes(const GenLaunch& L, const TcTables* T, int node, int64_t m, bool root_coll,
                           hipStream_t s) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(tc_sizes_kernel, dim3((unsigned)((m + kTcWG - 1) / kTcWG)), dim3(kTcWG), 0, s, L, T, node, m,
                     root_coll ? 1 : 0);
  return hipGetLastError();
}

int64_t tc_scan_flag_words(int64_t m) { return (m + kTcScanTile - 1) / kTcScanTile + 2; }

hipError_t launch_tc_size_scan(const GenLaunch& L, const TcTables* T, int node, int64_t m, bool root_coll,
                               int64_t* out, uint64_t* flags, hipStream_t s) {
  if (m <= 0) return hipMemsetAsync(out, 0, sizeof(int64_t), s);
  const int64_t tiles = (m + kTcScanTile - 1) / kTcScanTile;
  int64_t* part = reinterpret_cast<int64_t*>(flags);
  hipLaunchKernelGGL(tc_size_sums_kernel, dim3((unsigned)tiles), dim3(kTcWG), 0, s, L, T, node, m, root_coll ? 1 : 0,
                     out, part);
  hipLaunchKernelGGL(tc_part_scan_kernel, dim3(1), dim3(kTcWG), 0, s, part, tiles);
  hipLaunchKernelGGL(tc_scan_down_kernel, dim3((unsigned)tiles), dim3(kTcWG), 0, s, out, m, part);
  return hipGetLastError();
}

hipError_t launch_tc_rows(const GenLaunch& L, const TcTables* T, int64_t* sizes, hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(tc_rows_kernel, dim3((unsigned)((L.num_rows + kTcWG - 1) / kTcWG)), dim3(kTcWG), 0, s, L, T,
                     sizes);
  return hipGetLastError();
}

hipError_t launch_tc_write_rows(const GenLaunch& L, const TcTables* T, int nroot, const int64_t* offs, uint8_t* out,
                                int64_t capacity, int32_t* status, hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  if (L.frame == FORY_FRAME_COLLECTION) {
    hipLaunchKernelGGL(tc_write_coll_kernel, dim3((unsigned)((L.num_rows + kTcWG - 1) / kTcWG)), dim3(kTcWG), 0, s,
                       L, T, offs, out, capacity, status);
    return hipGetLastError();
  }
  const int fs = frame_header_bytes(L.frame) + L.bitmap_bytes + 8 * nroot;
  if (fs <= kTcStageMax) {
    raise_lds_cap(&tc_write_fields_lds_kernel<true>);
    hipLaunchKernelGGL(tc_write_fields_lds_kernel<true>, dim3((unsigned)((L.num_rows + kTcWG - 1) / kTcWG)),
                       dim3(kTcWG), (size_t)kTcWG * fs, s, L, T, -1, L.num_rows, offs, out, capacity, status, fs);
    return hipGetLastError();
  }
  const int64_t work = L.num_rows * tc_group_lanes(nroot);
  hipLaunchKernelGGL(tc_write_fields_kernel<true>, dim3((unsigned)((work + kTcWG - 1) / kTcWG)), dim3(kTcWG), 0, s,
                     L, T, -1, L.num_rows, offs, out, capacity, status);
  return hipGetLastError();
}

// tc_write_cont_kernel's instantiation for item (key) class kc and value class vc.
template <bool MAP, int KC>
auto* tc_cont_kernel_v(int vc) {
  switch (vc) {
    case kTcScalar: return &tc_write_cont_kernel<MAP, KC, kTcScalar>;
    case kTcStr: return &tc_write_cont_kernel<MAP, KC, kTcStr>;
    case kTcPos: return &tc_write_cont_kernel<MAP, KC, kTcPos>;
    default: return &tc_write_cont_kernel<MAP, KC, kTcOther>;
  }
}

auto* tc_cont_kernel_map(int kc, int vc) {
  switch (kc) {
    case kTcScalar: return tc_cont_kernel_v<true, kTcScalar>(vc);
    case kTcStr: return tc_cont_kernel_v<true, kTcStr>(vc);
    case kTcPos: return tc_cont_kernel_v<true, kTcPos>(vc);
    default: return tc_cont_kernel_v<true, kTcOther>(vc);
  }
}

auto* tc_cont_kernel_list(int kc) {  // (the value class is unused: one instantiation per item class)
  switch (kc) {
    case kTcScalar: return &tc_write_cont_kernel<false, kTcScalar, kTcScalar>;
    case kTcStr: return &tc_write_cont_kernel<false, kTcStr, kTcScalar>;
    case kTcPos: return &tc_write_cont_kernel<false, kTcPos, kTcScalar>;
    default: return &tc_write_cont_kernel<false, kTcOther, kTcScalar>;
  }
}

int tc_item_class(int kind) {
  return kind == KIND_FIXED || kind == KIND_BOOL ? kTcScalar
         : kind == KIND_BYTES                    ? kTcStr
         : kind == KIND_DECIMAL                  ? kTcOther
                                                 : kTcPos;
}

hipError_t launch_tc_write_node(const GenLaunch& L, const TcTables* T, int node, int64_t m, uint8_t* out,
                                int64_t capacity, int32_t* status, hipStream_t s, int kind, int nchild, int key_kind,
                                int val_kind) {
  if (m <= 0) return hipSuccess;
  if (kind == KIND_LIST || kind == KIND_MAP) {
    const int kc = tc_item_class(key_kind), vc = tc_item_class(val_kind);
    hipLaunchKernelGGL(kind == KIND_MAP ? tc_cont_kernel_map(kc, vc) : tc_cont_kernel_list(kc),
                       dim3((unsigned)((m + kTcWG - 1) / kTcWG)), dim3(kTcWG), 0, s, L, T, node, m, out, capacity,
                       status);
  } else {
    const int fs = (((nchild + 63) >> 6) << 3) + 8 * nchild;  // bitmap + slots
    if (nchild > 0 && fs <= kTcStageMax) {
      raise_lds_cap(&tc_write_fields_lds_kernel<false>);
      hipLaunchKernelGGL(tc_write_fields_lds_kernel<false>, dim3((unsigned)((m + kTcWG - 1) / kTcWG)), dim3(kTcWG),
                         (size_t)kTcWG * fs, s, L, T, node, m, nullptr, out, capacity, status, fs);
      return hipGetLastError();
    }
    const int64_t work = m * tc_group_lanes(nchild > 0 ? nchild : 1);
    hipLaunchKernelGGL(tc_write_fields_kernel<false>, dim3((unsigned)((work + kTcWG - 1) / kTcWG)), dim3(kTcWG), 0,
                       s, L, T, node, m, nullptr, out, capacity, status);
  }
  return hipGetLastError();
}

}  // namespace fory_amd
