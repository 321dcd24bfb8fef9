// treedec.hip — the columnar tree engine's decode: rows of any nesting to Arrow columns
// by per-node passes, the inverse of treecol.hip's encode.
//
// The per-lane decoder (generic.hip, g_decode) walks each record through a frame stack,
// once per container depth for the counts and once for the values. Here every pass is a
// grid over one node's instances (BaseBinaryEncoderBuilder's layout read back as
// RowEncoderBuilder.fromRow / ArrayDataForEach do, RowEncoderBuilder.java:215-318):
//   fields  rows (and each bean node): a lane per instance, its fields in order; the
//           lanes of a wave write consecutive elements of each output column. Per field
//           the lane reads the null bit and slot and writes the value (scalars: the slot's
//           low bytes; strings: the bytes at the slot's (offset, size); decimals: 32
//           bytes, the high 16 the sign extension; BigIntegers: their 1..16 big-endian
//           bytes sign-extended), the count of a string / list / map
//           at this decode level, or hands a bean / list / map its position.
//   items   each list / map node: a workgroup per 256 containers reads their headers
//           (count, and for maps the key array's bytes), checks the count against the
//           Arrow offsets the sizes passes wrote, then the elements item-parallel (the
//           container found by binary search over the workgroup's offsets in LDS); each
//           element is read like a field, its slot relative to its array.
// Positions (the instance's start, its extent and its record's end) live in the
// workspace for the call. decode_sizes runs level by level: level L's passes (the rows
// at L = 0, the items of the lists / maps of level L - 1, the beans of level L) write
// level L's counts and the positions of its beans / lists / maps, which the next
// level's passes start from (nothing persists between calls: each call starts at level
// 0). Every read is bounded by the record's end, with the per-lane decoder's checks
// (FORY_ERR_CORRUPT).
#include "gen_device.h"

namespace fory_amd {
namespace {

constexpr int kTdWG = 256;
constexpr int kTdBatch = 8;  // fields whose slot words an instance loads together (8 vs 4: BeanA decode 8.39 vs 8.55 ms, r05l)
constexpr int kTdU = 2;  // item groups per lane whose loads are in flight together (td_items_kernel)
constexpr int kTdStageMax = 264;  // bitmap + slots of up to 32 fields staged per lane

__device__ __forceinline__ bool td_leaf(int kind) { return kind == KIND_BYTES || kind == KIND_DECIMAL; }

// Validity of a wave's 64 consecutive positions from a 64-aligned base (lane l = base + l):
// a word per half wave by ballot. inr: the lane's position is this workgroup's; a word
// wholly inside the range is stored, a word shared with a neighbour's range (or past
// the column's items) takes only this range's bits, by atomics.
__device__ __forceinline__ void td_valid_words(uint8_t* validity, int64_t pos, bool inr, bool valid) {
  const uint64_t vb = __ballot(inr && valid), rb = __ballot(inr);
  const int lane = threadIdx.x & 63;
  if (lane & 31) return;
  const uint32_t v = (uint32_t)(vb >> (lane & 32)), r = (uint32_t)(rb >> (lane & 32));
  if (!r) return;
  uint32_t* word = reinterpret_cast<uint32_t*>(validity) + (pos >> 5);
  if (r == 0xffffffffu) {
    *gp(word) = v;
    return;
  }
  if (v) g_or(word, v);
  if (r & ~v) g_and(word, ~(r & ~v));
}

// Array header at `at` bounded by lim: numElements, or -1 (g_array_n).
__device__ __forceinline__ int64_t td_array_n(const GenLaunch& L, const uint8_t* rows, int item, int64_t at,
                                              int64_t lim) {
  if (at < 0 || at + 8 > lim) return -1;
  const int64_t n = (int64_t)gget(rows + at, 8);
  if (n < 0 || n > 0x7fffffffLL || at + 8 + gbm(n) + n * elem_size(L.nodes[item]) > lim) return -1;
  return n;
}

// A list / map payload at [at, at + size): its element count, or -1; *kat / *vat the (key)
// array and the value array (g_container_n; BinaryMap.pointTo, BinaryMap.java:62-77).
__device__ __forceinline__ int64_t td_container_n(const GenLaunch& L, const uint8_t* rows, int node, int64_t at,
                                                  int64_t size, int64_t* kat, int64_t* vat) {
  if (L.nodes[node].kind == KIND_LIST) {
    *kat = at;
    *vat = at;
    return td_array_n(L, rows, node + 1, at, at + size);
  }
  if (size < 8) return -1;
  const int64_t kb = (int64_t)gget(rows + at, 8);
  const int key = node + 1, val = L.nodes[key].end;
  *kat = at + 8;
  *vat = at + 8 + kb;
  if (kb < 8 || *vat + 8 > at + size) return -1;
  const int64_t nk = td_array_n(L, rows, key, *kat, *vat);
  const int64_t nv = td_array_n(L, rows, val, *vat, at + size);
  return nk < 0 || nk != nv ? -1 : nk;
}

// One value of node f, instance k, from its slot word sv in the row / array starting at
// `origin` (slots' offsets are relative to it), in a record ending at rend. Scalars and
// validity are the caller's. level >= 0: the counts of that decode level (and the positions
// the levels below need); -1: the values.
__device__ __forceinline__ void td_value(const GenLaunch& L, const TdTables* T, int f, const GNode& nd,
                                         const ColumnDev& col, int64_t k, const uint8_t* rows, uint64_t sv,
                                         int64_t origin, int64_t rend, bool isnull, int level, int32_t* status) {
  const bool values = level < 0;
  if (nd.kind == KIND_STRUCT) {
    if (!values && nd.cdepth > level) return;
    int64_t P = -1;
    if (!isnull) {  // BinaryRow.getStruct: the child row at the slot's offset
      const int64_t rel = (int32_t)(sv >> 32);
      const int64_t start = origin + rel;
      if (rel < 0 || start + gbm(nd.nchild) + 8LL * nd.nchild > rend) set_status(status, FORY_ERR_CORRUPT);
      else P = start;
    }
    gp(T->P[f])[k] = P;
    gp(T->TL[f])[k] = P < 0 ? 0 : (int32_t)(rend - P);
    return;
  }
  if (nd.kind == KIND_DECIMAL) {  // UnsafeTrait.getDecimal: 32 bytes, the high 16 the sign extension
    if (!col.out_values || (!values && nd.cdepth != level)) return;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (!isnull && g_bigint(nd)) {  // new BigInteger(bytes at the slot's (offset, len))
      const int64_t rel = (int64_t)(int32_t)(sv >> 32), at = origin + rel, len = (int64_t)(int32_t)(uint32_t)sv;
      if (rel < 0 || len < 0 || at + len > rend || !g_get_bigint(rows + at, len, w)) {
        set_status(status, FORY_ERR_CORRUPT);
        return;
      }
    } else if (!isnull) {
      const uint64_t os = sv;
      const int64_t rel = (int64_t)(int32_t)(os >> 32), at = origin + rel;
      if (rel < 0 || (uint32_t)os != 32u || at + 32 > rend || (at & 3)) {
        set_status(status, FORY_ERR_CORRUPT);
        return;
      }
      for (int q = 0; q < 4; ++q) w[q] = ld32(rows + at + 4 * q);
      const uint32_t ext = (w[3] >> 31) ? 0xffffffffu : 0u;
      bool fits = true;
      for (int q = 4; q < 8; ++q) fits = fits && ld32(rows + at + 4 * q) == ext;
      if (!fits) {
        set_status(status, FORY_ERR_CORRUPT);
        return;
      }
    }
    for (int q = 0; q < 4; ++q) *gp(reinterpret_cast<uint32_t*>(col.out_values + 16 * k + 4 * q)) = w[q];
    return;
  }
  // BYTES / LIST / MAP: (offset, size) relative to the enclosing row / array
  int64_t at = 0, size = 0;
  if (!isnull) {
    const uint64_t os = sv;
    at = origin + (int64_t)(int32_t)(os >> 32);
    size = (int64_t)(int32_t)(uint32_t)os;
    if ((int32_t)(os >> 32) < 0 || size < 0 || at + size > rend) {
      set_status(status, FORY_ERR_CORRUPT);
      if (nd.kind != KIND_BYTES && (values || nd.cdepth <= level)) gp(T->P[f])[k] = -1;
      return;
    }
  }
  if (!values) {
    if (nd.cdepth > level) return;
    if (nd.kind == KIND_BYTES && nd.cdepth == level && T->SRC[f]) gp(T->SRC[f])[k] = isnull ? -1 : at;  // for td_strings
    if (nd.cdepth == level && col.out_offsets) {  // this level's counts
      int64_t cnt = 0;
      if (!isnull) {
        if (nd.kind == KIND_BYTES) {
          cnt = size;
        } else {
          int64_t kat, vat;
          cnt = td_container_n(L, rows, f, at, size, &kat, &vat);
          if (cnt < 0) {
            set_status(status, FORY_ERR_CORRUPT);
            cnt = 0;
          }
        }
      }
      gp(col.out_offsets)[k + 1] = (int32_t)cnt;
    }
    if (nd.kind == KIND_BYTES) return;
    // a list / map: its position too, for the next level's items pass
  }
  if (nd.kind == KIND_BYTES) {
    if (isnull) return;
    const int64_t o0 = gp(col.out_offsets)[k];
    if ((int64_t)gp(col.out_offsets)[k + 1] - o0 != size) {  // differs from the sizes pass
      set_status(status, FORY_ERR_CORRUPT);
      return;
    }
    g_get_bytes(col.out_values + o0, rows + at, size);
    return;
  }
  gp(T->P[f])[k] = isnull ? -1 : at;
  gp(T->SZ[f])[k] = (int32_t)size;
  gp(T->TL[f])[k] = isnull ? 0 : (int32_t)(rend - at);
}

// A scalar of width w from the slot's low bytes (UnsafeTrait.getX), 0 for nulls.
__device__ __forceinline__ void td_scalar(const GNode& nd, const ColumnDev& col, int64_t k, uint64_t sv, bool isnull) {
  uint64_t v = isnull ? 0 : (nd.width >= 8 ? sv : sv & ((1ull << (8 * nd.width)) - 1));
  if (nd.kind == KIND_BOOL) v = (v & 0xff) ? 1 : 0;
  store_elem(col.out_values, nd.width, k, v);
}

// The fields of instance k (a row, or a bean at base; base < 0: absent, its fields null)
// in order: nf fields kids[k0..], bm bitmap bytes. Lanes of a wave hold consecutive
// instances from a 64-aligned one (inb: the lane's instance is in this call's range);
// every lane runs it (validity by ballot).
// The instance's bitmap / slot bytes at p (4-byte aligned), 4 or 8 of them: LDS loads from
// the wave's staged image (IMG), global loads from the rows otherwise. (One generic pointer
// for both compiled to flat loads, which wait on both counters.)
template <bool IMG>
__device__ __forceinline__ uint64_t td_hget(const uint8_t* p, int w) {
  uint32_t lo, hi = 0;
  if constexpr (IMG) {
    const __attribute__((address_space(3))) uint32_t* q = (const __attribute__((address_space(3))) uint32_t*)p;
    lo = q[0];
    if (w == 8) hi = q[1];
  } else {
    const GAS uint32_t* q = (const GAS uint32_t*)p;
    lo = q[0];
    if (w == 8) hi = q[1];
  }
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

template <bool IMG = false>
__device__ __forceinline__ void td_instance(const GenLaunch& L, const TdTables* T, int nf, int k0, int bm, int64_t k,
                                            bool inb, int64_t base, int64_t rend, const uint8_t* rows,
                                            int32_t* status, const uint8_t* img = nullptr) {
  const int level = L.fill_level;
  const bool values = level < 0;
  const bool present = base >= 0;
  const bool rd = inb && present;
  const uint8_t* hb = img ? img : rows + (present ? base : 0);  // bitmap + slots (img: staged in LDS)
  uint64_t nulls = 0;  // the bitmap word of fields [64 b, 64 b + 64)
  // fields in batches: the batch's slot words (and the bitmap word) are loaded together
  // before any is used, so an instance costs one memory latency per batch, not per field
  for (int q0 = 0; q0 < nf; q0 += kTdBatch) {
    uint64_t sv[kTdBatch];
    if ((q0 & 63) == 0) nulls = rd ? td_hget<IMG>(hb + (q0 >> 3), bm - (q0 >> 3) >= 8 ? 8 : 4) : ~0ull;
#pragma unroll
    for (int u = 0; u < kTdBatch; ++u) sv[u] = rd && q0 + u < nf ? td_hget<IMG>(hb + bm + 8 * (q0 + u), 8) : 0;
#pragma unroll 1
    for (int u = 0; u < kTdBatch; ++u) {  // rolled: one copy of the field body
      const int q = q0 + u;
      if (q >= nf) break;
      uint64_t w = sv[0];
#pragma unroll
      for (int t = 1; t < kTdBatch; ++t) w = u == t ? sv[t] : w;
      const int f = T->kids[k0 + q];
      const GNode nd = L.nodes[f];
      const ColumnDev col = L.cols[f];
      const bool isnull = !present || ((nulls >> (q & 63)) & 1);  // isNullAt
      // values, and every level's own fields (all but string bytes: td_strings copies those)
      const bool mine = values || nd.cdepth == level;
      if (mine && (nd.flags & 1) && col.out_validity) td_valid_words(col.out_validity, k, inb, !isnull);
      if (!inb) continue;
      if (is_scalar(nd.kind)) {
        if (mine && col.out_values) td_scalar(nd, col, k, w, isnull);
        continue;
      }
      td_value(L, T, f, nd, col, k, rows, w, present ? base : 0, rend, isnull, level, status);
    }
  }
}

// Rows (ROWS) or bean node s: a lane per instance, its fields in order (the row's
// header, bitmap and slots are one or two lines, read once); the lanes of a wave write
// consecutive elements of each field's column, validity a word per 32 lanes by ballot.
// FS > 0: each wave first loads its instances' bitmaps + slots as consecutive dwords of
// each (coalesced) into an LDS image of FS bytes per lane; FS = 0: each lane reads its own.
template <bool ROWS>
__global__ __launch_bounds__(kTdWG) void td_fields_kernel(GenLaunch L, const TdTables* __restrict__ T, int s,
                                                          int64_t m, const uint8_t* __restrict__ rows,
                                                          const int64_t* __restrict__ offs, int32_t* status,
                                                          int FS) {
  const int nf = ROWS ? T->nroot : L.nodes[s].nchild;
  const int k0 = ROWS ? 0 : T->kid0[s];
  const int bm = ROWS ? L.bitmap_bytes : gbm(nf);
  const int level = L.fill_level;
  const int64_t k = (int64_t)blockIdx.x * kTdWG + threadIdx.x;
  const bool inb = k < m;
  int64_t base = -1, rend = 0;
  if (inb) {
    if (ROWS) {  // the frame checks of gen_decode_kernel
      const int64_t beg = offs[k], end = offs[k + 1];
      const uint8_t* frame = rows + beg;
      const int64_t len = end - beg;
      int32_t err = 0;
      const int hdr = frame_header_bytes(L.frame);
      if (end < beg || len > 0x7fffffffLL + 12) err = FORY_ERR_CORRUPT;
      else if (hdr == 12) {
        if (len < 12) err = FORY_ERR_CORRUPT;
        else if (gget(frame + 4, 8) != (uint64_t)L.schema_hash) err = FORY_ERR_SCHEMA_MISMATCH;
        else if ((int64_t)ld32(frame) + 4 != len || len < 12 + L.fixed_size) err = FORY_ERR_CORRUPT;
      } else if (hdr == 8) {
        if (len < 8) err = FORY_ERR_CORRUPT;
        else if (gget(frame, 8) != (uint64_t)L.schema_hash) err = FORY_ERR_SCHEMA_MISMATCH;
        else if (len < 8 + L.fixed_size) err = FORY_ERR_CORRUPT;
      } else if (len < L.fixed_size) {
        err = FORY_ERR_CORRUPT;
      }
      if (err && level <= 0) set_status(status, err);  // each error once
      if (!err) {
        base = beg + hdr;
        rend = end;
      }
    } else {
      base = gp(T->P[s])[k];
      rend = base >= 0 ? base + gp(T->TL[s])[k] : 0;
    }
  }
  if (FS > 0) {  // the wave's bitmaps + slots staged by consecutive dwords of each instance
    extern __shared__ __attribute__((aligned(16))) uint8_t td_stage[];
    const int lane = threadIdx.x & 63;
    const int nd4 = (bm + 8 * nf) >> 2;
    uint8_t* wimg = td_stage + (size_t)(threadIdx.x - lane) * FS;
    for (int t = lane; t < 64 * nd4; t += 64) {  // (uniform trip count: the shuffles are)
      const int r = t / nd4, j = t - r * nd4;
      const int64_t br = __shfl(base, r);
      if (br >= 0) st32(wimg + (size_t)r * FS + 4 * j, ld32(rows + br + 4 * j));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    td_instance<true>(L, T, nf, k0, bm, k, inb, base, rend, rows, status, wimg + (size_t)lane * FS);
    return;
  }
  td_instance(L, T, nf, k0, bm, k, inb, base, rend, rows, status);
}

// Collection frames: [i32 size][the collection]: its position (COLLECTION frames).
__global__ __launch_bounds__(kTdWG) void td_coll_kernel(GenLaunch L, const TdTables* __restrict__ T,
                                                        const uint8_t* __restrict__ rows,
                                                        const int64_t* __restrict__ offs, int32_t* status) {
  const int64_t i = (int64_t)blockIdx.x * kTdWG + threadIdx.x;
  const bool inb = i < L.num_rows;
  const int level = L.fill_level;
  bool present = false;
  int64_t beg = 0, len = 0;
  if (inb) {
    beg = offs[i];
    const int64_t end = offs[i + 1];
    len = end - beg;
    present = !(end < beg || len > 0x7fffffffLL + 12);
    if (present) {
      const int64_t size = len >= 4 ? (int64_t)ld32(rows + beg) : -1;
      if (size < 8 || size + 4 != len) present = false;
    }
  }
  if (level <= 0 && (L.nodes[0].flags & 1) && L.cols[0].out_validity)
    td_valid_words(L.cols[0].out_validity, i, inb, present);
  if (!inb) return;
  if (!present && level <= 0) set_status(status, FORY_ERR_CORRUPT);
  const ColumnDev col = L.cols[0];
  if (level == 0) {
    int64_t cnt = 0;
    if (present) {
      int64_t kat, vat;
      cnt = td_container_n(L, rows, 0, beg + 4, len - 4, &kat, &vat);
      if (cnt < 0) {
        set_status(status, FORY_ERR_CORRUPT);
        cnt = 0;
      }
    }
    if (col.out_offsets) gp(col.out_offsets)[i + 1] = (int32_t)cnt;
  }
  gp(T->P[0])[i] = present ? beg + 4 : -1;
  gp(T->SZ[0])[i] = present ? (int32_t)(len - 4) : 0;
  gp(T->TL[0])[i] = present ? (int32_t)(len - 4) : 0;
}

// List / map node c: a workgroup per kTdWG containers; headers, then the elements.
// MAP: node c is a map (keys and values); FLAT: some item node is a bean of leaf fields
// (read inline). Instantiated per shape: each carries only the paths it takes.
template <bool MAP, bool FLAT>
__global__ __launch_bounds__(kTdWG) void td_items_kernel(GenLaunch L, const TdTables* __restrict__ T, int c,
                                                         int64_t m, const uint8_t* __restrict__ rows,
                                                         int32_t* status) {
  __shared__ int64_t sK[kTdWG], sV[kTdWG], sE[kTdWG];  // key / value array starts (-1: none), record end
  __shared__ int32_t sO[kTdWG + 1];                     // Arrow offsets of the workgroup's containers
  const int tid = threadIdx.x;
  const int64_t j0 = (int64_t)blockIdx.x * kTdWG;
  const int cnt = m - j0 < kTdWG ? (int)(m - j0) : kTdWG;
  const ColumnDev col = L.cols[c];
  constexpr bool map = MAP;
  const int key = c + 1, val = map ? L.nodes[key].end : -1;
  const int level = L.fill_level;
  if (tid < cnt) {
    const int64_t j = j0 + tid;
    const int64_t P = gp(T->P[c])[j];
    const int64_t o0 = gp(col.out_offsets)[j], o1 = gp(col.out_offsets)[j + 1];
    int64_t kat = -1, vat = -1;
    if (P >= 0) {
      const int64_t n = td_container_n(L, rows, c, P, gp(T->SZ[c])[j], &kat, &vat);
      if (n < 0 || n != o1 - o0) {  // corrupt, or the rows changed since the sizes pass
        set_status(status, FORY_ERR_CORRUPT);
        kat = vat = -1;
      }
    }
    sK[tid] = kat;
    sV[tid] = vat;
    sE[tid] = P >= 0 ? P + gp(T->TL[c])[j] : 0;
    sO[tid] = (int32_t)o0;
    if (tid == cnt - 1) sO[cnt] = (int32_t)o1;
  }
  __syncthreads();
  const int64_t e0 = sO[0], e1 = sO[cnt];
  constexpr int ends = map ? 2 : 1;
  // waves walk 64-aligned groups of items (uniform trip count: validity by ballot), kTdU
  // groups per round: every item's null byte and element of the round are loaded (both
  // unconditionally, an absent item's from the rows' first bytes) before any is used
  struct ItemIn {
    int64_t arr;
    bool inr, present;
    uint32_t nb;  // the null byte holding the item's bit
    uint64_t sv;  // its element (a null item's is read and dropped)
  };
  for (int64_t r0 = e0 & ~int64_t(63); r0 < e1; r0 += kTdU * kTdWG) {
    int A[kTdU];
    int64_t Q[kTdU];
    ItemIn I[kTdU][ends];
#pragma unroll
    for (int u = 0; u < kTdU; ++u) {
      const int64_t e = r0 + u * kTdWG + tid;
      const bool inr_all = e >= e0 && e < e1;
      int a = 0;
      if (inr_all) {
        int b = cnt - 1;  // the last container whose items start at or before e
        while (a < b) {
          const int mid = (a + b + 1) >> 1;
          if (sO[mid] <= e) a = mid;
          else b = mid - 1;
        }
      }
      const int64_t n = sO[a + 1] - sO[a], q = e - sO[a];
      A[u] = a, Q[u] = q;
#pragma unroll
      for (int w = 0; w < ends; ++w) {
        const int x = w ? val : key;
        const GNode it = L.nodes[x];
        ItemIn& in = I[u][w];
        in.inr = inr_all && e < T->m[x];
        in.arr = in.inr ? (w ? sV[a] : sK[a]) : -1;
        in.present = in.arr >= 0 && q < n;
        const int64_t nat = in.present ? in.arr + 8 + (q >> 3) : 0;
        const int64_t eat = in.present ? in.arr + 8 + gbm(n) + q * elem_size(it) : 0;
        in.nb = rows[nat];
        in.sv = gget(rows + eat, elem_size(it));
      }
    }
#pragma unroll
    for (int u = 0; u < kTdU; ++u) {
      const int64_t e = r0 + u * kTdWG + tid;
      const bool inr_all = e >= e0 && e < e1;
      const int a = A[u];
      const int64_t q = Q[u];
#pragma unroll
      for (int w = 0; w < ends; ++w) {
        const int x = w ? val : key;
        const GNode it = L.nodes[x];
        const ColumnDev ic = L.cols[x];
        const ItemIn& in = I[u][w];
        // an item past its output column's length (a short fory_column.length): nothing is
        // written for it (its arrays end there) and the call reports FORY_ERR_CAPACITY
        const bool inr = in.inr;
        if (inr_all && !inr && (level < 0 || it.cdepth == level || !is_scalar(it.kind)))
          set_status(status, FORY_ERR_CAPACITY);
        const int64_t arr = in.arr;
        const bool present = in.present;
        const bool isnull = !present || ((in.nb >> (q & 7)) & 1);
        if ((level < 0 || it.cdepth == level) && (it.flags & 1) && ic.out_validity)
          td_valid_words(ic.out_validity, e, inr, !isnull);
        const uint64_t sv = isnull ? 0 : in.sv;
        if (FLAT && (it.flags & kGNodeFlatBean)) {  // a bean of leaf fields: read here, no pass of its own
          int64_t P = -1;
          if (!isnull) {  // BinaryArray.getStruct: the child row at the element's offset
            const int64_t rel = (int32_t)(sv >> 32);
            if (rel < 0 || arr + rel + gbm(it.nchild) + 8LL * it.nchild > sE[a]) set_status(status, FORY_ERR_CORRUPT);
            else P = arr + rel;
          }
          td_instance(L, T, it.nchild, T->kid0[x], gbm(it.nchild), e, inr, P, P < 0 ? 0 : sE[a], rows, status);
          continue;
        }
        if (!inr) continue;
        if (is_scalar(it.kind)) {
          if ((level < 0 || it.cdepth == level) && ic.out_values) td_scalar(it, ic, e, sv, isnull);
          continue;
        }
        if (!present && td_leaf(it.kind)) continue;
        td_value(L, T, x, it, ic, e, rows, sv, present ? arr : 0, sE[a], isnull, level, status);
      }
    }
  }
}

// String / binary bytes of a column, a workgroup per kTdWG values. The values' Arrow
// bytes are one contiguous range: when it fits kTdStage, each lane reads its value's
// bytes (aligned dwords, all issued before any is used: a string's bytes start 4-aligned
// in the row and are padded to 8 there) into an LDS image of the range, and the
// workgroup stores the image with coalesced dword stores (edge dwords shared with a
// neighbour take only their own bytes). A larger range goes dword by dword, each lane
// finding its value by binary search over the offsets.
constexpr int kTdStage = 8192;

__global__ __launch_bounds__(kTdWG) void td_strings_kernel(ColumnDev col, const int64_t* __restrict__ src, int64_t m,
                                                           const uint8_t* __restrict__ rows) {
  __shared__ int32_t sO[kTdWG + 1];
  __shared__ int64_t sS[kTdWG];
  __shared__ uint32_t stage[kTdStage / 4];
  const int tid = threadIdx.x;
  const int64_t k0 = (int64_t)blockIdx.x * kTdWG;
  const int cnt = m - k0 < kTdWG ? (int)(m - k0) : kTdWG;
  int64_t my_o0 = 0, my_o1 = 0, my_s = -1;
  if (tid < cnt) {
    my_o0 = gp(col.out_offsets)[k0 + tid];
    my_o1 = gp(col.out_offsets)[k0 + tid + 1];
    my_s = src[k0 + tid];
    sO[tid] = (int32_t)my_o0;
    sS[tid] = my_s;
    if (tid == cnt - 1) sO[cnt] = (int32_t)my_o1;
  }
  __syncthreads();
  const int64_t b0 = sO[0], b1 = sO[cnt];
  const int64_t base = b0 & ~int64_t(3);
  uint8_t* out = col.out_values;
  const bool al = !(reinterpret_cast<uintptr_t>(out) & 3);  // (else every byte alone)
  if (al && b1 - base <= kTdStage) {
    uint8_t* st = reinterpret_cast<uint8_t*>(stage);
    if (my_s >= 0) {
      const uint32_t* w = reinterpret_cast<const uint32_t*>(rows + my_s);
      const int64_t len = my_o1 - my_o0;
      for (int64_t j = 0; j < len; j += 16) {
        uint32_t x[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) x[t] = j + 4 * t < len ? w[(j >> 2) + t] : 0u;
#pragma unroll
        for (int t = 0; t < 16; ++t)
          if (j + t < len) st[my_o0 - base + j + t] = (uint8_t)(x[t >> 2] >> (8 * (t & 3)));
      }
    }
    __syncthreads();
    for (int64_t d = base + 4 * tid; d < b1; d += 4 * kTdWG) {
      if (d >= b0 && d + 4 <= b1) {
        st32(out + d, stage[(d - base) >> 2]);
      } else {
        const uint32_t v = stage[(d - base) >> 2];
        for (int64_t q = d < b0 ? b0 : d; q < d + 4 && q < b1; ++q) out[q] = (uint8_t)(v >> (8 * (q - d)));
      }
    }
    return;
  }
  auto owner = [&](int64_t p) {  // the value whose bytes hold output byte p (b0 <= p < b1)
    int lo = 0, hi = cnt - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (sO[mid] <= p) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  };
  for (int64_t d = base + 4 * tid; d < b1; d += 4 * kTdWG) {
    const int64_t p0 = d < b0 ? b0 : d, p1 = d + 4 < b1 ? d + 4 : b1;
    int a = owner(p0);
    if (al && d >= b0 && d + 4 <= b1 && sO[a + 1] >= d + 4) {  // one value's four bytes
      const int64_t s0 = sS[a] + (d - sO[a]);
      const int ph = (int)(s0 & 3);
      const uint32_t* w = reinterpret_cast<const uint32_t*>(rows + (s0 - ph));
      uint32_t v = w[0];
      if (ph) v = (uint32_t)((((uint64_t)w[1] << 32) | v) >> (8 * ph));  // (w[1] only when needed)
      st32(out + d, v);
      continue;
    }
    uint32_t word = 0;
    for (int64_t q = p0; q < p1; ++q) {
      while (sO[a + 1] <= q) ++a;
      const uint8_t v = rows[sS[a] + (q - sO[a])];
      word |= (uint32_t)v << (8 * (q - d));
    }
    if (al && p0 == d && p1 == d + 4) st32(out + d, word);
    else
      for (int64_t q = p0; q < p1; ++q) out[q] = (uint8_t)(word >> (8 * (q - d)));
  }
}

}  // namespace

hipError_t launch_td_strings(uint8_t* out_values, int32_t* out_offsets, const int64_t* src, int64_t m,
                             const uint8_t* rows, hipStream_t s) {
  if (m <= 0 || !out_values || !out_offsets || !src) return hipSuccess;
  ColumnDev col{};
  col.out_values = out_values;
  col.out_offsets = out_offsets;
  hipLaunchKernelGGL(td_strings_kernel, dim3((unsigned)((m + kTdWG - 1) / kTdWG)), dim3(kTdWG), 0, s, col, src, m,
                     rows);
  return hipGetLastError();
}

hipError_t launch_td_rows(const GenLaunch& L, const TdTables* T, int nroot, const uint8_t* rows, const int64_t* offs,
                          int32_t* status, hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  const unsigned gx = (unsigned)((L.num_rows + kTdWG - 1) / kTdWG);
  if (L.frame == FORY_FRAME_COLLECTION)
    hipLaunchKernelGGL(td_coll_kernel, dim3(gx), dim3(kTdWG), 0, s, L, T, rows, offs, status);
  else
  {
    const int fs = L.bitmap_bytes + 8 * nroot;
    const int FS = fs <= kTdStageMax ? fs : 0;
    if (FS) raise_lds_cap(&td_fields_kernel<true>);
    hipLaunchKernelGGL(td_fields_kernel<true>, dim3(gx), dim3(kTdWG), (size_t)kTdWG * FS, s, L, T, -1, L.num_rows, rows,
                       offs, status, FS);
  }
  return hipGetLastError();
}

hipError_t launch_td_node(const GenLaunch& L, const TdTables* T, int node, int64_t m, int kind, int nchild,
                          int item_flags, const uint8_t* rows, int32_t* status, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  const unsigned gx = (unsigned)((m + kTdWG - 1) / kTdWG);
  if (kind == KIND_LIST || kind == KIND_MAP) {
    const bool map = kind == KIND_MAP, flat = (item_flags & kGNodeFlatBean) != 0;
    auto* k = map ? (flat ? &td_items_kernel<true, true> : &td_items_kernel<true, false>)
                  : (flat ? &td_items_kernel<false, true> : &td_items_kernel<false, false>);
    hipLaunchKernelGGL(k, dim3(gx), dim3(kTdWG), 0, s, L, T, node, m, rows, status);
  } else if (nchild > 0) {
    const int fs = (((nchild + 63) >> 6) << 3) + 8 * nchild;  // bitmap + slots
    const int FS = fs <= kTdStageMax ? fs : 0;
    if (FS) raise_lds_cap(&td_fields_kernel<false>);
    hipLaunchKernelGGL(td_fields_kernel<false>, dim3(gx), dim3(kTdWG), (size_t)kTdWG * FS, s, L, T, node, m, rows,
                       nullptr, status, FS);
  }
  return hipGetLastError();
}

}  // namespace fory_amd
