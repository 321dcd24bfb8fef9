// fixed.hip — gfx950 (CDNA4) kernels for fixed-width row-format schemas.
//
// Byte layout restated from the Java writer (the spec doc is empty,
// docs/specification/row_format_spec.md:22-24). F = java/fory-format/src/
// main/java/org/apache/fory/format:
//   row   = [null bitmap ((n+63)/64)*8 B, bit i = byte i>>3 bit i&7, 1 = null]
//           [n x 8-B slots]                              F/row/binary/writer/BinaryRowWriter.java:46-124
//   fixed = value in the slot's low bytes, zero-extended            BinaryRowWriter.java:92-124
//   frame = [i32 8+rowSize][i64 schemaHash][row]                   F/encoder/Encoders.java:213-225
//
// Fixed-width schemas (every top-level field 1/2/4/8 bytes) take the tiled
// path: tiles of records, columns read with coalesced loads, scattered into an
// LDS image of the tile's rows, and the whole tile (TR * stride contiguous
// bytes) leaves with 16-B stores. Decode is the inverse: the tile image comes
// in through LDS-DMA (global_load_lds_dwordx4), each lane reads its record's
// slots from LDS and stores coalesced columns. No MFMA: this is byte shuffling
// bound by HBM.
//
// Kernels: encode_fixed_v5_kernel (persistent, depth-2 pipelined, 16-byte
// column chunks; not-null and nullable schemas) with encode_fixed_kernel for the
// tail and wide rows; decode_fixed_v5_kernel likewise with decode_fixed_kernel. Rejected variants of
// round 1 (pipe, v3, v4, one-shot, decode v2/v3/pipe) are gone from the
// product library; their measurements are in DESIGN.md §6.1.
#include "kcommon.h"

namespace fory_amd {

// Debug-bounds build (`make debug` -> fury_amd/lib/debug/, -DFORY_DEBUG_BOUNDS; VERDICT r5
// item 2): each global access of the fixed-width kernels whose address follows the tile
// walk -- column chunks, validity words, row tiles, column stores -- is checked against
// the extent its caller promises (num_rows records; Arrow validity of (num_rows + 7) / 8
// bytes). A violation is counted per site, the first offending (tile or record, limit)
// kept, and the access goes to a safe address instead of faulting;
// fory_rowfmt_internal_debug_bounds reads the counters. Product builds compile the
// checks away (FORY_DBG is `true`).
#ifdef FORY_DEBUG_BOUNDS
struct DbgSite {
  unsigned long long count;
  long long a, b;
};
constexpr int kDbgSites = 16;
__device__ DbgSite g_dbg[kDbgSites];
__device__ __noinline__ bool dbg_ok(bool ok, int site, long long a, long long b) {
  if (!ok && atomicAdd(&g_dbg[site].count, 1ull) == 0) {
    g_dbg[site].a = a;
    g_dbg[site].b = b;
  }
  return ok;
}
#define FORY_DBG(ok, site, a, b) dbg_ok((ok), (site), (long long)(a), (long long)(b))
#else
#define FORY_DBG(ok, site, a, b) true
#endif
// sites
enum : int {
  kDbgEncMask = 0,     // NUL encode: validity word of a tile
  kDbgEncTile = 1,     // v5 encode: a tile's column chunks
  kDbgEncStore = 2,    // v5 encode: a tile's rows
  kDbgDecValid = 3,    // NUL decode: validity word of a tile
  kDbgDecTile = 4,     // v5 decode: a tile's rows
  kDbgDecStore = 5,    // v5 decode: a column chunk
  kDbgTailNull = 6,    // one-tile encode: a validity byte
  kDbgTailStore = 7,   // one-tile encode: the tile's rows
  kDbgTailValid = 8,   // one-tile decode: validity bytes
  kDbgTailLoad = 9,    // one-tile decode: the tile's rows
  kDbgEncTable = 10,   // NUL kernels: the slot-validity table
};

namespace {

// ---------------------------------------------------------------------------
// Fixed-width encode: columns -> rows (tiled through LDS)
// ---------------------------------------------------------------------------
// One tile = TR records. TR = 64: lane = record, one field per wave
// instruction (descriptor wave-uniform -> scalar loads). TR = 32/16/8 (wide
// rows): 64/TR fields per wave instruction. The host sorts the field table
// into width groups (8/4/2/1 bytes) so every load loop has a compile-time
// width and distinct destination registers: a batch of U column loads is in
// flight before the first LDS write. Dead lanes of a partial tile re-read
// record r0 (no divergent branch around the loads).

template <int TR>
__device__ __forceinline__ int field_of(int fb, int u, int fstep, int fsub) {
  const int f = fb + u * fstep + fsub;
  if constexpr (TR == 64) return __builtin_amdgcn_readfirstlane(f);
  return f;
}

// BinaryWriter.setNullAt's input: Arrow validity bit of record idx (nullable fields).
__device__ __forceinline__ bool input_null(const FixedFieldDev& fd, int64_t idx, int64_t num_rows) {
  if (!((fd.flags & 1) && fd.validity)) return false;
  if (!FORY_DBG(idx >= 0 && (idx >> 3) < (num_rows + 7) / 8, kDbgTailNull, idx, num_rows)) return false;
  return !((load_byte(fd.validity + (idx >> 3)) >> (idx & 7)) & 1);
}

// Stores a slot into the LDS row image (BinaryRowWriter.write: slot zeroed,
// value in the low bytes; null -> bit set, slot left zero; bool -> 0/1).
// HDR: frame header bytes before the row — 0 (raw rows), 12 (STREAM frames:
// [i32 size][i64 hash]), 8 (HASHED frames of Encoder.encode(T): [i64 hash]).
template <int HDR>
__device__ __forceinline__ void put_slot(uint8_t* row, int hdr_bm, int slot, uint64_t x, bool isnull, int flags) {
  if (flags & 2) x = x ? 1 : 0;  // MemoryBuffer.putBoolean
  if (isnull) {
    x = 0;
    atomicOr(reinterpret_cast<uint32_t*>(row + HDR + ((slot >> 5) << 2)), 1u << (slot & 31));
  }
  uint8_t* p = row + hdr_bm + 8 * slot;
  if (HDR == 12) {  // stream rows start 12 bytes into the frame: slots are only 4-byte aligned
    st32(p, (uint32_t)x);
    st32(p + 4, (uint32_t)(x >> 32));
  } else {
    *reinterpret_cast<uint64_t*>(p) = x;
  }
}

// The same without the bitmap: the nullable v5 kernels write whole bitmap words
// (v5_bitmaps); a null record's slot is 0.
template <int HDR>
__device__ __forceinline__ void put_slot_nb(uint8_t* row, int hdr_bm, int slot, uint64_t x, bool isnull, int flags) {
  if (flags & 2) x = x ? 1 : 0;  // MemoryBuffer.putBoolean
  if (isnull) x = 0;
  uint8_t* p = row + hdr_bm + 8 * slot;
  if (HDR == 12) {
    st32(p, (uint32_t)x);
    st32(p + 4, (uint32_t)(x >> 32));
  } else {
    *reinterpret_cast<uint64_t*>(p) = x;
  }
}

// Frame header [i32 8+rowSize][i64 hash] + zeroed null bitmap of this lane's row.
template <int HDR>
__device__ __forceinline__ void put_header(uint8_t* row, const FixedLaunch& L) {
  if (HDR == 8) {  // Encoder.encode(T): [i64 hash][row] (Encoders.java:203-210)
    st32(row, (uint32_t)(uint64_t)L.schema_hash);
    st32(row + 4, (uint32_t)((uint64_t)L.schema_hash >> 32));
  } else if (HDR == 12) {
    st32(row, (uint32_t)(8 + L.fixed_size));
    st32(row + 4, (uint32_t)(uint64_t)L.schema_hash);
    st32(row + 8, (uint32_t)((uint64_t)L.schema_hash >> 32));
  }
  for (int b = 0; b < L.bitmap_bytes; b += 4) st32(row + HDR + b, 0u);
}

// LDS tile image -> HBM: `bytes` contiguous bytes, 16-B stores, 4 in flight.
__device__ __forceinline__ void store_tile(const uint8_t* lds, uint8_t* __restrict__ dst, int bytes, int tid) {
  const int n16 = bytes >> 4;
  int c = tid;
  for (; c + 3 * kWG < n16; c += 4 * kWG) {
    const u32x4 x0 = *reinterpret_cast<const u32x4*>(lds + c * 16);
    const u32x4 x1 = *reinterpret_cast<const u32x4*>(lds + (c + kWG) * 16);
    const u32x4 x2 = *reinterpret_cast<const u32x4*>(lds + (c + 2 * kWG) * 16);
    const u32x4 x3 = *reinterpret_cast<const u32x4*>(lds + (c + 3 * kWG) * 16);
    *reinterpret_cast<u32x4*>(dst + c * 16) = x0;
    *reinterpret_cast<u32x4*>(dst + (c + kWG) * 16) = x1;
    *reinterpret_cast<u32x4*>(dst + (c + 2 * kWG) * 16) = x2;
    *reinterpret_cast<u32x4*>(dst + (c + 3 * kWG) * 16) = x3;
  }
  for (; c < n16; c += kWG) *reinterpret_cast<u32x4*>(dst + c * 16) = *reinterpret_cast<const u32x4*>(lds + c * 16);
  const int tail4 = (bytes & 15) >> 2;
  if (tid < tail4) st32(dst + n16 * 16 + tid * 4, ld32(lds + n16 * 16 + tid * 4));
}

// One width group [g0, g1) of the encode: U loads in flight, then U slots.
template <int W, int TR, int HDR>
__device__ __forceinline__ void enc_group(const FixedFieldDev* __restrict__ fields, int g0, int g1, int wave, int fsub,
                                          int64_t idx, uint8_t* row, int hdr_bm, int64_t num_rows) {
  constexpr int FPW = 64 / TR;
  constexpr int FSTEP = kWaves * FPW;
  constexpr int U = 16;
  for (int pb = g0 + wave * FPW; pb < g1; pb += FSTEP * U) {
    uint64_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = field_of<TR>(pb, u, FSTEP, fsub);
      v[u] = p < g1 ? ldw<W>(fields[p].values, idx) : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = field_of<TR>(pb, u, FSTEP, fsub);
      if (p < g1) {
        const FixedFieldDev& fd = fields[p];
        put_slot<HDR>(row, hdr_bm, fd.slot, v[u], input_null(fd, idx, num_rows), fd.flags);
      }
    }
  }
}

template <int TR, int HDR>
__global__ __launch_bounds__(kWG) void encode_fixed_kernel(FixedLaunch L, const FixedFieldDev* __restrict__ fields,
                                                           uint8_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane % TR;
  const int fsub = lane / TR;
  const int64_t r0 = (L.tile0 + (int64_t)blockIdx.x) * TR;
  const int64_t left = L.num_rows - r0;
  const int rows = left < TR ? (int)left : TR;
  const int hdr_bm = HDR + L.bitmap_bytes;
  uint8_t* row = lds + r * L.stride;
  const int64_t idx = r < rows ? r0 + r : r0;

  if (wave == 0 && fsub == 0) put_header<HDR>(row, L);
  if (L.any_nullable) __syncthreads();  // null bits are OR-ed into the zeroed bitmap

  enc_group<8, TR, HDR>(fields, L.group[0], L.group[1], wave, fsub, idx, row, hdr_bm, L.num_rows);
  enc_group<4, TR, HDR>(fields, L.group[1], L.group[2], wave, fsub, idx, row, hdr_bm, L.num_rows);
  enc_group<2, TR, HDR>(fields, L.group[2], L.group[3], wave, fsub, idx, row, hdr_bm, L.num_rows);
  enc_group<1, TR, HDR>(fields, L.group[3], L.group[4], wave, fsub, idx, row, hdr_bm, L.num_rows);
  __syncthreads();
  if (FORY_DBG(r0 >= 0 && r0 + rows <= L.num_rows, kDbgTailStore, r0, L.num_rows))
    store_tile(lds, out + r0 * L.stride, rows * L.stride, tid);
}

// Chunk instructions of the 16-byte-chunk encode (v5 below): instruction i of a
// tile of R records, numbered per width group (8, 4, 2, 1 bytes): its width and
// its first field; wave v issues v, v + NW, ....
template <int R>
__device__ __forceinline__ bool v3_insn_g(int i, const int32_t* group, int* w, int* p0, int* pend) {
  const int fpi8 = 1024 / (R * 8), fpi4 = 1024 / (R * 4), fpi2 = 1024 / (R * 2), fpi1 = 1024 / R;
  const int n8 = group[1] - group[0], n4 = group[2] - group[1];
  const int n2 = group[3] - group[2], n1 = group[4] - group[3];
  const int i8 = (n8 + fpi8 - 1) / fpi8, i4 = (n4 + fpi4 - 1) / fpi4;
  const int i2 = (n2 + fpi2 - 1) / fpi2, i1 = (n1 + fpi1 - 1) / fpi1;
  if (i < i8) { *w = 8; *p0 = group[0] + i * fpi8; *pend = group[1]; return true; }
  i -= i8;
  if (i < i4) { *w = 4; *p0 = group[1] + i * fpi4; *pend = group[2]; return true; }
  i -= i4;
  if (i < i2) { *w = 2; *p0 = group[2] + i * fpi2; *pend = group[3]; return true; }
  i -= i2;
  if (i < i1) { *w = 1; *p0 = group[3] + i * fpi1; *pend = group[4]; return true; }
  return false;
}

template <int R>
__device__ __forceinline__ bool v3_insn(int i, const FixedLaunch& L, int* w, int* p0, int* pend) {
  return v3_insn_g<R>(i, L.group, w, p0, pend);
}

template <int R>
__host__ __device__ inline int v3_insn_count(const int* group) {
  const int fpi8 = 1024 / (R * 8), fpi4 = 1024 / (R * 4), fpi2 = 1024 / (R * 2), fpi1 = 1024 / R;
  const int n8 = group[1] - group[0], n4 = group[2] - group[1];
  const int n2 = group[3] - group[2], n1 = group[4] - group[3];
  return (n8 + fpi8 - 1) / fpi8 + (n4 + fpi4 - 1) / fpi4 + (n2 + fpi2 - 1) / fpi2 + (n1 + fpi1 - 1) / fpi1;
}

// ---------------------------------------------------------------------------
// Encode v5: 16-byte column chunks per lane, depth-2 load pipeline
// ---------------------------------------------------------------------------
// Column reads are the encode's limiter: 4/8-byte loads of 256-byte column
// segments reach ~1.6 TB/s at two workgroups per CU, while 16-byte loads of
// >= 512-byte segments reach ~5.9 TB/s (scripts/microbench/colread.hip). So each
// lane loads one 16-byte chunk of ONE field's column segment (E = 16/w
// consecutive records) and scatters its E values into the LDS row image. A
// field of width w spans CPF = R*w/16 chunks per tile; one wave instruction
// (64 x 16 B) covers FPI = 64/CPF fields (v3_insn_g numbers the instructions per
// width group). Persistent workgroups; two tiles of column chunks are in flight
// per workgroup (register sets A/B, the loop unrolled by 2 so both stay
// static). Every lane issues exactly K loads per tile (inactive lanes / absent
// instructions re-read a valid dummy address), so hipcc waits with a counted
// vmcnt for the older set while the younger set stays in flight. Order per
// stage: write X -> barrier -> store this tile's rows -> issue X for tile +
// 2*grid -> barrier. Nullable schemas take the NUL form (validity bits loaded
// with the chunks, null bits OR-ed into the LDS bitmaps, bitmaps re-zeroed as the
// rows leave).
template <int R, int K, int OPT = 0>
__device__ __forceinline__ void v5_issue(const uint8_t* const (&ptr)[K], const int (&wk)[K], int64_t r0,
                                         u32x4 (&d)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const u32x4* a = reinterpret_cast<const u32x4*>(ptr[k] + r0 * wk[k]);
    if constexpr (OPT & 1) d[k] = __builtin_nontemporal_load(gp(a));  // once-read column streams
    else d[k] = *gp(a);
  }
}

// sf[k]: slot | flags << 16 | nullable-with-validity << 19 | live << 20 | rb << 21.
// Nullable schemas (NUL): the tile's null masks per slot are in LDS (mt[slot], bit r:
// record r of the tile is null, from the Arrow validity words v5_masks loaded); a null
// record's slot is written 0, its bit set by v5_bitmaps.
// The records of a 4- or 8-byte chunk go into the image starting at record
// (c >> rot) mod E (c: the lane's chunk in the field, E records per chunk), so the
// lanes of one LDS store instruction spread over the banks: at Struct104's raw stride
// (848 B = 212 dwords) the in-order writes of a 4-byte field put a 16-lane store group on
// 4 banks (v5_rotation picks rot per plan from the store grouping).
template <int R, int K, int HDR, bool NUL = false>
__device__ __forceinline__ void v5_write(uint8_t* lds, int stride, int hdr_bm, const int (&wk)[K],
                                         const uint32_t (&sf)[K], const u32x4 (&d)[K], const uint64_t* mt,
                                         int rot4, int rot8) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int w = wk[k];
    if (!(sf[k] & (1u << 20))) continue;
    const int slot = sf[k] & 0xffff, flags = (sf[k] >> 16) & 0x7, rb = sf[k] >> 21;
    uint32_t nm = 0;  // bit e: record rb + e is null
    if constexpr (NUL) nm = (uint32_t)(mt[slot] >> rb);
    auto nul = [&](int e) { return NUL && ((nm >> e) & 1); };
    uint8_t* row = lds + rb * stride;
    const u32x4 x = d[k];
    if (w == 8) {
      const bool s = ((rb >> 1) >> rot8) & 1;  // the chunk's records in order 1, 0
      const uint32_t a0 = s ? x.z : x.x, a1 = s ? x.w : x.y, b0 = s ? x.x : x.z, b1 = s ? x.y : x.w;
      uint8_t* ra = row + (s ? stride : 0);
      put_slot_nb<HDR>(ra, hdr_bm, slot, (uint64_t)a0 | ((uint64_t)a1 << 32), nul(s), flags);
      put_slot_nb<HDR>(row + (s ? 0 : stride), hdr_bm, slot, (uint64_t)b0 | ((uint64_t)b1 << 32), nul(!s), flags);
    } else if (w == 4) {
      const int s = ((rb >> 2) >> rot4) & 3;  // the chunk's records from record s, wrapping
      // the dwords rotated by s in place (by 2, then by 1): y[e] = x[(e + s) & 3]
      const bool h = s & 2, o = s & 1;
      const uint32_t p0 = h ? x.z : x.x, p1 = h ? x.w : x.y, p2 = h ? x.x : x.z, p3 = h ? x.y : x.w;
      const uint32_t y0 = o ? p1 : p0, y1 = o ? p2 : p1, y2 = o ? p3 : p2, y3 = o ? p0 : p3;
      uint8_t* r0 = row + s * stride;
      const int wrap = 4 * stride;
      put_slot_nb<HDR>(r0, hdr_bm, slot, y0, nul(s), flags);
      put_slot_nb<HDR>(r0 + stride - (s >= 3 ? wrap : 0), hdr_bm, slot, y1, nul((s + 1) & 3), flags);
      put_slot_nb<HDR>(r0 + 2 * stride - (s >= 2 ? wrap : 0), hdr_bm, slot, y2, nul((s + 2) & 3), flags);
      put_slot_nb<HDR>(r0 + 3 * stride - (s >= 1 ? wrap : 0), hdr_bm, slot, y3, nul((s + 3) & 3), flags);
    } else if constexpr (NUL) {  // 2- and 1-byte fields, rolled (the dword of record e picked by selects)
      const int E = 16 / w;
#pragma unroll 1
      for (int e = 0; e < E; ++e) {
        const int q = e / (E / 4);
        const uint32_t wd = q == 0 ? x.x : q == 1 ? x.y : q == 2 ? x.z : x.w;
        const uint32_t v = (wd >> (8 * w * (e % (E / 4)))) & (w == 2 ? 0xffffu : 0xffu);
        put_slot_nb<HDR>(row + e * stride, hdr_bm, slot, v, nul(e), flags);
      }
    } else if (w == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        put_slot<HDR>(row + e * stride, hdr_bm, slot, (x[e >> 1] >> (16 * (e & 1))) & 0xffff, false, flags);
    } else if (w == 1) {
#pragma unroll
      for (int e = 0; e < 16; ++e)
        put_slot<HDR>(row + e * stride, hdr_bm, slot, (x[e >> 2] >> (8 * (e & 3))) & 0xff, false, flags);
    }
  }
}

// Nullable schemas: row r's null bitmap, word j (slots 32j .. 32j + 31), from the tile's
// masks in LDS (BinaryWriter.setNullAt: bit = 1 for null); wave j builds word j of the
// 64 rows (lane = row). Masks past the last field are 0, so are the padding bits.
template <int HDR>
__device__ __forceinline__ void v5_bitmaps(uint8_t* lds, int stride, int nbw, const uint64_t* mt, int wave, int lane) {
  if (wave >= nbw) return;
  const uint64_t* m = mt + 32 * wave;
  uint32_t acc = 0;
#pragma unroll 8
  for (int b = 0; b < 32; ++b) acc |= (uint32_t)((m[b] >> lane) & 1) << b;
  st32(lds + lane * stride + HDR + 4 * wave, acc);
}

// The tile's rows (R * stride contiguous bytes) leave with non-temporal 16-B
// stores: the once-written row stream does not displace L2 lines
// (18.43 -> 18.03 ms at 64M Struct104 rows).
// (OPT & 4, an A/B form only -- scripts/microbench/enc_ab.hip: plain stores instead)
template <int R, int WG, int OPT = 0>
__device__ __forceinline__ void v5_store(const FixedLaunch& L, uint8_t* lds, uint8_t* dst, int tid) {
  const int bytes = R * L.stride;
  const int n16 = bytes >> 4;
  for (int c = tid; c < n16; c += WG)
    if constexpr (OPT & 4) *gp(reinterpret_cast<u32x4*>(dst + c * 16)) = *reinterpret_cast<const u32x4*>(lds + c * 16);
    else __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(lds + c * 16), gp(reinterpret_cast<u32x4*>(dst + c * 16)));
  const int tail4 = (bytes & 15) >> 2;
  if (tid < tail4) st32(dst + n16 * 16 + tid * 4, ld32(lds + n16 * 16 + tid * 4));
}

// LDS store cycles of one v5_write field chunk step over a wave (64 lanes: fields of
// 4 w chunks each, consecutive slots) for a record rotation shift `rot` -- ds_write_b64
// (4 groups of 16 lanes, 2 dwords each) or, in stream frames (4-byte aligned slots), two
// ds_write_b32 (2 groups of 32), banks (address / 4) mod 32 (MI355X_MICROARCH.md, LDS).
// read: the decode's d5_columns instead -- per record a ds_read_b32 of its null-bitmap
// word and one per value dword (2 groups of 32 lanes, banks (address / 4) mod 32).
int v5_store_cycles(int stride, int hdr, int hdr_bm, int w, int rot, bool read = false) {
  const int lpf = 4 * w, E = 16 / w;
  int total = 0;
  for (int e = 0; e < E; ++e) {
    int64_t addr[64];
    for (int l = 0; l < 64; ++l) {
      const int f = l / lpf, c = l % lpf;
      const int q = (e + (rot >= 31 ? 0 : (c >> rot))) % E;
      addr[l] = (int64_t)(c * E + q) * stride + hdr_bm + 8 * f;
    }
    const bool b32 = read || hdr == 12;
    const int groups = b32 ? 2 : 4, gl = 64 / groups;
    const int reads = read ? 1 + w / 4 : (hdr == 12 ? 2 : 1);  // instructions per step
    for (int d = 0; d < reads; ++d)
      for (int g = 0; g < groups; ++g) {
        int load[32] = {0};
        for (int l = g * gl; l < (g + 1) * gl; ++l) {
          // (read: instruction 0 is the bitmap word, at the row start + hdr)
          const int64_t a = read && d == 0 ? addr[l] - hdr_bm - 8 * (l / lpf) + hdr : addr[l] + 4 * (read ? d - 1 : d);
          for (int dw = 0; dw < (b32 ? 1 : 2); ++dw) ++load[(a / 4 + dw) % 32];
        }
        int mx = 0;
        for (int b = 0; b < 32; ++b) mx = load[b] > mx ? load[b] : mx;
        total += mx;
      }
  }
  return total;
}

// XCD-grouped tile order: workgroups are dispatched round-robin over the 8 XCDs
// (workgroup b on XCD b % 8), so in dispatch order every XCD takes every 8th tile.
// Within each block of 8*C consecutive logical tiles the C tiles one XCD's
// workgroups take are made contiguous: each XCD's L2 and write stream see one run
// of C tiles. In-process A/B at 64Mi Struct104 rows on four boxes
// (scripts/microbench/fixed_ab.hip, profiles/r02/ab_fixed_*.jsonl), dispatch order
// vs grouped: encode R64/WG512 19.16 -> 17.85, 18.08 -> 17.29, 18.13 -> 18.95,
// 17.89 -> 17.80 ms; R64/WG1024 grouped 17.20, 18.12, 17.82 / 17.61 ms. One run
// per XCD over the whole batch (C = tiles / 8) did better still for the encode
// (launch_encode_v5); decode v5 is fastest in dispatch order (15.15 vs 15.68 ms
// grouped, 15.89 XCD-blocked). C = 0: dispatch order. The last partial block
// keeps the dispatch order.
__device__ __forceinline__ int64_t map_tile(int64_t t, int64_t tiles, int64_t C) {
  if (C <= 0) return t;
  const int64_t blk = t / (8 * C);
  if ((blk + 1) * 8 * C > tiles) return t;
  const int64_t b = t - blk * 8 * C;
  return blk * 8 * C + (b % 8) * C + b / 8;
}

template <int R, int WG, int K, int HDR, int OPT, bool NUL>
__device__ __forceinline__ void encode_v5_body(const FixedLaunch& L, const FixedFieldDev* __restrict__ fields,
                                               uint8_t* __restrict__ out, int64_t tiles, int64_t xcd_run) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int NW = WG / 64;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int stride = L.stride;
  const int hdr_bm = HDR + L.bitmap_bytes;
  int64_t t = blockIdx.x;
  if (t >= tiles) return;

  const uint8_t* dummy = fields[L.group[0]].values;  // any valid column (never null: num_rows > 0)
  const uint8_t* ptr[K];
  int wk[K];
  uint32_t sf[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    int w = 0, p0 = 0, pend = 0;
    const bool ok = v3_insn<R>(wave + k * NW, L, &w, &p0, &pend);
    wk[k] = ok ? w : 0;  // absent instruction: width 0 -> re-reads the dummy address
    const int cpf = R * (ok ? w : 8) / 16;
    const int p = p0 + lane / cpf, c = lane % cpf;
    ptr[k] = dummy;
    sf[k] = 0;
    if (ok && p < pend) {
      const FixedFieldDev& fd = fields[p];
      const int rb = c * (16 / w);
      ptr[k] = fd.values + c * 16;
      sf[k] = (uint32_t)fd.slot | ((uint32_t)fd.flags << 16) | (1u << 20) | ((uint32_t)rb << 21);
    }
  }
  // Nullable schemas: lane l of wave w loads the tile's Arrow validity word (64 records,
  // 8 bytes) of slot 64 w + l with the tile's column chunks (one more load per lane and
  // tile; lanes without a nullable slot re-read the table). A stage ahead of its tile the
  // words go into an LDS mask table (two, by stage parity): the chunk writes zero null
  // slots from it and v5_bitmaps builds whole bitmap words -- no atomics, no per-chunk
  // validity loads, no bitmap re-zeroing (round 4's NUL form: ~90 VGPRs, one workgroup
  // per CU).
  const int nmask = (L.num_fields + 63) & ~63;
  uint64_t* mtab = reinterpret_cast<uint64_t*>(lds + R * stride);  // [2][nmask]
  const uint8_t* vw = reinterpret_cast<const uint8_t*>(L.slot_validity);
  bool vw_on = false;
  if constexpr (NUL) {
    const int sl = 64 * wave + lane;
    const uint8_t* v = sl < L.num_fields && FORY_DBG(sl >= 0, kDbgEncTable, sl, L.num_fields)
                           ? L.slot_validity[sl] : nullptr;
    vw_on = v != nullptr;
    if (vw_on) vw = v;
  }
  // frame header + zeroed bitmaps; the header is constant across tiles (nullable
  // schemas: v5_bitmaps rewrites whole bitmap words per tile)
  if (tid < R) put_header<HDR>(lds + tid * stride, L);
  u32x4 dA[K], dB[K];
  uint64_t mA = 0, mB = 0;
  const int64_t last = tiles - 1;
  // logical tile t -> tile map_tile(t): xcd_run = grid / 8 (each step's grid tiles,
  // one contiguous run per XCD) or 0
  // OPT & 2: blocked order (A/B) -- workgroup b walks tiles [b*per, (b+1)*per) in order
  const int64_t per = (tiles + gridDim.x - 1) / gridDim.x;
  auto mt = [&](int64_t x) -> int64_t {
    if constexpr (OPT & 2) return min((x % (int64_t)gridDim.x) * per + x / (int64_t)gridDim.x, last);
    return map_tile(x, tiles, xcd_run);
  };
  int64_t tend = tiles;
  if constexpr (OPT & 2) {  // this workgroup's logical steps: x = b + j * grid while its tile < tiles
    const int64_t mine = min(per, tiles - (int64_t)blockIdx.x * per);
    if (mine <= 0) return;
    tend = (int64_t)blockIdx.x + mine * gridDim.x;
  }
  auto issue = [&](int64_t tile, u32x4 (&d)[K], uint64_t& m) {
#ifdef FORY_DEBUG_BOUNDS
    if (!FORY_DBG(tile >= 0 && (tile + 1) * R <= L.num_rows, kDbgEncTile, tile, L.num_rows)) tile = 0;
    const bool mask_ok = !vw_on || FORY_DBG(tile * 8 + 8 <= (L.num_rows + 7) / 8, kDbgEncMask, tile, L.num_rows);
#else
    constexpr bool mask_ok = true;
#endif
    if constexpr (NUL) m = *gp(reinterpret_cast<const uint64_t*>(vw_on && mask_ok ? vw + tile * 8 : vw));  // masks first
    v5_issue<R, K, OPT>(ptr, wk, tile * R, d);
  };
  auto put_masks = [&](uint64_t m, int b) {  // (Arrow: 1 = valid; rows: 1 = null)
    if constexpr (NUL)
      if (64 * wave < nmask) mtab[b * nmask + 64 * wave + lane] = vw_on ? ~m : 0ull;
  };
  issue(mt(t), dA, mA);
  issue(mt(min(t + (int64_t)gridDim.x, tend - 1)), dB, mB);
  put_masks(mA, 0);
  if constexpr (NUL) __syncthreads();
  const int nbw = L.bitmap_bytes >> 2;
  // stage of set X (tile t, masks in table bx); the other set's masks go into table by
  auto stage = [&](u32x4 (&d)[K], uint64_t& m, int bx, uint64_t mo, int by) {
    v5_write<R, K, HDR, NUL>(lds, stride, hdr_bm, wk, sf, d, mtab + bx * nmask, L.rot4, L.rot8);
    if constexpr (NUL) v5_bitmaps<HDR>(lds, stride, nbw, mtab + bx * nmask, wave, lane);
    __syncthreads();
    put_masks(mo, by);  // (loaded a stage ago; only the other set's chunks are younger)
    if (FORY_DBG(mt(t) >= 0 && (mt(t) + 1) * R <= L.num_rows, kDbgEncStore, mt(t), L.num_rows))
      v5_store<R, WG, OPT>(L, lds, out + mt(t) * R * stride, tid);
    issue(mt(min(t + 2 * (int64_t)gridDim.x, tend - 1)), d, m);
    __syncthreads();
    t += gridDim.x;
  };
  for (;;) {
    stage(dA, mA, 0, mB, 1);
    if (t >= tend) break;
    stage(dB, mB, 1, mA, 0);
    if (t >= tend) break;
  }
}

// Round 4's NUL form (per-chunk validity loads, atomics into the bitmaps) took ~90
// VGPRs: one 1024-thread workgroup per CU instead of two; 5.56 vs 4.69 ms for not-null
// at 16Mi rows. The mask-table form above takes 76-78: still one workgroup per CU (held
// to 64 for two it spilled 14-18 and measured 5.42 vs 5.19 ms at 16Mi boxed rows,
// profiles/r05/nullable/); encode 5.56 -> 5.19 ms raw, 5.37 -> 4.84 ms frames.
template <int R, int WG, int K, int HDR, int OPT = 0, bool NUL = false>
__global__ __launch_bounds__(WG, 1) void encode_fixed_v5_kernel(FixedLaunch L, const FixedFieldDev* __restrict__ fields,
                                                                 uint8_t* __restrict__ out, int64_t tiles,
                                                                 int64_t xcd_run) {
  encode_v5_body<R, WG, K, HDR, OPT, NUL>(L, fields, out, tiles, xcd_run);
}

// ---------------------------------------------------------------------------
// Fixed-width decode: rows -> columns
// ---------------------------------------------------------------------------
// LDS-DMA of `bytes` contiguous bytes into the LDS image (1 KiB per wave
// instruction; lanes past the end masked off).
// NT & 4: non-temporal policy (aux = 2) on the once-read row stream.
template <int NT = 0>
__device__ __forceinline__ void dma_tile(uint8_t* lds, const uint8_t* __restrict__ src, int bytes, int tid, int wave) {
  const int n16 = bytes >> 4;
  for (int c0 = 0; c0 < n16; c0 += kWG) {
    const int c = c0 + tid;
    if (c < n16)
      __builtin_amdgcn_global_load_lds((const GAS void*)(src + (int64_t)c * 16),
                                       (__attribute__((address_space(3))) void*)(lds + (c0 + wave * 64) * 16), 16,
                                       0, (NT & 4) ? 2 : 0);
  }
  const int tail4 = (bytes & 15) >> 2;
  if (tid < tail4) st32(lds + n16 * 16 + tid * 4, ld32(src + n16 * 16 + tid * 4));
}

template <int HDR>
__device__ __forceinline__ void check_frame(const uint8_t* row, const FixedLaunch& L, int32_t* status) {
  if (HDR == 8) {  // Encoder.decode(byte[]): the schema hash only (Encoders.java:181-190, 195-197)
    const uint64_t h = (uint64_t)ld32(row) | ((uint64_t)ld32(row + 4) << 32);
    if (h != (uint64_t)L.schema_hash) set_status(status, FORY_ERR_SCHEMA_MISMATCH);
    return;
  }
  // Encoders.decode (Encoders.java:177-190): size, then the schema hash.
  const uint32_t len = ld32(row);
  const uint64_t h = (uint64_t)ld32(row + 4) | ((uint64_t)ld32(row + 8) << 32);
  if (h != (uint64_t)L.schema_hash) set_status(status, FORY_ERR_SCHEMA_MISMATCH);
  else if (len != (uint32_t)(8 + L.fixed_size)) set_status(status, FORY_ERR_CORRUPT);
}

// Slot of an LDS row (UnsafeTrait.getX: the low W bytes).
template <int W, int HDR>
__device__ __forceinline__ uint64_t get_slot(const uint8_t* row, int hdr_bm, int slot) {
  const uint8_t* p = row + hdr_bm + 8 * slot;
  if constexpr (W == 8) {
    if (HDR == 12) return (uint64_t)ld32(p) | ((uint64_t)ld32(p + 4) << 32);
    return *reinterpret_cast<const uint64_t*>(p);
  }
  return ld32(p);
}

// Arrow validity of field fd for the TR records of this lane group.
template <int TR>
__device__ __forceinline__ void put_validity(const FixedFieldDev& fd, bool isnull, bool live, int r, int fsub,
                                             int64_t r0, int rows) {
  const uint64_t m = __ballot(!isnull && live);
  if (r == 0) {
    const uint64_t mine = (m >> (fsub * TR)) & (TR == 64 ? ~0ull : ((1ull << TR) - 1));
    uint8_t* vb = fd.out_validity + (r0 >> 3);
    const int nb = (rows + 7) >> 3;
    for (int b = 0; b < nb; ++b)
      if (FORY_DBG((r0 >> 3) + b < (r0 + rows + 7) / 8, kDbgTailValid, r0 + 8 * b, r0 + rows))
        store_byte(vb + b, (uint8_t)(mine >> (8 * b)));
  }
}

// Decodes slot values of one width group: null -> 0 (RowEncoderBuilder.java:239-246),
// bool -> 0/1 (MemoryBuffer.getBoolean), coalesced column stores.
template <int W, int TR, int HDR, int NT = 0>
__device__ __forceinline__ void dec_group(const FixedFieldDev* __restrict__ fields, int g0, int g1, int wave, int fsub,
                                          int r, const uint8_t* row, int hdr_bm, int hdr, bool live, int64_t grow,
                                          int64_t r0, int rows) {
  constexpr int FPW = 64 / TR;
  constexpr int FSTEP = kWaves * FPW;
  constexpr int U = 8;
  for (int pb = g0 + wave * FPW; pb < g1; pb += FSTEP * U) {
    uint64_t x[U];
    bool nul[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = field_of<TR>(pb, u, FSTEP, fsub);
      x[u] = 0;
      nul[u] = true;
      if (p < g1) {
        const int slot = fields[p].slot;
        nul[u] = (ld32(row + hdr + ((slot >> 5) << 2)) >> (slot & 31)) & 1;  // BinaryRow.isNullAt
        x[u] = get_slot<W, HDR>(row, hdr_bm, slot);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = field_of<TR>(pb, u, FSTEP, fsub);
      if (p < g1) {
        const FixedFieldDev& fd = fields[p];
        uint64_t v = nul[u] ? 0 : x[u];
        if (fd.flags & 2) v = (v & 0xff) ? 1 : 0;
        if (live) {
          if constexpr ((NT & 8) && W >= 4) {  // non-temporal column stores
            if constexpr (W == 8) __builtin_nontemporal_store(v, gp(reinterpret_cast<uint64_t*>(fd.out_values)) + grow);
            else __builtin_nontemporal_store((uint32_t)v, gp(reinterpret_cast<uint32_t*>(fd.out_values)) + grow);
          } else {
            stw<W>(fd.out_values, grow, v);
          }
        }
        if ((fd.flags & 1) && fd.out_validity) put_validity<TR>(fd, nul[u], live, r, fsub, r0, rows);
      }
    }
  }
}

template <int TR, int HDR, int NT = 0>
__global__ __launch_bounds__(kWG) void decode_fixed_kernel(FixedLaunch L, const FixedFieldDev* __restrict__ fields,
                                                           const uint8_t* __restrict__ in, int32_t* status) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane % TR;
  const int fsub = lane / TR;
  const int64_t r0 = (L.tile0 + map_tile((int64_t)blockIdx.x, gridDim.x, L.xcd_run)) * TR;
  const int64_t left = L.num_rows - r0;
  const int rows = left < TR ? (int)left : TR;
  const int stride = L.stride;
  const int hdr_bm = HDR + L.bitmap_bytes;

  if (FORY_DBG(r0 >= 0 && r0 + rows <= L.num_rows, kDbgTailLoad, r0, L.num_rows))
    dma_tile<NT>(lds, in + r0 * stride, rows * stride, tid, wave);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const uint8_t* row = lds + r * stride;
  const int64_t grow = r0 + r;
  const bool live = r < rows;
  if (HDR && wave == 0 && fsub == 0 && live) check_frame<HDR>(row, L, status);
  dec_group<8, TR, HDR, NT>(fields, L.group[0], L.group[1], wave, fsub, r, row, hdr_bm, HDR, live, grow, r0, rows);
  dec_group<4, TR, HDR, NT>(fields, L.group[1], L.group[2], wave, fsub, r, row, hdr_bm, HDR, live, grow, r0, rows);
  dec_group<2, TR, HDR, NT>(fields, L.group[2], L.group[3], wave, fsub, r, row, hdr_bm, HDR, live, grow, r0, rows);
  dec_group<1, TR, HDR, NT>(fields, L.group[3], L.group[4], wave, fsub, r, row, hdr_bm, HDR, live, grow, r0, rows);
}

// ---------------------------------------------------------------------------
// Decode v5: the encode v5 mirrored. Persistent workgroups; the row stream of a
// tile (R * stride contiguous bytes) comes in as K 16-B chunks per thread, two
// tiles in flight in registers (sets A/B, the loop unrolled by 2; every thread
// issues exactly K loads per tile, inactive ones re-read chunk 0, so the compiler
// waits with a counted vmcnt for the older set while the younger set and the
// column stores stay in flight: no vmcnt(0) drain per tile). Per stage: rows ->
// LDS -> barrier -> each lane gathers ONE field's 16-B column chunk (E = 16/w
// consecutive records, null -> 0, bool -> 0/1) and stores it non-temporally
// (one 1-KiB wave instruction per FPI fields, numbered like the encode's,
// v3_insn_g) -> issue the rows of tile + 2*grid -> barrier. Schemas whose column
// chunks fit K2 instructions per wave; nullable ones also write the Arrow validity
// (NUL form, d5_validity). Null bits are always read: a set bit decodes to 0, as
// in decode_fixed_kernel.
// (OPT & 8, an A/B form only -- scripts/microbench/enc_ab.hip: plain row loads)
template <int R, int K, int OPT = 0>
__device__ __forceinline__ void d5_issue(const uint8_t* in, int64_t base, int stride, int tid, int n16, int WGT,
                                         u32x4 (&d)[K], int64_t num_rows) {
  if (!FORY_DBG(base >= 0 && base + R <= num_rows, kDbgDecTile, base, num_rows)) base = 0;
  const uint8_t* tile = in + base * stride;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int c = tid + k * WGT;
    const u32x4* a = reinterpret_cast<const u32x4*>(tile + (int64_t)(c < n16 ? c : 0) * 16);
    if constexpr (OPT & 8) d[k] = *gp(a);
    else d[k] = __builtin_nontemporal_load(gp(a));
  }
}

template <int K>
__device__ __forceinline__ void d5_write(uint8_t* lds, int tid, int n16, int WGT, const u32x4 (&d)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int c = tid + k * WGT;
    if (c < n16) *reinterpret_cast<u32x4*>(lds + c * 16) = d[k];
  }
}

// Nullable schemas (NUL): the Arrow validity of the tile's 64 records, per slot, from the
// rows' null bitmaps in LDS. Wave w takes slots [64 w, 64 w + 64): lane r reads the two
// bitmap words of row r that hold them, a ballot per slot gives the slot's 64 null bits
// across the tile (BinaryRow.isNullAt), and lane s keeps slot 64 w + s's word and stores
// it, inverted (Arrow: 1 = valid), as 8 bytes at the tile's byte offset of the field's
// validity (vo: the output validity of slot 64 w + lane, or null). One LDS read and 64
// ballots per wave and tile instead of a bitmap read per record and chunk.
template <int HDR>
__device__ __forceinline__ void d5_validity(const uint8_t* lds, int stride, int nbits, uint8_t* vo, int64_t tile,
                                            int wave, int lane, int64_t num_rows) {
  if (64 * wave >= nbits) return;
  const uint8_t* bm = lds + lane * stride + HDR + 8 * wave;
  const uint32_t lo = ld32(bm), hi = 64 * wave + 32 < nbits ? ld32(bm + 4) : 0u;
  uint64_t mine = 0;
#pragma unroll 8
  for (int b = 0; b < 64; ++b) {
    const uint32_t wd = b < 32 ? lo : hi;
    const uint64_t nb = __ballot((wd >> (b & 31)) & 1);
    mine = lane == b ? nb : mine;
  }
  if (vo && FORY_DBG(tile >= 0 && tile * 8 + 8 <= (num_rows + 7) / 8, kDbgDecValid, tile, num_rows))
    *gp(reinterpret_cast<uint64_t*>(vo + tile * 8)) = ~mine;
}

// (OPT & 4, an A/B form only: plain column stores)
template <int R, int K2, int HDR, int OPT = 0>
__device__ __forceinline__ void d5_columns(const uint8_t* lds, int stride, int hdr_bm, const int (&wk)[K2],
                                           const uint32_t (&sf)[K2], uint8_t* const (&optr)[K2], int64_t r0,
                                           int rot4, int rot8, int64_t num_rows) {
#pragma unroll
  for (int k = 0; k < K2; ++k) {
    if (!(sf[k] & (1u << 20))) continue;
    const int w = wk[k];
    const int slot = sf[k] & 0xffff, flags = (sf[k] >> 16) & 0xf, rb = sf[k] >> 21;
    const uint8_t* row = lds + rb * stride;
    const int bmo = HDR + ((slot >> 5) << 2);
    const uint32_t bit = 1u << (slot & 31);
    auto val = [&](int e) -> uint64_t {  // UnsafeTrait.getX of record rb + e; null -> 0
      const uint8_t* r = row + e * stride;
      if (ld32(r + bmo) & bit) return 0;
      const uint8_t* p = r + hdr_bm + 8 * slot;
      return w == 8 ? ((uint64_t)ld32(p) | ((uint64_t)ld32(p + 4) << 32)) : (uint64_t)ld32(p);
    };
    u32x4 x;
    if (w == 8) {  // the chunk's records read in order 1, 0 on lanes with s (LDS bank spread, v5_rotation)
      const bool s = ((rb >> 1) >> rot8) & 1;
      const uint64_t a = val(s ? 1 : 0), b = val(s ? 0 : 1);
      const uint64_t v0 = s ? b : a, v1 = s ? a : b;
      x = u32x4{(uint32_t)v0, (uint32_t)(v0 >> 32), (uint32_t)v1, (uint32_t)(v1 >> 32)};
    } else if (w == 4) {  // records read from record s, wrapping; y[e] = record (e + s) & 3
      const int s = ((rb >> 2) >> rot4) & 3;
      const uint32_t y0 = (uint32_t)val(s), y1 = (uint32_t)val((s + 1) & 3), y2 = (uint32_t)val((s + 2) & 3),
                     y3 = (uint32_t)val((s + 3) & 3);
      // x[j] = y[(j - s) & 3]: rotate back by s (by 2, then by 1)
      const bool h = s & 2, o = s & 1;
      const uint32_t p0 = h ? y2 : y0, p1 = h ? y3 : y1, p2 = h ? y0 : y2, p3 = h ? y1 : y3;
      x = u32x4{o ? p3 : p0, o ? p0 : p1, o ? p1 : p2, o ? p2 : p3};
    } else {
      // 2- and 1-byte fields: one dword (2 or 4 records) per iteration of a rolled
      // loop, placed by selects; unrolled, the 16 records' LDS reads were all hoisted
      // and the kernel spilled ~30 VGPRs on every schema (this branch is cold for
      // Struct104, the spill code was not)
      const int per = 4 / w;  // records per dword
      uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
#pragma unroll 1
      for (int q = 0; q < 4; ++q) {
        uint32_t acc = 0;
        for (int e = 0; e < per; ++e) {
          uint32_t b = (uint32_t)val(per * q + e) & (w == 2 ? 0xffffu : 0xffu);
          if (flags & 2) b = b ? 1 : 0;  // MemoryBuffer.getBoolean
          acc |= b << (8 * w * e);
        }
        h0 = q == 0 ? acc : h0;
        h1 = q == 1 ? acc : h1;
        h2 = q == 2 ? acc : h2;
        h3 = q == 3 ? acc : h3;
      }
      x = u32x4{h0, h1, h2, h3};
    }
    if (FORY_DBG(r0 + rb + 16 / w <= num_rows, kDbgDecStore, r0 + rb, num_rows)) {
      if constexpr (OPT & 4) *gp(reinterpret_cast<u32x4*>(optr[k] + r0 * w)) = x;
      else __builtin_nontemporal_store(x, gp(reinterpret_cast<u32x4*>(optr[k] + r0 * w)));
    }
  }
}

template <int R, int WG, int K, int K2, int HDR, int OPT = 0, bool NUL = false>
__global__ __launch_bounds__(WG, 1) void decode_fixed_v5_kernel(FixedLaunch L,
                                                                 const FixedFieldDev* __restrict__ fields,
                                                                 const uint8_t* __restrict__ in, int64_t tiles,
                                                                 int32_t* status) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int NW = WG / 64;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int stride = L.stride;
  const int hdr_bm = HDR + L.bitmap_bytes;
  const int n16 = R * stride / 16;
  int64_t t = blockIdx.x;
  if (t >= tiles) return;

  int wk[K2];
  uint32_t sf[K2];
  uint8_t* optr[K2];
#pragma unroll
  for (int k = 0; k < K2; ++k) {
    int w = 0, p0 = 0, pend = 0;
    const bool ok = v3_insn<R>(wave + k * NW, L, &w, &p0, &pend);
    wk[k] = ok ? w : 8;
    const int cpf = R * wk[k] / 16;
    const int p = p0 + lane / cpf, c = lane % cpf;
    sf[k] = 0;
    optr[k] = nullptr;
    if (ok && p < pend) {
      const FixedFieldDev& fd = fields[p];
      const int rb = c * (16 / w);
      sf[k] = (uint32_t)fd.slot | ((uint32_t)fd.flags << 16) | (1u << 20) | ((uint32_t)rb << 21);
      optr[k] = fd.out_values + (int64_t)rb * w;
    }
  }
  // NUL: the output validity of slot 64 * wave + lane (d5_validity)
  uint8_t* vo = nullptr;
  if constexpr (NUL) {
    const int sl = 64 * wave + lane;
    if (sl < L.num_fields && FORY_DBG(sl >= 0, kDbgEncTable, sl, L.num_fields))
      vo = const_cast<uint8_t*>(L.slot_validity[sl]);
  }
  const int nbits = L.bitmap_bytes * 8;
  u32x4 dA[K], dB[K];
  const int64_t last = tiles - 1;
  // OPT & 2: blocked order -- workgroup b walks tiles [b*per, (b+1)*per) in order
  const int64_t per = (tiles + gridDim.x - 1) / gridDim.x;
  auto mt = [&](int64_t x) -> int64_t {
    if constexpr (OPT & 2) return min((x % (int64_t)gridDim.x) * per + x / (int64_t)gridDim.x, last);
    return map_tile(x, tiles, L.xcd_run);
  };
  int64_t tend = tiles;
  if constexpr (OPT & 2) {
    const int64_t mine = min(per, tiles - (int64_t)blockIdx.x * per);
    if (mine <= 0) return;
    tend = (int64_t)blockIdx.x + mine * gridDim.x;
  }
  d5_issue<R, K, OPT>(in, mt(t) * R, stride, tid, n16, WG, dA, L.num_rows);
  d5_issue<R, K, OPT>(in, mt(min(t + (int64_t)gridDim.x, tend - 1)) * R, stride, tid, n16, WG, dB, L.num_rows);
  auto stage = [&](u32x4 (&d)[K]) {
    d5_write<K>(lds, tid, n16, WG, d);
    __syncthreads();
    if (HDR && tid < R) check_frame<HDR>(lds + tid * stride, L, status);
    d5_columns<R, K2, HDR, OPT>(lds, stride, hdr_bm, wk, sf, optr, mt(t) * R, L.drot4, L.drot8, L.num_rows);
    if constexpr (NUL) d5_validity<HDR>(lds, stride, nbits, vo, mt(t), wave, lane, L.num_rows);
    d5_issue<R, K, OPT>(in, mt(min(t + 2 * (int64_t)gridDim.x, tend - 1)) * R, stride, tid, n16, WG, d, L.num_rows);
    __syncthreads();
    t += gridDim.x;
  };
  for (;;) {
    stage(dA);
    if (t >= tend) break;
    stage(dB);
    if (t >= tend) break;
  }
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
// Encode v5: R = 64 records per tile, 1024 threads (two workgroups per CU: LDS),
// <= 3 chunk loads per wave per tile (Struct104: 39 load instructions over 16
// waves), nt column loads and row stores, XCD-blocked tile order (map_tile with
// runs of tiles/8: every XCD walks one contiguous eighth of the batch, its
// workgroups on adjacent tiles). In-process A/B at 64Mi Struct104 rows on two
// boxes (profiles/r02/ab_order_box*.jsonl): runs of grid/8 17.98 / 17.53 ms,
// XCD-blocked 16.45 / 16.35, + nt column loads 16.38 / 16.12.
constexpr int kV5R = 64, kV5WG = 1024, kV5K = 3;
#ifndef FORY_V5R_NOTNULL  // (build-time A/B: records per tile of the not-null encode)
#define FORY_V5R_NOTNULL 64
#endif

template <int HDR, bool NUL>
hipError_t launch_encode_v5(const FixedLaunch& L, uint8_t* out, hipStream_t s) {
  constexpr int R = NUL ? kV5R : FORY_V5R_NOTNULL, K = R == 128 ? 5 : kV5K;
  const int64_t full = L.num_rows / R;
  if (full > 0) {
    auto* k = &encode_fixed_v5_kernel<R, kV5WG, K, HDR, 1, NUL>;
    raise_lds_cap(k);
    const size_t lds = (size_t)R * L.stride + (NUL ? (size_t)2 * 8 * ((L.num_fields + 63) & ~63) : 0);
    const int64_t grid = persistent_grid(k, lds, full, kV5WG);
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(kV5WG), lds, s, L, L.fields, out, full, (int64_t)(full / 8));
  }
  if (L.num_rows > full * R) {  // tail (< R records): one-tile kernel
    FixedLaunch T = L;
    T.tile0 = full * R / 64;
    auto* k = &encode_fixed_kernel<64, HDR>;
    raise_lds_cap(k);
    const int64_t tail_tiles = (L.num_rows - full * R + 63) / 64;
    hipLaunchKernelGGL(k, dim3((unsigned)tail_tiles), dim3(kWG), (size_t)64 * L.stride, s, T, L.fields, out);
  }
  return hipGetLastError();
}

template <int TR, int HDR>
hipError_t launch_encode_tr(const FixedLaunch& L, uint8_t* out, hipStream_t s) {
  const int64_t tiles = (L.num_rows + TR - 1) / TR;
  const size_t lds = (size_t)TR * L.stride;
  if constexpr (TR == 64) {
    // v5: schemas whose chunk instructions fit K per wave (nullable ones: the NUL form)
    // nullable: the mask-table form needs 8-byte aligned validity words and a mask wave
    // per 64 slots, a bitmap word per wave
    constexpr int RN = FORY_V5R_NOTNULL, KN = RN == 128 ? 5 : kV5K;  // the not-null form's tile
    if ((L.any_nullable ? (v3_insn_count<kV5R>(L.group) + kV5WG / 64 - 1) / (kV5WG / 64) <= kV5K
                        : (v3_insn_count<RN>(L.group) + kV5WG / 64 - 1) / (kV5WG / 64) <= KN) &&
        (!L.any_nullable || (L.valid8 && L.num_fields <= 64 * (kV5WG / 64) && L.bitmap_bytes / 4 <= kV5WG / 64)))
      return L.any_nullable ? launch_encode_v5<HDR, true>(L, out, s) : launch_encode_v5<HDR, false>(L, out, s);
  }
  auto* k = &encode_fixed_kernel<TR, HDR>;
  raise_lds_cap(k);
  hipLaunchKernelGGL(k, dim3((unsigned)tiles), dim3(kWG), lds, s, L, L.fields, out);
  return hipGetLastError();
}

// Decode v5: 64 records per tile, 1024 threads (LDS: two workgroups per CU), <= 4
// row-chunk loads per thread (stride <= 1024 B), <= 3 column-chunk instructions
// per wave. In-process A/B at 64Mi Struct104 rows (scripts/microbench/fixed_ab.hip,
// profiles/r02/ab_dec5.jsonl): 17.51 -> 15.31 ms; WG 512 15.65, WG 256 18.00.
constexpr int kD5R = 64, kD5WG = 1024, kD5K = 4, kD5K2 = 3;

#ifndef FORY_D5R_NOTNULL  // (build-time A/B: records per tile of the not-null decode)
#define FORY_D5R_NOTNULL 64
#endif
constexpr int kD5RN = FORY_D5R_NOTNULL, kD5KN = kD5RN == 128 ? 7 : kD5K, kD5K2N = kD5RN == 128 ? 5 : kD5K2;

template <int HDR>
bool decode_v5_fits(const FixedLaunch& L) {
  if (!L.any_nullable)
    return L.cols_aligned16 && kD5RN * L.stride <= kD5KN * kD5WG * 16 && (kD5RN * L.stride) % 16 == 0 &&
           v3_insn_count<kD5RN>(L.group) <= kD5K2N * (kD5WG / 64);
  return L.cols_aligned16 && kD5R * L.stride <= kD5K * kD5WG * 16 &&
         (kD5R * L.stride) % 16 == 0 && v3_insn_count<kD5R>(L.group) <= kD5K2 * (kD5WG / 64) &&
         (!L.any_nullable || (L.valid8 && L.bitmap_bytes * 8 <= 64 * (kD5WG / 64)));
}

template <int HDR>
hipError_t launch_decode_v5(const FixedLaunch& L, const uint8_t* in, int32_t* status, hipStream_t s) {
  // (decode_v5_fits: nullable schemas need 8-byte aligned validity outputs and <= 64 slots per wave)
  const int R = L.any_nullable ? kD5R : kD5RN;
  const int64_t full = L.num_rows / R;
  if (full > 0) {
    auto* k = L.any_nullable ? &decode_fixed_v5_kernel<kD5R, kD5WG, kD5K, kD5K2, HDR, 0, true>
                             : &decode_fixed_v5_kernel<kD5RN, kD5WG, kD5KN, kD5K2N, HDR, 0, false>;
    raise_lds_cap(k);
    const size_t lds = (size_t)R * L.stride;
    const int64_t grid = persistent_grid(k, lds, full, kD5WG);
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(kD5WG), lds, s, L, L.fields, in, full, status);
  }
  if (L.num_rows > full * R) {  // tail (< R records): the one-tile kernel, 64 records per tile
    FixedLaunch T = L;
    T.tile0 = full * R / 64;
    auto* k = &decode_fixed_kernel<64, HDR, 12>;
    raise_lds_cap(k);
    hipLaunchKernelGGL(k, dim3((unsigned)((L.num_rows - full * R + 63) / 64)), dim3(kWG), (size_t)64 * L.stride, s, T,
                       L.fields, in, status);
  }
  return hipGetLastError();
}

template <int TR, int HDR>
hipError_t launch_decode_tr(const FixedLaunch& L, const uint8_t* in, int32_t* status, hipStream_t s) {
  if constexpr (TR == 64) {
    if (decode_v5_fits<HDR>(L)) return launch_decode_v5<HDR>(L, in, status, s);
  }
  const int64_t tiles = (L.num_rows + TR - 1) / TR;
  const size_t lds = (size_t)TR * L.stride;
  // TR = 64: non-temporal LDS-DMA row loads + column stores (17.72 -> 17.52 ms at 64M Struct104)
  auto* k = TR == 64 ? &decode_fixed_kernel<TR, HDR, 12> : &decode_fixed_kernel<TR, HDR, 0>;
  raise_lds_cap(k);
  hipLaunchKernelGGL(k, dim3((unsigned)tiles), dim3(kWG), lds, s, L, L.fields, in, status);
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

namespace {

template <int HDR>
hipError_t encode_hdr(const FixedLaunch& L, uint8_t* out, hipStream_t s) {
  switch (pick_tr(L.stride)) {
    case 64: return launch_encode_tr<64, HDR>(L, out, s);
    case 32: return launch_encode_tr<32, HDR>(L, out, s);
    case 16: return launch_encode_tr<16, HDR>(L, out, s);
    case 8: return launch_encode_tr<8, HDR>(L, out, s);
    default: return hipErrorInvalidValue;
  }
}

template <int HDR>
hipError_t decode_hdr(const FixedLaunch& L, const uint8_t* in, int32_t* status, hipStream_t s) {
  switch (pick_tr(L.stride)) {
    case 64: return launch_decode_tr<64, HDR>(L, in, status, s);
    case 32: return launch_decode_tr<32, HDR>(L, in, status, s);
    case 16: return launch_decode_tr<16, HDR>(L, in, status, s);
    case 8: return launch_decode_tr<8, HDR>(L, in, status, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

// v5_write's rotation shift for w-byte fields at this row layout: the fewest modelled
// LDS store cycles (v5_store_cycles), in order (31) on ties.
int v5_rotation(int stride, int hdr, int hdr_bm, int w, bool read) {
  int best = 31, cyc = v5_store_cycles(stride, hdr, hdr_bm, w, 31, read);
  for (int r = 0; r <= 4; ++r) {
    const int c = v5_store_cycles(stride, hdr, hdr_bm, w, r, read);
    if (c < cyc) best = r, cyc = c;
  }
  return best;
}

// Library-internal, for a CPU test (not in the public header): the rotation v5_rotation
// picks and the modelled store / read cycles of a rotation.
extern "C" int fory_rowfmt_internal_v5_rotation(int stride, int hdr, int hdr_bm, int w, int read) {
  return v5_rotation(stride, hdr, hdr_bm, w, read != 0);
}
extern "C" int fory_rowfmt_internal_v5_cycles(int stride, int hdr, int hdr_bm, int w, int rot, int read) {
  return v5_store_cycles(stride, hdr, hdr_bm, w, rot, read != 0);
}

hipError_t launch_encode_fixed(const FixedLaunch& L, uint8_t* out, hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  switch (frame_header_bytes(L.frame)) {
    case 0: return encode_hdr<0>(L, out, s);
    case 8: return encode_hdr<8>(L, out, s);
    case 12: return encode_hdr<12>(L, out, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_decode_fixed(const FixedLaunch& L, const uint8_t* in, int32_t* status, hipStream_t s) {
  if (L.num_rows <= 0) return hipSuccess;
  switch (frame_header_bytes(L.frame)) {
    case 0: return decode_hdr<0>(L, in, status, s);
    case 8: return decode_hdr<8>(L, in, status, s);
    case 12: return decode_hdr<12>(L, in, status, s);
    default: return hipErrorInvalidValue;
  }
}

bool fixed_tiled_supported(int stride) { return pick_tr(stride) != 0; }

// Library-internal, for the debug-bounds runs (not in the public header): per site the
// violation count and the first offending (value, limit), 3 int64 per site into out[3 *
// n]; returns the number of sites, -1 in a product build (no checks compiled in), -2 on
// a HIP error. The counters are cleared after reading when `clear` is set.
extern "C" int fory_rowfmt_internal_debug_bounds(long long* out, int n, int clear) {
#ifdef FORY_DEBUG_BOUNDS
  DbgSite h[kDbgSites];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_dbg), sizeof h) != hipSuccess) return -2;
  for (int i = 0; i < n && i < kDbgSites; ++i) {
    out[3 * i] = (long long)h[i].count;
    out[3 * i + 1] = h[i].a;
    out[3 * i + 2] = h[i].b;
  }
  if (clear) {
    DbgSite z[kDbgSites] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), z, sizeof z) != hipSuccess) return -2;
  }
  return kDbgSites;
#else
  (void)out;
  (void)n;
  (void)clear;
  return -1;
#endif
}

}  // namespace fory_amd
