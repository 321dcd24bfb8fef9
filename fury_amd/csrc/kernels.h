// kernels.h — launchers for the gfx950 row-format kernels (fixed.hip, scan.hip,
// varlen.hip; launch state in launch_state.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "plan.h"

namespace fory_amd {

// Bytes before the row in each framing (include/fory_rowfmt.h): RAW none, STREAM
// [i32 size][i64 hash], COLLECTION [i32 size] (the payload replaces the row),
// HASHED [i64 hash].
__host__ __device__ inline int frame_header_bytes(int mode) {
  return mode == FORY_FRAME_STREAM ? 12 : mode == FORY_FRAME_HASHED ? 8 : mode == FORY_FRAME_COLLECTION ? 4 : 0;
}

struct FixedLaunch {
  const FixedFieldDev* fields;  // device table
  int32_t num_fields;
  int32_t bitmap_bytes;
  int32_t fixed_size;
  int32_t stride;               // fixed_size (+12 in frame mode)
  int64_t schema_hash;
  int64_t num_rows;
  int32_t any_nullable;
  int32_t frame;
  int32_t group[5];             // table index where the 8/4/2/1-byte groups start; group[4] = num_fields
  int64_t tile0;                // first tile of this launch (tail launches after a persistent kernel)
  int64_t xcd_run;              // XCD-grouped tile order: tiles per XCD run (0 = dispatch order)
  int32_t cols_aligned16;       // decode: every output column 16-byte aligned (decode v5's chunk stores)
  int32_t valid8;               // every validity pointer of slot_validity 8-byte aligned
  int32_t rot4, rot8;           // encode v5: lane c of a 4- / 8-byte field writes its records starting at
                                // (c >> rot) mod records-per-chunk (LDS bank spread; 31 = in order)
  int32_t drot4, drot8;         // decode v5: the same for the records a lane reads
  const uint8_t* const* slot_validity;  // per slot (schema ordinal): the field's validity (encode:
                                        // input, decode: output), null when not nullable / absent
};

hipError_t launch_encode_fixed(const FixedLaunch& L, uint8_t* out, hipStream_t s);
int v5_rotation(int stride, int hdr, int hdr_bm, int w, bool read);
hipError_t launch_decode_fixed(const FixedLaunch& L, const uint8_t* rows, int32_t* status,
                               hipStream_t s);
hipError_t launch_fill_offsets(int64_t* offs, int64_t n, int64_t stride, hipStream_t s);

struct VarLaunch {
  const Op* prog;               // device
  int32_t num_ops;
  const ColumnDev* cols;        // device
  int32_t num_top;
  int32_t bitmap_bytes;
  int32_t fixed_size;
  int64_t schema_hash;
  int64_t num_rows;
  int32_t frame;
  int32_t tile_cap;             // LDS bytes per 64-record tile image (tile engine)
  // Cooperative tile kernels (every plan the device path accepts, up to 32 var
  // fields and kMaxTileStructs nested structs; name kept from when they took
  // flat plans only).
  int32_t flat;
  int32_t num_var;              // OP_BYTES / OP_LIST ops at any struct level, program order
  int32_t stg_bytes;            // LDS staging per wave (slot) for one record group's span
  int32_t nested_fixed;         // fixed bytes of child rows + list headers per record (staging estimate)
  int32_t var_est_row;          // widest var field's static payload estimate per record (decode staging)
  int32_t fix_group[5];         // width groups [8][4][2][1] of `fix`
  const FixedFieldDev* fix;     // device: fixed fields (any struct level), width-sorted
  const VarFieldDev* vf;        // device: var fields (any struct level), program order
  const StructDev* st;          // device: nested struct fields, pre-order (id = index + 1)
  int32_t num_struct;
  uint64_t* prof;               // debug (FORY_ROWFMT_VARPROF): 8 timestamps per tile, else null
  int32_t* spill;               // workspace: tiles spilled to the big-image launch (ceil(n/64))
  int32_t* spill_count;         // workspace: number of spilled tiles
  int64_t mean_row;             // decode: mean row/frame bytes of the batch (tile image sizing), 0 = unknown
  int32_t pl_all;               // encode tile kernel: wave 0 places var payloads too (A/B)
  int32_t iv_split;             // decode tile kernel: the one var field is a list with item validity (wave 1 assembles it)
  int32_t level2;               // decode lengths pass 2: sizes of string/binary list/map
                                // elements (container offsets already scanned)
  LaunchKnobs kn;               // the plan's knobs (host-side launch decisions only)
  int32_t num_list;             // list fields among the var fields
  uint32_t list_mask;           // bit v: var field v is a list (v < 32)
  int32_t nullable;             // bit 0: some fixed column has validity, bit 1: some var column (encode v9)
  int32_t bool_items;           // some list field has bool items (0/1 normalised per item)
  int32_t st_hdr[kMaxTileStructs];  // host copy of each struct's child bitmap bytes (launch sizing)
  int32_t fr_bytes;             // decode totals pass: stage only each record's first fr_bytes (0 = whole rows)
};

// sizes -> d_row_offsets[0..n-1] (row/frame byte sizes), then exclusive scan.
hipError_t launch_var_sizes(const VarLaunch& L, int64_t* d_row_offsets, hipStream_t s);
hipError_t launch_var_encode(const VarLaunch& L, const int64_t* d_row_offsets, uint8_t* out,
                             int64_t capacity, int32_t* status, hipStream_t s);
// decode sizes. Flat plans on the tile engine: per-tile payload totals into
// tile_tot (var_tile_totals_words int64), scanned here, tile bases scattered
// to out_offsets[64 t] and out_offsets[n]; the values pass fills the rest.
// Otherwise: per-row lengths into out_offsets[i+1] (caller scans per column).
hipError_t launch_var_decode_lengths(const VarLaunch& L, const uint8_t* rows,
                                     const int64_t* d_row_offsets, int64_t* tile_tot,
                                     int64_t* partials, int32_t* status, hipStream_t s);
bool var_decode_tiled_offsets(const VarLaunch& L);
int64_t var_tile_totals_words(int64_t num_var, int64_t n);
int64_t var_spill_words(int64_t n);
hipError_t launch_var_decode(const VarLaunch& L, const uint8_t* rows,
                             const int64_t* d_row_offsets, int32_t* status, hipStream_t s);

// Exclusive scan of n int64 values in place; data[n] receives the total.
// partials: >= scan_partials(n) int64 of workspace.
int64_t scan_partials(int64_t n);

// Debug timeline buffer for the flat tile kernels (FORY_ROWFMT_VARPROF=1).
uint64_t* var_prof_buffer(int64_t tiles, bool on);
int64_t var_prof_copy(uint64_t* host, int64_t max_words);
hipError_t launch_scan_i64(int64_t* data, int64_t n, int64_t* partials, hipStream_t s);
// `count` scans of n int64 at data + y * stride in one set of launches; partials:
// scan_multi_partials(n, count) words.
hipError_t launch_scan_i64_multi(int64_t* data, int64_t n, int64_t stride, int count, int64_t* partials,
                                 hipStream_t s);
int64_t scan_multi_partials(int64_t n, int count);
// Arrow offsets columns of one decode level scanned together (lengths at [1..n]).
constexpr int kMaxScanSeg = 16;
struct OffsScanSeg {
  int32_t* offs;
  int64_t n;
  int64_t pofs;  // first partials word
};
struct OffsScanBatch {
  OffsScanSeg seg[kMaxScanSeg];
  int32_t count;
};
int64_t scan_batch_partials(int64_t n);
hipError_t launch_scan_offsets_batch(int32_t* const* cols, const int64_t* n, int count, int64_t* partials,
                                     int32_t* status, hipStream_t s);
// Arrow offsets: offs[1..n] hold lengths; writes offs[0]=0 and inclusive
// prefix into offs[1..n] (int32). Overflow past INT32_MAX sets *status.
hipError_t launch_scan_offsets_i32(int32_t* offs, int64_t n, int64_t* partials,
                                   int32_t* status, hipStream_t s);
// The same over an offsets array of any length with a partials buffer of
// partial_words int64 (segments of 4096 x (partial_words - 1) items, carried).
hipError_t launch_scan_offsets_i32_segmented(int32_t* offs, int64_t n, int64_t* partials, int64_t partial_words,
                                             int32_t* status, hipStream_t s);
// Host decode pipeline: offs[0..n] += base; bits [0, nbits) of src to bits
// [shift, shift + nbits) of dst ((shift + nbits + 7) / 8 bytes, zero elsewhere).
hipError_t launch_offsets_add(int32_t* offs, int64_t n, int32_t base, hipStream_t s);
hipError_t launch_bits_shift(const uint8_t* src, int64_t nbits, uint8_t* dst, int shift, hipStream_t s);

// Tree engine (generic.hip): any nesting, one lane per record.
struct GenLaunch {
  const GNode* nodes;      // device, pre-order (index = column index)
  const ColumnDev* cols;   // device
  int32_t num_nodes;
  int32_t bitmap_bytes;
  int32_t fixed_size;
  int32_t frame;
  int64_t schema_hash;
  int64_t num_rows;
  int32_t fill_level;      // decode: lengths pass of container depth L (>= 0), or -1 = values
  int32_t max_depth;       // schema depth (Plan::max_depth): frames per lane
};
hipError_t launch_gen_sizes(const GenLaunch& L, int64_t* sizes, hipStream_t s);
hipError_t launch_gen_encode(const GenLaunch& L, const int64_t* offs, uint8_t* out, int64_t capacity,
                             int32_t* status, hipStream_t s);
hipError_t launch_gen_decode(const GenLaunch& L, const uint8_t* rows, const int64_t* offs, int32_t* status,
                             hipStream_t s);

// Columnar tree engine (treecol.hip): the tree engine's encode as per-node passes over
// instance columns. An instance is one element of a schema node's column (a row of a
// top-level field, a struct child of an instance, a list item / map entry). Sizes go
// bottom-up (A[c][j] = bytes instance j of var node c adds to its parent; item nodes
// are scanned in place, A[x][m] = total); then the writes go top-down, one pass per var
// node: each instance writes its whole fixed part at its position P[c][j] and hands its
// var children theirs (-1: absent or null), so every output byte is written once.
constexpr int kTcMaxNodes = 128;  // plans with more nodes keep the per-lane engine
struct TcVar {     // a var node (string / decimal / struct / list / map)
  int32_t node;    // schema node (column index)
  int32_t parent;  // entry of the parent (-1: the row)
  int32_t items;   // 1: the parent is a list / map and this node its items / keys / values
  int32_t depth;   // 1 + the parent's depth (top-level fields: 1)
};
struct TcTables {               // device, in the workspace
  int64_t* A[kTcMaxNodes];      // var nodes: sizes (items: exclusive prefix, total at [m]); else null
  int64_t* P[kTcMaxNodes];      // var nodes: output positions of the instances (-1 = none); else null
  int64_t m[kTcMaxNodes];       // instances of each node in this call
  int32_t vidx[kTcMaxNodes];    // node -> entry, -1 for scalars
  TcVar var[kTcMaxNodes];       // entries by depth, pre-order within a depth
  int32_t kids[kTcMaxNodes];    // fields by parent: the rows' top-level fields, then each bean's
  int32_t kid0[kTcMaxNodes];    // bean node -> its first field in kids
  int32_t nvar, depths, nroot;  // nroot: top-level fields
};
hipError_t launch_tc_sizes(const GenLaunch& L, const TcTables* T, int node, int64_t m, bool root_coll, hipStream_t s);
hipError_t launch_tc_rows(const GenLaunch& L, const TcTables* T, int64_t* sizes, hipStream_t s);
// Sizes + exclusive scan (node < 0: the rows' sizes): out[0..m], out[m] the total.
// flags: tc_scan_flag_words(m) words of workspace (the tile sums).
int64_t tc_scan_flag_words(int64_t m);
hipError_t launch_tc_size_scan(const GenLaunch& L, const TcTables* T, int node, int64_t m, bool root_coll,
                               int64_t* out, uint64_t* flags, hipStream_t s);
// Writes: the rows (frame headers, fixed parts, top-level positions), then each var node's
// instances (node, m = its instance count), parents before children.
hipError_t launch_tc_write_rows(const GenLaunch& L, const TcTables* T, int nroot, const int64_t* offs, uint8_t* out,
                                int64_t capacity, int32_t* status, hipStream_t s);
// kind / nchild: the node's; key_kind / val_kind: a list's item kind (a map's key and
// value kinds), for the container kernel's instantiation
hipError_t launch_tc_write_node(const GenLaunch& L, const TcTables* T, int node, int64_t m, uint8_t* out,
                                int64_t capacity, int32_t* status, hipStream_t s, int kind, int nchild, int key_kind,
                                int val_kind);

// Columnar decode (treedec.hip): per-node passes over instances, field-major for rows and
// beans, item-parallel for lists / maps. Positions of the bean / list / map instances:
// P (start, -1 = absent / null), SZ (slot size), TL (record end - start).
struct TdTables {
  int64_t* P[kTcMaxNodes];
  int32_t* SZ[kTcMaxNodes];
  int32_t* TL[kTcMaxNodes];
  int64_t* SRC[kTcMaxNodes];  // string / binary nodes: each value's bytes in the rows (-1: null)
  int64_t m[kTcMaxNodes];     // instances of each node in this call (the output columns' lengths)
  int32_t kids[kTcMaxNodes];  // fields by parent: the rows' top-level fields, then each bean's
  int32_t kid0[kTcMaxNodes];
  int32_t nroot;
};
// The rows' fields (or collection frames), then one bean / list / map node (m instances);
// L.fill_level >= 0: that level's counts, -1: the values.
hipError_t launch_td_rows(const GenLaunch& L, const TdTables* T, int nroot, const uint8_t* rows, const int64_t* offs,
                          int32_t* status, hipStream_t s);
// The string / binary bytes of node `node` (m values) from the positions its level's
// pass recorded (TdTables.SRC) to the Arrow values at its scanned offsets.
hipError_t launch_td_strings(uint8_t* out_values, int32_t* out_offsets, const int64_t* src, int64_t m,
                             const uint8_t* rows, hipStream_t s);
hipError_t launch_td_node(const GenLaunch& L, const TdTables* T, int node, int64_t m, int kind, int nchild,
                          int item_flags, const uint8_t* rows, int32_t* status, hipStream_t s);

// Frame index of a STREAM batch (frames.hip): the starts of the first num_rows
// frames of rows_bytes bytes, found on the device from the stream alone.
struct FrameIndexLaunch {
  int64_t rows_bytes;
  int64_t num_rows;
  int64_t schema_hash;
  int32_t fixed_size;
  int32_t idx_frames;  // frames per chunk (0 = 20; LaunchKnobs::idx_frames)
  int64_t chunk;   // bytes per chunk (frame_index_plan)
  int64_t chunks;
};
void frame_index_plan(int64_t num_rows, int64_t rows_bytes, int32_t idx_frames, int64_t* chunk, int64_t* chunks);
int64_t frame_index_words(int64_t num_rows, int64_t rows_bytes, int32_t idx_frames);  // int64 workspace words
hipError_t launch_frame_index(const FrameIndexLaunch& L, const uint8_t* rows, int64_t* d_row_offsets, int64_t* ws,
                              int32_t* status, hipStream_t s);

}  // namespace fory_amd
