// plan.h — host-side layout planner for the MI355X row-format path.
//
// Restates, once per schema, what the reference computes once per bean class
// in Encoders.bean (java/fory-format/.../encoder/Encoders.java:75-78,155):
//   - field order/nullability come from the caller (TypeInference order,
//     TypeInference.java:141-254; Descriptor.java:415-423)
//   - DataTypes.getTypeWidth            (DataTypes.java:68-133,225-227)
//   - BinaryRowWriter fixed size        (BinaryRowWriter.java:46-52)
//   - BitUtils.calculateBitmapWidthInBytes (BitUtils.java:175-177)
//   - DataTypes.computeSchemaHash       (DataTypes.java:499-544)
// and compiles the per-record write/read sequence the JIT codec would
// generate (RowEncoderBuilder.java:177-270, BaseBinaryEncoderBuilder.java:149-490)
// into a small op program executed by one GPU lane per record.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/fory_rowfmt.h"

namespace fory_amd {

// Field kinds the device path distinguishes.
enum FieldKind : int32_t {
  KIND_FIXED = 0,   // 1/2/4/8-byte value stored zero-extended in an 8-byte slot
  KIND_BOOL = 1,    // 1 byte 0/1 (MemoryBuffer.putBoolean)
  KIND_BYTES = 2,   // utf8 / binary: (offset<<32|size) slot + padded bytes
  KIND_STRUCT = 3,  // nested row inline in the variable section
  KIND_LIST = 4,    // BinaryArray inline in the variable section
  KIND_MAP = 5,     // BinaryMap inline: [i64 keyArrayBytes][key BinaryArray][value BinaryArray]
  KIND_DECIMAL = 6, // decimal128 column -> 32 sign-extended bytes behind an (offset, 32) slot (tree engine);
                    // prec 0: a BigInteger field -> toByteArray()'s 1..16 big-endian bytes, (offset, len)
};

// Per top-level field of a fixed-width plan (read by the tiled kernels).
struct FixedFieldDev {
  const uint8_t* values;    // column values (bound per call)
  const uint8_t* validity;  // Arrow validity (nullable fields only), may be null
  uint8_t* out_values;      // decode target
  uint8_t* out_validity;    // decode target
  int32_t width;            // 1,2,4,8
  int32_t flags;            // bit0 nullable, bit1 bool
  int32_t slot;             // schema ordinal (slot index in the row / enclosing struct)
  int32_t parent;           // varlen tile kernels: enclosing struct id (0 = the row itself)
};
// The device table is sorted into width groups [8-byte][4-byte][2-byte][1-byte]
// (stable within a group) so every load loop has a compile-time width.

// Op program for varlen plans: executed per record by one lane.
enum OpCode : int32_t {
  OP_FIXED = 0,        // a=ordinal b=col c=width d=flags(bit0 nullable, bit1 bool)
  OP_BYTES = 1,        // a=ordinal b=col d=flags
  OP_STRUCT_BEGIN = 2, // a=ordinal b=col c=nfields d=flags e=index of matching END
  OP_STRUCT_END = 3,
  OP_LIST = 4,         // a=ordinal b=col c=item col d=flags e=item width | item flags<<8
  OP_MAP = 5,          // a=ordinal b=col c=key col (value col = c+1) d=flags
                       // e=key width | value width<<8 | key flags<<16 | value flags<<24
                       // item flags: bit0 nullable, bit1 bool, bit2 string/binary (width 8)
  OP_LIST_STRUCT = 6,  // list<struct of fixed fields>: a=ordinal b=list col c=struct col
                       // d=list flags | struct nullable<<2, e=pc after the element fields;
                       // followed by one OP_FIXED per struct field (a=child ordinal)
};

struct Op {
  int32_t code, a, b, c, d, e;
};

// Flat plans: one top-level STRING/BINARY or LIST<fixed> field (bound per call;
// read with scalar loads by the flat tile kernels).
struct VarFieldDev {
  const int32_t* offsets;        // Arrow offsets: bytes (STRING/BINARY) or items (LIST)
  const uint8_t* values;         // string bytes / item values
  const uint8_t* validity;       // field validity (nullable) or null
  const uint8_t* item_validity;  // LIST item validity (nullable items) or null
  int32_t* out_offsets;          // decode targets (same buffers, output side)
  uint8_t* out_values;
  uint8_t* out_validity;
  uint8_t* out_item_validity;
  int32_t slot;                  // schema ordinal
  int32_t is_list;
  int32_t w;                     // item width (1 for bytes)
  int32_t iflags;                // item flags: bit0 nullable, bit1 bool
  int32_t flags;                 // field flags: bit0 nullable
  int32_t parent;                // enclosing struct id (0 = the row itself)
  int32_t pad[2];
};

// Nested struct fields of a tile-engine plan, in pre-order (id = index + 1; id
// 0 is the top-level row). A struct's child row is written inline at the
// writerIndex its field is reached (BaseBinaryEncoderBuilder.java:436-490).
struct StructDev {
  const uint8_t* validity;       // struct column validity (nullable) or null
  uint8_t* out_validity;         // decode target
  int32_t parent;                // enclosing struct id
  int32_t slot;                  // ordinal in the parent
  int32_t hdr;                   // child null-bitmap bytes
  int32_t nfields;               // child field count
  int32_t flags;                 // bit0 nullable
  int32_t pad;
};
constexpr int kMaxTileStructs = 16;  // struct fields a tile-engine plan may hold

struct ColumnDev {  // per-column device view (bound per call)
  const uint8_t* values;
  const int32_t* offsets;
  const uint8_t* validity;
  uint8_t* out_values;
  int32_t* out_offsets;
  uint8_t* out_validity;
};

// Schema tree node of the tree engine (generic.hip), one per pre-order
// descriptor: a node's children follow it, its subtree ends at `end`.
// GNode.flags: a struct whose fields are all leaves (fixed, bool, string / binary,
// decimal): the columnar engine writes / reads it inside its container's items pass.
constexpr int32_t kGNodeFlatBean = 2;
struct GNode {
  int32_t kind;    // FieldKind
  int32_t width;   // 1/2/4/8 for fixed width, else -1
  int32_t flags;   // bit0 nullable; kGNodeFlatBean
  int32_t end;     // index after the subtree
  int32_t nchild;
  int32_t cdepth;  // list / map ancestors: the decode lengths pass that sizes this column
  int32_t prec;    // KIND_DECIMAL: precision (|unscaled| <= 10^prec - 1); 0: BigInteger bytes; else 0
};

struct Node {
  int32_t type_id = 0;
  int32_t nullable = 0;
  int32_t width = -1;
  int32_t kind = 0;
  int32_t prec = 0;               // KIND_DECIMAL: precision (descriptor's reserved word, 0 = 38);
                                  // 0 for FORY_DECIMAL_BIGINTEGER (java.math.BigInteger)
  std::vector<int32_t> children;  // desc indices
};

// Test / A-B knobs of the launchers, read from the environment ONCE, when a plan is
// created (fory_rowfmt_plan_create), and carried by value in the launch structs: no
// getenv on a launch path (a setenv on another thread cannot race a launch). They
// force the fallback engines and LDS budgets so the parity suite reaches every path;
// none selects a rejected variant. 0 = unset.
//   FORY_ROWFMT_VARTILE=0   per-record global interpreter for every tile
//   FORY_ROWFMT_VARFLAT=0   generic tile interpreter for cooperative plans too
//   FORY_ROWFMT_VARCAP / SPILLCAP / VARFIT   LDS image budgets, VARSTG staging slot bytes
//   FORY_ROWFMT_VARNW=2|4   waves per cooperative tile
//   FORY_ROWFMT_SIZES_PROGRAM  sizes by the op-program walk for flat plans too
//   FORY_ROWFMT_IDXFRAMES   frames per frame-index chunk
//   FORY_ROWFMT_VARPROF=1   phase timeline (debug), FORY_ROWFMT_VARDIAG=1 LDS sizing to stderr
//   FORY_ROWFMT_VARENC=1|7|9  encode with the round-3 tile kernel / v7 / v9 (each byte-identical)
// No knob changes the bytes or skips work (tests/test_kernel_isa.py checks the product reads
// no debug knob that could).
struct LaunchKnobs {
  int32_t no_tiles;
  int32_t no_flat;
  int32_t var_cap;
  int32_t var_fit;
  int32_t var_stg;
  int32_t spill_cap;
  int32_t var_nw;
  int32_t sizes_program;
  int32_t idx_frames;
  int32_t prof;
  int32_t diag;
  int32_t var_enc;   // FORY_ROWFMT_VARENC (A/B): 0 = defaults of launch_flat_enc, 1 / 7 / 9 force a kernel
  int32_t var_xcd;   // FORY_ROWFMT_VARXCD=C: varlen tile kernels take tiles in XCD runs of C (-1: one run per XCD), 0 = dispatch order
  int32_t dec_regs;  // FORY_ROWFMT_DECREGS=1: varlen decode stages its tile rows through registers, not LDS-DMA (A/B)
  int32_t tree_col;  // FORY_ROWFMT_TREECOL: 0 = tree-engine encode per lane only; else the columnar engine when the workspace allows
};
LaunchKnobs knobs_from_env();

struct Plan {
  std::vector<fory_field_desc> desc;
  std::vector<Node> nodes;
  std::vector<int32_t> top;       // desc indices of top-level fields
  int64_t schema_hash = 17;
  int32_t bitmap_bytes = 0;
  int32_t fixed_size = 0;
  bool fixed_width = true;
  bool any_nullable = false;
  std::vector<Op> program;        // varlen plans
  int32_t max_depth = 0;
  // Nestings the op programs do not cover (list<list<...>>, List<Bean> with var
  // fields, maps of structs / lists) run on the tree engine over `gnodes`.
  bool generic = false;
  std::vector<GNode> gnodes;
  int32_t max_cdepth = 0;
  LaunchKnobs kn{};  // read from the environment once, at plan creation
};

// Returns FORY_OK or an error code, with a message in `err`.
int build_plan(const fory_field_desc* fields, int32_t num_desc, Plan* out, std::string* err);

int32_t type_width(int32_t type_id);

}  // namespace fory_amd
