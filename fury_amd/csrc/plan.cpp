// plan.cpp — schema → layout plan (see plan.h for the reference mapping).
#include "plan.h"

#include <cstdio>

namespace fory_amd {

int32_t type_width(int32_t t) {
  // DataTypes.getTypeWidth (DataTypes.java:68-133): bool 1, intN N/8,
  // float 4, double 8, date 4, timestamp 8; struct/list/map/utf8/binary/decimal -1.
  switch (t) {
    case FORY_TYPE_BOOL:
    case FORY_TYPE_INT8:
      return 1;
    case FORY_TYPE_INT16:
      return 2;
    case FORY_TYPE_INT32:
    case FORY_TYPE_FLOAT:
    case FORY_TYPE_DATE32:
      return 4;
    case FORY_TYPE_INT64:
    case FORY_TYPE_DOUBLE:
    case FORY_TYPE_TIMESTAMP:
      return 8;
    default:
      return -1;
  }
}

static bool supported_type(int32_t t) {
  switch (t) {
    case FORY_TYPE_BOOL: case FORY_TYPE_INT8: case FORY_TYPE_INT16: case FORY_TYPE_INT32:
    case FORY_TYPE_INT64: case FORY_TYPE_FLOAT: case FORY_TYPE_DOUBLE: case FORY_TYPE_STRING:
    case FORY_TYPE_BINARY: case FORY_TYPE_DATE32: case FORY_TYPE_TIMESTAMP: case FORY_TYPE_LIST:
    case FORY_TYPE_STRUCT: case FORY_TYPE_MAP: case FORY_TYPE_DECIMAL:
      return true;
    default:
      return false;
  }
}

static int parse_node(const fory_field_desc* d, int32_t n, int32_t at, Plan* p, int depth,
                      int32_t* next, std::string* err) {
  if (at >= n) {
    *err = "schema descriptor truncated";
    return FORY_ERR_ENCODER;
  }
  if (depth > 16) {
    *err = "schema nesting deeper than 16";
    return FORY_ERR_UNSUPPORTED;
  }
  const fory_field_desc& f = d[at];
  const bool dec = f.type_id == FORY_TYPE_DECIMAL;  // reserved = precision (0 = 38) | FORY_DECIMAL_BIGINTEGER
  const int32_t dprec = f.reserved & 0xff;
  const bool bigint = dec && (f.reserved & FORY_DECIMAL_BIGINTEGER);
  const bool dec_ok = (f.reserved & ~(int32_t)(0xff | FORY_DECIMAL_BIGINTEGER)) == 0 && dprec <= 38 &&
                      (!bigint || dprec == 0 || dprec == 38);
  if ((!dec && f.reserved != 0) || (dec && !dec_ok) || f.num_children < 0) {
    *err = "invalid field descriptor at index " + std::to_string(at);
    return FORY_ERR_INVALID_ARGUMENT;
  }
  if (!supported_type(f.type_id)) {
    // DataTypes.unsupported(type) -> UnsupportedOperationException
    *err = "Unsupported type id " + std::to_string(f.type_id) + " at field descriptor " +
           std::to_string(at);
    return FORY_ERR_UNSUPPORTED;
  }
  Node& nd = p->nodes[at];
  nd.type_id = f.type_id;
  nd.nullable = f.nullable ? 1 : 0;
  nd.width = type_width(f.type_id);
  if (nd.nullable) p->any_nullable = true;
  if (f.type_id == FORY_TYPE_LIST && f.num_children != 1) {
    *err = "list field must have exactly one child (DataTypes.arrayField)";
    return FORY_ERR_ENCODER;
  }
  if (f.type_id == FORY_TYPE_MAP && f.num_children != 2) {
    *err = "map field must have exactly two children: key and value (DataTypes.mapField)";
    return FORY_ERR_ENCODER;
  }
  if (f.type_id != FORY_TYPE_LIST && f.type_id != FORY_TYPE_STRUCT && f.type_id != FORY_TYPE_MAP &&
      f.num_children != 0) {
    // DataTypes.java:533-538 "field type should not be nested"
    *err = "field type should not be nested, but got type id " + std::to_string(f.type_id);
    return FORY_ERR_ENCODER;
  }
  switch (f.type_id) {
    case FORY_TYPE_BOOL: nd.kind = KIND_BOOL; break;
    case FORY_TYPE_STRING: case FORY_TYPE_BINARY: nd.kind = KIND_BYTES; break;
    case FORY_TYPE_STRUCT: nd.kind = KIND_STRUCT; break;
    case FORY_TYPE_LIST: nd.kind = KIND_LIST; break;
    case FORY_TYPE_MAP: nd.kind = KIND_MAP; break;
    case FORY_TYPE_DECIMAL:  // TypeInference: BigDecimal -> Decimal(38, 18), BigInteger -> Decimal(38, 0)
      nd.kind = KIND_DECIMAL;
      nd.prec = bigint ? 0 : (dprec > 0 ? dprec : 38);  // 0: BigInteger.toByteArray() bytes
      break;
    default: nd.kind = KIND_FIXED; break;
  }
  int32_t cur = at + 1;
  for (int32_t c = 0; c < f.num_children; ++c) {
    nd.children.push_back(cur);
    int32_t nx = 0;
    int rc = parse_node(d, n, cur, p, depth + 1, &nx, err);
    if (rc) return rc;
    cur = nx;
  }
  if (depth + 1 > p->max_depth) p->max_depth = depth + 1;
  *next = cur;
  return FORY_OK;
}

// DataTypes.computeHash (DataTypes.java:507-544).
static int64_t hash_node(int64_t h, const Plan& p, int32_t idx) {
  const Node& nd = p.nodes[idx];
  for (;;) {
    int64_t m, s;
    if (!__builtin_mul_overflow(h, (int64_t)31, &m) &&
        !__builtin_add_overflow(m, (int64_t)nd.type_id, &s)) {
      h = s;
      break;
    }
    h >>= 2;  // catch (ArithmeticException e) { hash = hash >> 2; }
  }
  for (int32_t c : nd.children) h = hash_node(h, p, c);
  return h;
}

static int32_t bitmap_bytes(int64_t n) { return (int32_t)(((n + 63) / 64) * 8); }

// Array element flags (OP_LIST / OP_MAP parts): bit0 nullable, bit1 bool, bit2
// string/binary (8-byte (offset, size) slot + padded bytes after the fixed part).
static int32_t elem_flags(const Node& it) {
  return (it.nullable ? 1 : 0) | (it.kind == KIND_BOOL ? 2 : 0) | (it.kind == KIND_BYTES ? 4 : 0);
}
static int32_t elem_width(const Node& it) { return it.kind == KIND_BYTES ? 8 : it.width; }

static int compile_field(const Plan& p, int32_t idx, int32_t ordinal, std::vector<Op>* prog,
                         std::string* err) {
  const Node& nd = p.nodes[idx];
  int32_t flags = (nd.nullable ? 1 : 0) | (nd.kind == KIND_BOOL ? 2 : 0);
  switch (nd.kind) {
    case KIND_FIXED:
    case KIND_BOOL:
      prog->push_back({OP_FIXED, ordinal, idx, nd.width, flags, 0});
      return FORY_OK;
    case KIND_BYTES:
      prog->push_back({OP_BYTES, ordinal, idx, 0, flags, 0});
      return FORY_OK;
    case KIND_STRUCT: {
      size_t begin = prog->size();
      prog->push_back({OP_STRUCT_BEGIN, ordinal, idx, (int32_t)nd.children.size(), flags, 0});
      for (size_t k = 0; k < nd.children.size(); ++k) {
        int rc = compile_field(p, nd.children[k], (int32_t)k, prog, err);
        if (rc) return rc;
      }
      (*prog)[begin].e = (int32_t)prog->size();
      prog->push_back({OP_STRUCT_END, ordinal, idx, 0, flags, 0});
      return FORY_OK;
    }
    case KIND_LIST: {
      int32_t item = nd.children[0];
      const Node& it = p.nodes[item];
      if (it.kind == KIND_STRUCT) {
        // List<Bean> (serializeForArrayByWriter, BaseBinaryEncoderBuilder.java:293-351, with
        // serializeForBean per element :436-490): element slots hold (offset, size) of
        // child rows appended after the array's fixed part. Device path: bean fields
        // of fixed width only.
        for (int32_t ch : it.children) {
          const Node& cn = p.nodes[ch];
          if (cn.kind != KIND_FIXED && cn.kind != KIND_BOOL) {
            *err = "device path supports list<struct of fixed-width fields> only (got field type id " +
                   std::to_string(cn.type_id) + ")";
            return FORY_ERR_UNSUPPORTED;
          }
        }
        const size_t begin = prog->size();
        prog->push_back({OP_LIST_STRUCT, ordinal, idx, item, flags | (it.nullable ? 4 : 0), 0});
        for (size_t k = 0; k < it.children.size(); ++k) {
          const Node& cn = p.nodes[it.children[k]];
          const int32_t cf = (cn.nullable ? 1 : 0) | (cn.kind == KIND_BOOL ? 2 : 0);
          prog->push_back({OP_FIXED, (int32_t)k, it.children[k], cn.width, cf, 0});
        }
        (*prog)[begin].e = (int32_t)prog->size();
        return FORY_OK;
      }
      if (it.kind != KIND_FIXED && it.kind != KIND_BOOL && it.kind != KIND_BYTES) {
        *err = "device path supports list<fixed-width | string | binary | struct> only (got element type id " +
               std::to_string(it.type_id) + ")";
        return FORY_ERR_UNSUPPORTED;
      }
      // string/binary elements: 8-byte (offset, size) element slots, the bytes appended
      // after the array's fixed part (BinaryArrayWriter elemSize 8, :75-85; write(int,
      // String) through writeUnaligned, BinaryWriter.java:162-194)
      const int32_t iflags = elem_flags(it);
      prog->push_back({OP_LIST, ordinal, idx, item, flags, elem_width(it) | (iflags << 8)});
      return FORY_OK;
    }
    case KIND_DECIMAL:  // writeDecimal (BinaryWriter.java:214-230): the tree engine's
      *err = "decimal fields run on the tree engine";
      return FORY_ERR_UNSUPPORTED;
    case KIND_MAP: {  // serializeForMap (BaseBinaryEncoderBuilder.java:370-427)
      const int32_t key = nd.children[0], val = nd.children[1];
      const Node& k = p.nodes[key];
      const Node& v = p.nodes[val];
      if (k.nullable) {
        *err = "Map's keys must be non-nullable";  // DataTypes.mapField (DataTypes.java:419)
        return FORY_ERR_ENCODER;
      }
      auto scalar = [](const Node& x) { return x.kind == KIND_FIXED || x.kind == KIND_BOOL || x.kind == KIND_BYTES; };
      if (!scalar(k) || !scalar(v)) {
        *err = "device path supports map keys/values of fixed width, string or binary only (got key type id " +
               std::to_string(k.type_id) + ", value type id " + std::to_string(v.type_id) + ")";
        return FORY_ERR_UNSUPPORTED;
      }
      const int32_t kf = elem_flags(k), vf = elem_flags(v);
      prog->push_back({OP_MAP, ordinal, idx, key, flags,
                       elem_width(k) | (elem_width(v) << 8) | (kf << 16) | (vf << 24)});
      return FORY_OK;
    }
  }
  *err = "unknown field kind";
  return FORY_ERR_ENCODER;
}

// Pre-order node table of the tree engine: subtree ends and container depths.
static int32_t fill_gnode(Plan* p, int32_t idx, int32_t cdepth) {
  const Node& nd = p->nodes[idx];
  GNode& g = p->gnodes[idx];
  g.kind = nd.kind;
  g.width = nd.width;
  g.flags = nd.nullable ? 1 : 0;
  if (nd.kind == KIND_STRUCT && !nd.children.empty()) {  // a bean of leaf fields only
    bool flat = true;
    for (int32_t ch : nd.children) {
      const int32_t k = p->nodes[ch].kind;
      flat = flat && (k == KIND_FIXED || k == KIND_BOOL || k == KIND_BYTES || k == KIND_DECIMAL);
    }
    if (flat) g.flags |= kGNodeFlatBean;
  }
  g.nchild = (int32_t)nd.children.size();
  g.cdepth = cdepth;
  g.prec = nd.prec;
  if (cdepth > p->max_cdepth) p->max_cdepth = cdepth;
  const int32_t inner = cdepth + (nd.kind == KIND_LIST || nd.kind == KIND_MAP ? 1 : 0);
  int32_t end = idx + 1;
  for (int32_t ch : nd.children) end = fill_gnode(p, ch, inner);
  p->gnodes[idx].end = end;
  return end;
}

static void build_gnodes(Plan* p) {
  p->gnodes.assign(p->nodes.size(), GNode{});
  p->max_cdepth = 0;
  for (int32_t t : p->top) fill_gnode(p, t, 0);
}

int build_plan(const fory_field_desc* fields, int32_t num_desc, Plan* p, std::string* err) {
  if (num_desc < 0 || (num_desc > 0 && fields == nullptr)) {
    *err = "fields is null or num_desc < 0";
    return FORY_ERR_INVALID_ARGUMENT;
  }
  p->desc.assign(fields, fields + num_desc);
  p->nodes.assign(num_desc, Node());
  p->top.clear();
  int32_t at = 0;
  while (at < num_desc) {
    p->top.push_back(at);
    int32_t nx = 0;
    int rc = parse_node(fields, num_desc, at, p, 0, &nx, err);
    if (rc) return rc;
    at = nx;
  }
  int64_t h = 17;  // DataTypes.computeSchemaHash (DataTypes.java:499-505)
  for (int32_t t : p->top) h = hash_node(h, *p, t);
  p->schema_hash = h;
  p->bitmap_bytes = bitmap_bytes((int64_t)p->top.size());
  p->fixed_size = p->bitmap_bytes + 8 * (int32_t)p->top.size();
  p->fixed_width = true;
  for (int32_t t : p->top) {
    int k = p->nodes[t].kind;
    if (k != KIND_FIXED && k != KIND_BOOL) p->fixed_width = false;
  }
  p->program.clear();
  build_gnodes(p);
  p->generic = false;
  if (!p->fixed_width) {
    for (size_t k = 0; k < p->top.size(); ++k) {
      int rc = compile_field(*p, p->top[k], (int32_t)k, &p->program, err);
      if (rc == FORY_ERR_UNSUPPORTED) {  // a nesting the op programs do not cover: tree engine
        p->generic = true;
        p->program.clear();
        err->clear();
        break;
      }
      if (rc) return rc;
    }
  }
  if (p->generic) {  // the checks compile_field made on the way (map keys) for every map
    for (const Node& nd : p->nodes)
      if (nd.kind == KIND_MAP && p->nodes[nd.children[0]].nullable) {
        *err = "Map's keys must be non-nullable";  // DataTypes.mapField (DataTypes.java:419)
        return FORY_ERR_ENCODER;
      }
  }
  return FORY_OK;
}

}  // namespace fory_amd
