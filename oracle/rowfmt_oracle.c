/*
 * rowfmt_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * A scalar CPU restatement of Apache Fory's Java row-format writer/reader
 * (java/fory-format), used as the parity checker for the HIP path. Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library; the product (fury_amd/, libfory_rowfmt.so) never links it.
 *
 * Every routine restates one reference routine and cites it (paths relative
 * to the reference tree; F = java/fory-format/src/main/java/org/apache/fory/
 * format, C = java/fory-core/src/main/java/org/apache/fory):
 *   - schema hash          F/type/DataTypes.java:499-544
 *   - row writer           F/row/binary/writer/BinaryRowWriter.java:46-136
 *   - writer base          F/row/binary/writer/BinaryWriter.java:40-194
 *   - array writer         F/row/binary/writer/BinaryArrayWriter.java:93-206
 *   - map layout           F/row/binary/BinaryMap.java:30-77 (writer:
 *                          F/encoder/BaseBinaryEncoderBuilder.java:370-427)
 *   - per-type dispatch    F/encoder/BaseBinaryEncoderBuilder.java:149-490
 *                          (BigInteger: :192-194 write, :559-560 read)
 *   - framing              F/encoder/Encoders.java:177-225
 *   - readers              F/row/binary/BinaryRow.java:110-123,
 *                          F/row/binary/UnsafeTrait.java:68-197,
 *                          F/row/binary/BinaryArray.java:69-130
 *   - bitmap               C/memory/BitUtils.java:36-90,175-177
 *
 * Parity pinning: the Java reference cannot run in
 * this container (no JDK) and the reference's C++ row writer is unbuildable
 * under this project's rules (needs absl). The schema hash is pinned by
 * golden values produced by the reference's own Python implementation
 * (python/pyfory/format/infer.py:160-190); row bytes are pinned by the
 * sha256 of the reference C++ writer's output recorded in SURVEY.md §8c and
 * by the reference's round-trip tests restated in tests/. Byte layouts not
 * covered by either are "parity unpinned" and say so where tested.
 *
 * Memory model: the output buffer is zeroed first, which is what Java sees on
 * a fresh MemoryBuffer (MemoryUtils.java:30-32); null slots are therefore 0.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/fory_rowfmt.h"

/* ---------------------------------------------------------------------- */
/* schema tree                                                             */
/* ---------------------------------------------------------------------- */

typedef struct onode {
  int type_id;
  int nullable;
  int width;      /* DataTypes.getTypeWidth (DataTypes.java:68-133), -1 = varlen */
  int precision;  /* DECIMAL: from the descriptor's reserved word (0 = 38) */
  int biginteger; /* DECIMAL with FORY_DECIMAL_BIGINTEGER: a java.math.BigInteger field */
  int nchild;
  int child[64];  /* desc indices of children (struct fields / list item) */
} onode;

typedef struct otree {
  int n;          /* number of descs */
  onode* nodes;
  int ntop;
  int top[4096];
} otree;

static int type_width(int t) {
  switch (t) {
    case FORY_TYPE_BOOL: case FORY_TYPE_INT8: return 1;
    case FORY_TYPE_INT16: return 2;
    case FORY_TYPE_INT32: case FORY_TYPE_FLOAT: case FORY_TYPE_DATE32: return 4;
    case FORY_TYPE_INT64: case FORY_TYPE_DOUBLE: case FORY_TYPE_TIMESTAMP: return 8;
    default: return -1;
  }
}

static int parse(const fory_field_desc* d, int n, int at, otree* t) {
  if (at >= n) return -1;
  onode* nd = &t->nodes[at];
  nd->type_id = d[at].type_id;
  nd->nullable = d[at].nullable;
  nd->width = type_width(d[at].type_id);
  nd->biginteger = d[at].type_id == FORY_TYPE_DECIMAL && (d[at].reserved & FORY_DECIMAL_BIGINTEGER);
  nd->precision = d[at].type_id == FORY_TYPE_DECIMAL ? ((d[at].reserved & 0xff) > 0 ? (d[at].reserved & 0xff) : 38) : 0;
  if (nd->precision > 38) return -1;
  nd->nchild = 0;
  int next = at + 1;
  int want = d[at].num_children;
  if (want > 64) return -1;
  for (int c = 0; c < want; c++) {
    nd->child[nd->nchild++] = next;
    next = parse(d, n, next, t);
    if (next < 0) return -1;
  }
  return next;
}

static int build_tree(const fory_field_desc* d, int n, otree* t) {
  t->n = n;
  t->nodes = (onode*)calloc((size_t)(n > 0 ? n : 1), sizeof(onode));
  t->ntop = 0;
  int at = 0;
  while (at < n) {
    if (t->ntop >= 4096) return -1;
    t->top[t->ntop++] = at;
    at = parse(d, n, at, t);
    if (at < 0) return -1;
  }
  return 0;
}

static void free_tree(otree* t) { free(t->nodes); }

/* ---------------------------------------------------------------------- */
/* schema hash: DataTypes.computeSchemaHash (DataTypes.java:499-544)       */
/* h = Math.addExact(Math.multiplyExact(h, 31), id); on ArithmeticException */
/* h >>= 2 (arithmetic) and retry. Then recurse into list item / struct     */
/* children.                                                                */
/* ---------------------------------------------------------------------- */

static int64_t hash_node(int64_t h, const otree* t, int idx) {
  const onode* nd = &t->nodes[idx];
  for (;;) {
    int64_t m, s;
    if (!__builtin_mul_overflow(h, (int64_t)31, &m) &&
        !__builtin_add_overflow(m, (int64_t)nd->type_id, &s)) {
      h = s;
      break;
    }
    h = h >> 2;
  }
  for (int c = 0; c < nd->nchild; c++) h = hash_node(h, t, nd->child[c]);
  return h;
}

int64_t oracle_schema_hash(const fory_field_desc* d, int n) {
  otree t;
  if (build_tree(d, n, &t) != 0) { free_tree(&t); return 0; }
  int64_t h = 17;
  for (int i = 0; i < t.ntop; i++) h = hash_node(h, &t, t.top[i]);
  free_tree(&t);
  return h;
}

/* ---------------------------------------------------------------------- */
/* MemoryBuffer little-endian puts (MemoryBuffer.java:408-570)             */
/* ---------------------------------------------------------------------- */

typedef struct obuf {
  uint8_t* p;
  int64_t cap;
  int64_t wi;      /* writerIndex */
  int overflow;
  int unsupported; /* a decimal beyond its precision (sticky: sizing passes overflow too) */
} obuf;

static void grow(obuf* b, int64_t need) {
  if (b->wi + need > b->cap) b->overflow = 1;
}
static void put8(obuf* b, int64_t at, uint8_t v) { if (at >= 0 && at + 1 <= b->cap) b->p[at] = v; else b->overflow = 1; }
static void put16(obuf* b, int64_t at, uint16_t v) { if (at >= 0 && at + 2 <= b->cap) memcpy(b->p + at, &v, 2); else b->overflow = 1; }
static void put32(obuf* b, int64_t at, uint32_t v) { if (at >= 0 && at + 4 <= b->cap) memcpy(b->p + at, &v, 4); else b->overflow = 1; }
static void put64(obuf* b, int64_t at, uint64_t v) { if (at >= 0 && at + 8 <= b->cap) memcpy(b->p + at, &v, 8); else b->overflow = 1; }
static void putbytes(obuf* b, int64_t at, const uint8_t* s, int64_t n) {
  if (n == 0) return;
  if (at >= 0 && at + n <= b->cap) memcpy(b->p + at, s, (size_t)n); else b->overflow = 1;
}

static int64_t round8(int64_t n) { /* BinaryWriter.roundNumberOfBytesToNearestWord :40-47 */
  int64_t r = n & 7;
  return r == 0 ? n : n + (8 - r);
}
static int bitmap_bytes(int64_t n) { return (int)(((n + 63) / 64) * 8); } /* BitUtils:175-177 */

/* ---------------------------------------------------------------------- */
/* writer state: BinaryWriter {startIndex, bytesBeforeBitMap} +            */
/* BinaryRowWriter{headerInBytes} / BinaryArrayWriter{elementSize,header}  */
/* ---------------------------------------------------------------------- */

typedef struct owriter {
  obuf* b;
  int64_t start;        /* startIndex */
  int before_bitmap;    /* 0 for rows, 8 for arrays (BinaryWriter ctor :59-63) */
  int64_t header;       /* bitmap bytes (row) or 8+bitmap (array) */
  int elem_size;        /* 8 for rows; element width (or 8 for varlen) for arrays */
  int is_array;
} owriter;

static int64_t w_offset(const owriter* w, int64_t ordinal) {
  /* BinaryRowWriter.getOffset :87-89 / BinaryArrayWriter.getOffset :126-128 */
  return w->start + w->header + ordinal * w->elem_size;
}

static void w_set_null(owriter* w, int64_t ordinal) {
  /* BinaryWriter.setNullAt :127-129 -> BitUtils.set :36-43 (1 = null) */
  int64_t at = w->start + w->before_bitmap + (ordinal >> 3);
  if (at < w->b->cap) w->b->p[at] |= (uint8_t)(1u << (ordinal & 7));
  else w->b->overflow = 1;
}

static void w_set_offset_and_size(owriter* w, int64_t ordinal, int64_t abs_off, int64_t size) {
  /* BinaryWriter.setOffsetAndSize :110-114 */
  int64_t rel = abs_off - w->start;
  uint64_t v = ((uint64_t)rel << 32) | (uint64_t)(uint32_t)size;
  put64(w->b, w_offset(w, ordinal), v);
}

static void row_reset(owriter* w, obuf* b, int nfields) {
  /* BinaryRowWriter(Schema) :46-52 and reset() :76-84 */
  w->b = b;
  w->before_bitmap = 0;
  w->header = bitmap_bytes(nfields);
  w->elem_size = 8;
  w->is_array = 0;
  w->start = b->wi;
  int64_t fixed = w->header + 8LL * nfields;
  grow(b, fixed);
  b->wi += fixed;
  for (int64_t i = w->start; i < w->start + w->header; i += 8) put64(b, i, 0);
}

static void array_reset(owriter* w, obuf* b, int64_t n, int elem_size) {
  /* BinaryArrayWriter.reset(numElements) :93-118 */
  w->b = b;
  w->before_bitmap = 8;
  w->elem_size = elem_size;
  w->is_array = 1;
  w->start = b->wi;
  w->header = 8 + bitmap_bytes(n);
  int64_t data = n * (int64_t)elem_size;
  int64_t fixed_part = round8(data);
  grow(b, w->header + fixed_part);
  put64(b, w->start, (uint64_t)n);
  for (int64_t i = w->start + 8; i < w->start + w->header; i += 8) put64(b, i, 0);
  for (int64_t i = data; i < fixed_part; i++) put8(b, w->start + w->header + i, 0);
  b->wi += w->header + fixed_part;
}

/* BinaryWriter.writeUnaligned(ordinal, byte[], off, n) :187-194 */
static void w_write_unaligned(owriter* w, int64_t ordinal, const uint8_t* src, int64_t n) {
  obuf* b = w->b;
  int64_t rounded = round8(n);
  grow(b, rounded);
  if ((n & 7) > 0) put64(b, b->wi + ((n >> 3) << 3), 0); /* zeroOutPaddingBytes :117-121 */
  putbytes(b, b->wi, src, n);
  w_set_offset_and_size(w, ordinal, b->wi, n);
  b->wi += rounded;
}

/* BinaryWriter.writeDecimal (BinaryWriter.java:214-230) of an Arrow decimal128 value
 * (16 bytes, little-endian two's complement of the unscaled value):
 * DecimalUtility.checkPrecisionAndScale (|unscaled| <= 10^precision - 1, else
 * UnsupportedOperationException; the scale is the column's), then
 * writeBigDecimalToArrowBuf(value, buf, 0, DECIMAL_BYTE_LENGTH = 32): the value's
 * little-endian bytes sign-extended to 32 (DecimalUtils.java:23), copied at the
 * writerIndex, slot = (offset, 32), writerIndex += 32 (already a multiple of 8).
 * Returns 0, or -3 when the precision check fails. */
static int w_write_decimal(owriter* w, int64_t ordinal, const uint8_t* v16, int precision) {
  __int128 v;
  memcpy(&v, v16, 16);
  unsigned __int128 mag = v < 0 ? (unsigned __int128)(-(v + 1)) + 1 : (unsigned __int128)v;
  unsigned __int128 lim = 1;
  for (int k = 0; k < precision; k++) lim *= 10;
  if (mag > lim - 1) return -3;
  uint8_t dec[32];
  memcpy(dec, v16, 16);
  memset(dec + 16, (v16[15] & 0x80) ? 0xFF : 0x00, 16);
  obuf* b = w->b;
  grow(b, 32);
  putbytes(b, b->wi, dec, 32);
  w_set_offset_and_size(w, ordinal, b->wi, 32);
  b->wi += 32;
  return 0;
}

/* A java.math.BigInteger field (BaseBinaryEncoderBuilder.java:192-194):
 * writer.write(ordinal, value.toByteArray()) -> BinaryWriter.write(int, byte[])
 * (BinaryWriter.java:167-170) -> writeUnaligned. toByteArray() is the minimal big-endian
 * two's complement: bitLength() / 8 + 1 bytes, bitLength() = the bits of v without its
 * sign bit (of ~v = -v - 1 when v < 0). The value here is an Arrow decimal128 (16 bytes,
 * little-endian two's complement, scale 0). */
static int bigint_to_bytes(const uint8_t* v16, uint8_t out[16]) {
  __int128 v;
  memcpy(&v, v16, 16);
  unsigned __int128 m = v < 0 ? (unsigned __int128)~v : (unsigned __int128)v;
  int bits = 0;
  while (m) { bits++; m >>= 1; }
  int len = bits / 8 + 1;
  for (int j = 0; j < len; j++) out[j] = v16[len - 1 - j];  /* big-endian: most significant first */
  return len;
}

static void w_write_biginteger(owriter* w, int64_t ordinal, const uint8_t* v16) {
  uint8_t be[16];
  int len = bigint_to_bytes(v16, be);
  w_write_unaligned(w, ordinal, be, len);
}

/* new BigInteger(byte[]) (BaseBinaryEncoderBuilder.java:559-560) of n row bytes into a
 * decimal128: big-endian two's complement, sign-extended. n == 0 is Java's
 * NumberFormatException ("Zero length BigInteger"); more than 16 bytes do not fit a
 * decimal128 (toByteArray never pads, so such a value exceeds 128 bits). Returns 0 or -1. */
static int bigint_from_bytes(const uint8_t* p, int64_t n, uint8_t out16[16]) {
  if (n < 1 || n > 16) return -1;
  memset(out16, (p[0] & 0x80) ? 0xFF : 0x00, 16);
  for (int64_t j = 0; j < n; j++) out16[j] = p[n - 1 - j];
  return 0;
}

/* ---------------------------------------------------------------------- */
/* column access                                                           */
/* ---------------------------------------------------------------------- */

static int col_valid(const fory_column* c, int64_t i) {
  if (!c->validity) return 1;
  return (c->validity[i >> 3] >> (i & 7)) & 1;
}

static uint64_t col_fixed(const fory_column* c, int width, int64_t i) {
  const uint8_t* p = (const uint8_t*)c->values + i * width;
  uint64_t v = 0;
  memcpy(&v, p, (size_t)width);
  return v;
}

/* ---------------------------------------------------------------------- */
/* encode one value at `ordinal` of writer w — the dispatch of             */
/* BaseBinaryEncoderBuilder.serializeFor (:149-285)                        */
/* ---------------------------------------------------------------------- */

static void write_value(owriter* w, int64_t ordinal, const otree* t, int idx,
                        const fory_column* cols, int64_t i);

static void write_struct_body(owriter* parent, int64_t ordinal, const otree* t, int idx,
                              const fory_column* cols, int64_t i) {
  /* serializeForBean :473-486: offset=writerIndex; child.reset(); toRow;
   * size = writerIndex - offset; parent.setOffsetAndSize(ordinal, offset, size) */
  const onode* nd = &t->nodes[idx];
  obuf* b = parent->b;
  int64_t off = b->wi;
  owriter child;
  row_reset(&child, b, nd->nchild);
  for (int c = 0; c < nd->nchild; c++) write_value(&child, c, t, nd->child[c], cols, i);
  w_set_offset_and_size(parent, ordinal, off, b->wi - off);
}

/* The BinaryArray of list idx's entry i at the writerIndex: serializeForArrayByWriter
 * :293-351 (reset(n), then serializeFor(j, elem, arrayWriter, ...) per element). */
static void write_list_payload(obuf* b, const otree* t, int idx, const fory_column* cols, int64_t i) {
  const onode* nd = &t->nodes[idx];
  const fory_column* c = &cols[idx];
  int item = nd->child[0];
  const onode* it = &t->nodes[item];
  int64_t b0 = c->offsets[i], b1 = c->offsets[i + 1];
  int64_t n = b1 - b0;
  owriter aw;
  array_reset(&aw, b, n, it->width < 0 ? 8 : it->width); /* BinaryArrayWriter ctor :75-85 */
  for (int64_t j = 0; j < n; j++) write_value(&aw, j, t, item, cols, b0 + j);
}

static void write_list_body(owriter* parent, int64_t ordinal, const otree* t, int idx,
                            const fory_column* cols, int64_t i) {
  /* BaseBinaryEncoderBuilder :240-249 (offset, serializeForArray, size, setOffsetAndSize) */
  obuf* b = parent->b;
  int64_t off = b->wi;
  write_list_payload(b, t, idx, cols, i);
  w_set_offset_and_size(parent, ordinal, off, b->wi - off);
}

static void write_map_payload(obuf* b, const otree* t, int idx, const fory_column* cols, int64_t i);

static void write_map_body(owriter* parent, int64_t ordinal, const otree* t, int idx,
                           const fory_column* cols, int64_t i) {
  obuf* b = parent->b;
  int64_t off = b->wi;
  write_map_payload(b, t, idx, cols, i);
  w_set_offset_and_size(parent, ordinal, off, b->wi - off);
}

static void write_map_payload(obuf* b, const otree* t, int idx, const fory_column* cols, int64_t i) {
  /* serializeForMap (BaseBinaryEncoderBuilder.java:370-427): offset = writerIndex;
   * writeDirectly(-1) reserves 8 bytes (BinaryWriter.java:232-236); the key set
   * and the values are written as two BinaryArrays (serializeForArray); the key
   * array's size is back-patched at offset (writeDirectly(offset, size) :239-241);
   * then setOffsetAndSize(ordinal, offset, writerIndex - offset). Entries are the
   * Arrow map's entries [offsets[i], offsets[i+1]) in order. */
  const onode* nd = &t->nodes[idx];
  const fory_column* c = &cols[idx];
  int64_t b0 = c->offsets[i], n = c->offsets[i + 1] - b0;
  int64_t off = b->wi;
  grow(b, 8);
  put64(b, off, (uint64_t)-1);
  b->wi += 8;
  int64_t key_bytes = 0;
  for (int part = 0; part < 2; part++) {
    int child = nd->child[part];
    const onode* it = &t->nodes[child];
    int64_t a0 = b->wi;
    owriter aw;
    array_reset(&aw, b, n, it->width < 0 ? 8 : it->width);
    for (int64_t j = 0; j < n; j++) write_value(&aw, j, t, child, cols, b0 + j);
    if (part == 0) key_bytes = b->wi - a0;
  }
  put64(b, off, (uint64_t)key_bytes);
}

static void write_value(owriter* w, int64_t ordinal, const otree* t, int idx,
                        const fory_column* cols, int64_t i) {
  const onode* nd = &t->nodes[idx];
  const fory_column* c = &cols[idx];
  if (nd->nullable && !col_valid(c, i)) { /* setValueOrNull: v == null -> setNullAt */
    w_set_null(w, ordinal);
    return;
  }
  obuf* b = w->b;
  int64_t at = w_offset(w, ordinal);
  switch (nd->type_id) {
    case FORY_TYPE_BOOL: {
      uint8_t v = ((const uint8_t*)c->values)[i] ? 1 : 0;
      if (!w->is_array) put64(b, at, 0);       /* BinaryRowWriter.write(int,boolean) :98-103 */
      put8(b, at, v);                          /* putBoolean writes 0/1 */
      return;
    }
    case FORY_TYPE_INT8:
      if (!w->is_array) put64(b, at, 0);       /* :91-96 */
      put8(b, at, (uint8_t)col_fixed(c, 1, i));
      return;
    case FORY_TYPE_INT16:
      if (!w->is_array) put64(b, at, 0);       /* :105-110 */
      put16(b, at, (uint16_t)col_fixed(c, 2, i));
      return;
    case FORY_TYPE_INT32: case FORY_TYPE_FLOAT: case FORY_TYPE_DATE32:
      if (!w->is_array) put64(b, at, 0);       /* :112-124: zero-extended, not sign-extended */
      put32(b, at, (uint32_t)col_fixed(c, 4, i));
      return;
    case FORY_TYPE_INT64: case FORY_TYPE_DOUBLE: case FORY_TYPE_TIMESTAMP:
      put64(b, at, col_fixed(c, 8, i));        /* BinaryWriter.write(int,long) :153-159 */
      return;
    case FORY_TYPE_STRING: case FORY_TYPE_BINARY: {
      int64_t s0 = c->offsets[i], s1 = c->offsets[i + 1];
      w_write_unaligned(w, ordinal, (const uint8_t*)c->values + s0, s1 - s0); /* :162-194 */
      return;
    }
    case FORY_TYPE_DECIMAL:
      if (nd->biginteger) {  /* BigInteger: toByteArray() bytes, no precision check */
        w_write_biginteger(w, ordinal, (const uint8_t*)c->values + 16 * i);
        return;
      }
      if (w_write_decimal(w, ordinal, (const uint8_t*)c->values + 16 * i, nd->precision)) b->unsupported = 1;
      return;
    case FORY_TYPE_STRUCT:
      write_struct_body(w, ordinal, t, idx, cols, i);
      return;
    case FORY_TYPE_LIST:
      write_list_body(w, ordinal, t, idx, cols, i);
      return;
    case FORY_TYPE_MAP:
      write_map_body(w, ordinal, t, idx, cols, i);
      return;
    default:
      b->overflow = 2;
      return;
  }
}

/* ---------------------------------------------------------------------- */
/* batch encode                                                            */
/* ---------------------------------------------------------------------- */

/* Encode N rows. frame_mode 0: rows back to back (BinaryRow.toBytes of each
 * toRow); 1: N calls of Encoder.encode(MemoryBuffer, T) (Encoders.java:213-225);
 * 2: N calls of ArrayEncoder / MapEncoder.encode(MemoryBuffer, T); 3: N calls of
 * Encoder.encode(T) -> byte[] = [i64 schemaHash][row] (Encoders.java:203-210),
 * concatenated.
 * out is zeroed first. row_offsets (N+1, nullable) receives row/frame starts.
 * Returns total bytes, -1 on capacity overflow, -2 on bad schema. */
int64_t oracle_encode(const fory_field_desc* d, int n_desc, const fory_column* cols,
                      int64_t nrows, int frame_mode, uint8_t* out, int64_t cap,
                      int64_t* row_offsets) {
  otree t;
  if (build_tree(d, n_desc, &t) != 0) { free_tree(&t); return -2; }
  int64_t hash = 17;
  for (int k = 0; k < t.ntop; k++) hash = hash_node(hash, &t, t.top[k]);
  if (out && cap > 0) memset(out, 0, (size_t)cap);
  obuf b = {out, out ? cap : 0, 0, 0, 0};
  for (int64_t i = 0; i < nrows; i++) {
    if (row_offsets) row_offsets[i] = b.wi;
    int64_t frame = b.wi;
    if (frame_mode == 2) {
      /* ArrayEncoder / MapEncoder.encode(MemoryBuffer, T) (Encoders.java:418-431,
       * 559-572): writeInt32(-1), the collection's BinaryArray / BinaryMap at the
       * writerIndex (toArray / toMap), back-patched size. A null collection is
       * written from its offsets (the device path's documented policy). */
      const onode* top = t.ntop == 1 ? &t.nodes[t.top[0]] : NULL;
      if (!top || (top->type_id != FORY_TYPE_LIST && top->type_id != FORY_TYPE_MAP)) { free_tree(&t); return -2; }
      put32(&b, b.wi, 0xFFFFFFFFu); b.wi += 4;
      if (top->type_id == FORY_TYPE_LIST) write_list_payload(&b, &t, t.top[0], cols, i);
      else write_map_payload(&b, &t, t.top[0], cols, i);
      put32(&b, frame, (uint32_t)(b.wi - frame - 4));
      if (b.overflow == 2) { free_tree(&t); return -2; }
      if (b.unsupported) { free_tree(&t); return -3; }
      continue;
    }
    if (frame_mode == 3) {                            /* encode(T): buffer.writeInt64(schemaHash) */
      put64(&b, b.wi, (uint64_t)hash); b.wi += 8;
    } else if (frame_mode) {
      put32(&b, b.wi, 0xFFFFFFFFu); b.wi += 4;        /* writeInt32(-1) */
      put64(&b, b.wi, (uint64_t)hash); b.wi += 8;     /* writeInt64(schemaHash) */
    }
    owriter w;
    row_reset(&w, &b, t.ntop);
    for (int k = 0; k < t.ntop; k++) write_value(&w, k, &t, t.top[k], cols, i);
    if (frame_mode == 1) put32(&b, frame, (uint32_t)(b.wi - frame - 4)); /* back-patch */
    if (b.overflow == 2) { free_tree(&t); return -2; }
    if (b.unsupported) { free_tree(&t); return -3; }  /* decimal precision */
  }
  if (row_offsets) row_offsets[nrows] = b.wi;
  free_tree(&t);
  if (b.overflow) return out ? -1 : b.wi;
  return b.wi;
}

/* ---------------------------------------------------------------------- */
/* decode (RowEncoderBuilder.buildDecodeExpression :215-270 + readers)     */
/* ---------------------------------------------------------------------- */

typedef struct odec {
  const uint8_t* p;
  int64_t len;
  int bad;
  int sizing;           /* 1 = count only: no column writes */
  int64_t* cursor;      /* per-column append cursor (items for lists, bytes for strings) */
  int64_t* slots;       /* per-column number of slots visited */
} odec;

static uint64_t rd(odec* D, int64_t at, int n) {
  uint64_t v = 0;
  if (at < 0 || at + n > D->len) { D->bad = 1; return 0; }
  memcpy(&v, D->p + at, (size_t)n);
  return v;
}

static void set_valid(const fory_column* c, int64_t i, int v) {
  if (!c->validity) return;
  if (v) c->validity[i >> 3] |= (uint8_t)(1u << (i & 7));
  else c->validity[i >> 3] &= (uint8_t)~(1u << (i & 7));
}

/* Null (or absent) value of node idx at output slot i: Java leaves the
 * default (0 / null) -> zeros, validity 0, empty var data; struct children
 * and list items of a null parent are absent (struct children still get a
 * slot, zero-filled, since they share the parent's length). */
static void null_value(odec* D, const otree* t, int idx, const fory_column* cols, int64_t i) {
  const onode* nd = &t->nodes[idx];
  const fory_column* c = &cols[idx];
  D->slots[idx]++;
  if (D->sizing) {
    if (nd->type_id == FORY_TYPE_STRUCT)
      for (int k = 0; k < nd->nchild; k++) null_value(D, t, nd->child[k], cols, i);
    return;
  }
  if (nd->nullable) set_valid(c, i, 0);
  if (nd->width > 0) {
    memset((uint8_t*)c->values + i * nd->width, 0, (size_t)nd->width);
  } else if (nd->type_id == FORY_TYPE_DECIMAL) {
    memset((uint8_t*)c->values + i * 16, 0, 16);
  } else if (nd->type_id == FORY_TYPE_STRUCT) {
    for (int k = 0; k < nd->nchild; k++) null_value(D, t, nd->child[k], cols, i);
  } else {
    c->offsets[i + 1] = (int32_t)D->cursor[idx];
  }
}

/* Read one value of node idx whose slot is at `slot_at` inside the row or
 * array starting at `base` (relative offsets are relative to it) and write
 * it to output slot i. */
static void read_payload(odec* D, const otree* t, int idx, const fory_column* cols, int64_t i, int64_t at,
                         int64_t size);

static void read_value(odec* D, const otree* t, int idx, const fory_column* cols,
                       int64_t i, int is_null, int64_t slot_at, int64_t base) {
  const onode* nd = &t->nodes[idx];
  const fory_column* c = &cols[idx];
  if (!D->sizing && i == 0 && nd->width < 0 && nd->type_id != FORY_TYPE_STRUCT && nd->type_id != FORY_TYPE_DECIMAL)
    c->offsets[0] = (int32_t)D->cursor[idx];
  if (is_null) { null_value(D, t, idx, cols, i); return; }  /* RowEncoderBuilder.java:239-246 */
  D->slots[idx]++;
  if (nd->nullable && !D->sizing) set_valid(c, i, 1);
  if (nd->width > 0) {
    /* UnsafeTrait.getX :68-111: the low `width` bytes of the slot */
    uint64_t v = rd(D, slot_at, nd->width);
    if (nd->type_id == FORY_TYPE_BOOL) v = v ? 1 : 0;  /* MemoryBuffer.getBoolean: byte != 0 */
    if (!D->sizing) memcpy((uint8_t*)c->values + i * nd->width, &v, (size_t)nd->width);
    return;
  }
  uint64_t os = rd(D, slot_at, 8);
  int64_t rel = (int32_t)(os >> 32);   /* (int)(offsetAndSize >> 32) */
  int64_t size = (int32_t)os;          /* (int)offsetAndSize */
  read_payload(D, t, idx, cols, i, base + rel, size);
}

/* The var payload of node idx at [at, at+size) -> output slot i (the part of
 * read_value after the slot; also the whole record of a collection frame). */
static void read_payload(odec* D, const otree* t, int idx, const fory_column* cols, int64_t i, int64_t at,
                         int64_t size) {
  const onode* nd = &t->nodes[idx];
  const fory_column* c = &cols[idx];
  if (size < 0 || at < 0 || at + size > D->len) { D->bad = 1; return; }
  switch (nd->type_id) {
    case FORY_TYPE_STRING: case FORY_TYPE_BINARY: { /* getBinary :116-137 */
      int64_t dst = D->cursor[idx];
      if (!D->sizing) {
        if (dst + size > c->capacity) { D->bad = 2; return; }
        memcpy((uint8_t*)c->values + dst, D->p + at, (size_t)size);
        c->offsets[i + 1] = (int32_t)(dst + size);
      }
      D->cursor[idx] = dst + size;
      return;
    }
    case FORY_TYPE_DECIMAL: { /* UnsafeTrait.getDecimal :139-150: DECIMAL_BYTE_LENGTH = 32 bytes at the slot's
                                 offset, DecimalUtility.getBigDecimalFromArrowBuf; an Arrow decimal128
                                 output holds it when bytes 16..31 are the sign extension of byte 15 */
      if (nd->biginteger) {  /* getBinary -> new BigInteger(bytes) */
        uint8_t v16[16];
        if (bigint_from_bytes(D->p + at, size, v16)) { D->bad = 1; return; }
        if (!D->sizing) memcpy((uint8_t*)c->values + 16 * i, v16, 16);
        return;
      }
      if (size != 32) { D->bad = 1; return; }
      const uint8_t* p = D->p + at;
      const uint8_t ext = (p[15] & 0x80) ? 0xFF : 0x00;
      for (int k = 16; k < 32; k++)
        if (p[k] != ext) { D->bad = 1; return; }
      if (!D->sizing) memcpy((uint8_t*)c->values + 16 * i, p, 16);
      return;
    }
    case FORY_TYPE_STRUCT: { /* getStruct :160-173, then the child codec's fromRow */
      int64_t bm = bitmap_bytes(nd->nchild);
      for (int k = 0; k < nd->nchild; k++) {
        int nul = (int)((rd(D, at + (k >> 3), 1) >> (k & 7)) & 1);
        read_value(D, t, nd->child[k], cols, i, nul, at + bm + 8LL * k, at);
      }
      return;
    }
    case FORY_TYPE_LIST: { /* getArray :175-186 + BinaryArray.pointTo :69-78 */
      int64_t n = (int32_t)rd(D, at, 8);  /* (int) buffer.getInt64(offset) */
      if (n < 0) { D->bad = 1; return; }
      int item = nd->child[0];
      const onode* it = &t->nodes[item];
      int64_t es = it->width < 0 ? 8 : it->width;
      int64_t hdr = 8 + bitmap_bytes(n);  /* BinaryArray.calculateHeaderInBytes :278-280 */
      int64_t first = D->cursor[idx];
      for (int64_t j = 0; j < n; j++) {
        int nul = (int)((rd(D, at + 8 + (j >> 3), 1) >> (j & 7)) & 1); /* BinaryArray.isNullAt :128-130 */
        read_value(D, t, item, cols, first + j, nul, at + hdr + j * es, at);
      }
      D->cursor[idx] = first + n;
      if (!D->sizing) c->offsets[i + 1] = (int32_t)(first + n);
      return;
    }
    case FORY_TYPE_MAP: { /* getMap + BinaryMap.pointTo (BinaryMap.java:62-77) */
      int64_t kbytes = (int32_t)rd(D, at, 4);  /* buf.getInt32(offset) */
      int64_t kat = at + 8, vat = at + 8 + kbytes;
      if (kbytes < 8 || vat + 8 > at + size) { D->bad = 1; return; }
      int64_t n = (int32_t)rd(D, kat, 8), nv = (int32_t)rd(D, vat, 8);
      if (n < 0 || n != nv) { D->bad = 1; return; } /* UnsupportedOperationException */
      int64_t first = D->cursor[idx];
      int64_t hdr = 8 + bitmap_bytes(n);
      for (int part = 0; part < 2; part++) {
        int child = nd->child[part];
        const onode* it = &t->nodes[child];
        int64_t es = it->width < 0 ? 8 : it->width;
        int64_t aat = part ? vat : kat;
        for (int64_t j = 0; j < n; j++) {
          int nul = (int)((rd(D, aat + 8 + (j >> 3), 1) >> (j & 7)) & 1);
          read_value(D, t, child, cols, first + j, nul, aat + hdr + j * es, aat);
        }
      }
      D->cursor[idx] = first + n;
      if (!D->sizing) c->offsets[i + 1] = (int32_t)(first + n);
      return;
    }
    default:
      D->bad = 3;
      return;
  }
}

/* Decode N rows/frames (Encoders.decode :177-195 / RowEncoder.fromRow).
 * row_offsets (N+1) may be NULL: STREAM frames are then parsed sequentially
 * from their int32 size fields, RAW rows assume the fixed size. With
 * sizing=1 nothing is written to `cols`; out_slots / out_bytes (num_desc
 * each) receive every column's slot count and string byte total.
 * Returns 0 ok, 4 schema mismatch, 5 corrupt, 3 capacity, 2 bad schema. */
int oracle_decode(const fory_field_desc* d, int n_desc, const uint8_t* buf, int64_t len,
                  const int64_t* row_offsets, int64_t nrows, int frame_mode,
                  const fory_column* cols, int sizing, int64_t* out_slots, int64_t* out_bytes) {
  otree t;
  if (build_tree(d, n_desc, &t) != 0) { free_tree(&t); return 2; }
  int64_t hash = 17;
  for (int k = 0; k < t.ntop; k++) hash = hash_node(hash, &t, t.top[k]);
  size_t nc = (size_t)(n_desc > 0 ? n_desc : 1);
  int64_t* cursor = (int64_t*)calloc(nc, sizeof(int64_t));
  int64_t* slots = (int64_t*)calloc(nc, sizeof(int64_t));
  odec D = {buf, len, 0, sizing, cursor, slots};
  int64_t bm = bitmap_bytes(t.ntop);
  int64_t fixed = bm + 8LL * t.ntop;
  int64_t pos = 0;
  int rc = 0;
  for (int64_t i = 0; i < nrows && !rc; i++) {
    int64_t start = row_offsets ? row_offsets[i] : pos;
    int64_t row_at = start;
    if (frame_mode == 2) {  /* ArrayEncoder / MapEncoder.decode: [i32 size][payload] (Encoders.java:394-404) */
      int64_t size = (int32_t)rd(&D, start, 4);
      int64_t end = row_offsets ? row_offsets[i + 1] : start + 4 + size;
      if (D.bad || size < 8 || start + 4 + size != end || end > len) { rc = 5; break; }
      if (i == 0 && !sizing) cols[t.top[0]].offsets[0] = 0;
      D.slots[t.top[0]]++;
      if (t.nodes[t.top[0]].nullable && !sizing) set_valid(&cols[t.top[0]], i, 1);  /* never null */
      read_payload(&D, &t, t.top[0], cols, i, start + 4, size);
      pos = end;
      if (D.bad == 2) rc = 3;
      else if (D.bad) rc = 5;
      continue;
    }
    if (frame_mode == 3) {  /* decode(byte[] bytes) = decode(wrap(bytes), bytes.length) (Encoders.java:195-197) */
      int64_t peer = (int64_t)rd(&D, start, 8);       /* buffer.readInt64() */
      int64_t end = row_offsets ? row_offsets[i + 1] : start + 8 + fixed;
      if (D.bad) { rc = 5; break; }
      if (peer != hash) { rc = 4; break; }            /* ClassNotCompatibleException */
      if (end - start < 8 + fixed || end > len) { rc = 5; break; }
      row_at = start + 8;
      pos = end;
    } else if (frame_mode) {
      int64_t size = (int32_t)rd(&D, start, 4);       /* buffer.readInt32() */
      int64_t peer = (int64_t)rd(&D, start + 4, 8);   /* buffer.readInt64() */
      if (D.bad) { rc = 5; break; }
      if (peer != hash) { rc = 4; break; }            /* ClassNotCompatibleException */
      if (size < 8 + fixed || start + 4 + size > len) { rc = 5; break; }
      row_at = start + 12;
      pos = start + 4 + size;
    } else {
      pos = start + fixed;
    }
    for (int k = 0; k < t.ntop; k++) {
      int nul = (int)((rd(&D, row_at + (k >> 3), 1) >> (k & 7)) & 1); /* BinaryRow.isNullAt :119-123 */
      read_value(&D, &t, t.top[k], cols, i, nul, row_at + bm + 8LL * k, row_at);
    }
    if (D.bad == 2) rc = 3;
    else if (D.bad) rc = 5;
  }
  if (out_slots) memcpy(out_slots, slots, nc * sizeof(int64_t));
  if (out_bytes) memcpy(out_bytes, cursor, nc * sizeof(int64_t));
  free(cursor);
  free(slots);
  free_tree(&t);
  return rc;
}

/* ---------------------------------------------------------------------- */
/* java.util.Random restatement — generator of the benchmark Struct        */
/* values (java/benchmark/.../data/Struct.java:112-134).                   */
/* ---------------------------------------------------------------------- */

typedef struct jrand { uint64_t seed; } jrand;
static void jr_init(jrand* r, int64_t s) { r->seed = ((uint64_t)s ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1); }
static int32_t jr_next(jrand* r, int bits) {
  r->seed = (r->seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
  return (int32_t)(int64_t)(r->seed >> (48 - bits));
}

/* Fill the Struct(numFields) columns for rows [row0, row0+n): field k is
 * declared f{k}, type (k%4) in {int, long, float, double}; row r uses
 * Random(seed_base + r) drawn in declaration order. cols[k] = column of
 * DECLARED field k (caller maps to schema order). */
void oracle_gen_struct(int num_decl_fields, int64_t seed_base, int64_t row0, int64_t n,
                       void* const* cols) {
  for (int64_t r = 0; r < n; r++) {
    jrand g;
    jr_init(&g, seed_base + row0 + r);
    for (int k = 0; k < num_decl_fields; k++) {
      switch (k & 3) {
        case 0: ((int32_t*)cols[k])[r] = jr_next(&g, 32); break;
        case 1: {
          int64_t hi = (int64_t)jr_next(&g, 32);
          int64_t lo = (int64_t)jr_next(&g, 32);
          ((int64_t*)cols[k])[r] = (int64_t)(((uint64_t)hi << 32) + (uint64_t)lo);
          break;
        }
        case 2: {
          float f = (float)jr_next(&g, 24) / (float)(1 << 24);
          ((float*)cols[k])[r] = f;
          break;
        }
        default: {
          int64_t a = (int64_t)(uint32_t)jr_next(&g, 26);
          int64_t b2 = (int64_t)(uint32_t)jr_next(&g, 27);
          double v = (double)((a << 27) + b2) * (1.0 / (double)(1LL << 53));
          ((double*)cols[k])[r] = v;
          break;
        }
      }
    }
  }
}
