/*
 * fory_rowfmt.h — C-ABI of the MI355X bulk row-format encoder/decoder.
 *
 * This is the drop-in boundary for Apache Fory's row-format path
 * (java/fory-format). The reference has no FFI for this path: it is the
 * pure-Java API
 *   Encoders.bean(Class)            java/fory-format/.../encoder/Encoders.java:63-231
 *   RowEncoder<T>.toRow / fromRow   java/fory-format/.../encoder/RowEncoder.java:26-32
 *   Encoder<T>.encode(MemoryBuffer,T) / decode(MemoryBuffer)
 *                                   java/fory-format/.../encoder/Encoder.java:27-40,
 *                                   Encoders.java:177-225
 * driving BinaryRowWriter / BinaryArrayWriter / BinaryRow once per object.
 * Each entry point below replaces a per-object loop of those calls with one
 * batched call over columns (the bean fields of N objects laid out as
 * Arrow-style columns) and produces the same bytes.
 * A JNI shim binds these symbols one-to-one.
 *
 * Conventions
 *  - Plain C: pointers, sizes, int status codes. No HIP/torch types; `stream`
 *    is a hipStream_t passed as void* (NULL = default stream).
 *  - Every data pointer named d_* is DEVICE memory (hipMalloc'd or
 *    device-visible pinned host memory). Descriptor arrays (fory_column*,
 *    fory_field_desc*) live in HOST memory and are copied by the call.
 *  - Calls only enqueue work on `stream`; they never allocate device memory
 *    and never synchronise, except fory_rowfmt_read_status (documented).
 *  - Plans are immutable after creation and may be shared across threads and
 *    streams. Workspaces may not be shared by concurrent calls.
 *  - Errors: non-zero fory_status; fory_rowfmt_last_error() returns a
 *    thread-local message. The Java exception each code maps to is listed.
 *  - Byte layout: docs/specification/row_format_spec.md is empty
 *    (":22-24 Coming soon"); the Java writer is the spec. See DESIGN.md.
 */
#ifndef FORY_ROWFMT_H_
#define FORY_ROWFMT_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FORY_ROWFMT_ABI_VERSION 1

/* Status codes (mapped to the reference's exceptions). */
typedef enum fory_status {
  FORY_OK = 0,
  FORY_ERR_INVALID_ARGUMENT = 1,  /* IllegalArgumentException / Preconditions */
  FORY_ERR_UNSUPPORTED = 2,       /* UnsupportedOperationException
                                     (DataTypes.java:unsupported, BinaryArrayWriter.java:99-101) */
  FORY_ERR_CAPACITY = 3,          /* IndexOutOfBoundsException (MemoryBuffer.java:303-309):
                                     output buffer too small, or a row > 2^31-1 bytes */
  FORY_ERR_SCHEMA_MISMATCH = 4,   /* ClassNotCompatibleException (Encoders.java:182-190) */
  FORY_ERR_CORRUPT = 5,           /* malformed frame / row (size field out of range) */
  FORY_ERR_DEVICE = 6,            /* HIP runtime error */
  FORY_ERR_ENCODER = 7            /* EncoderException (Encoders.java:227-230): bad schema */
} fory_status;

/* Arrow type ids — the ordinals of org.apache.fory.format.type.ArrowType
 * (java/fory-format/.../type/ArrowType.java:25-160), which are also the ids
 * DataTypes.computeSchemaHash folds in (DataTypes.java:499-544). */
enum fory_type_id {
  FORY_TYPE_BOOL = 1,
  FORY_TYPE_INT8 = 3,
  FORY_TYPE_INT16 = 5,
  FORY_TYPE_INT32 = 7,
  FORY_TYPE_INT64 = 9,
  FORY_TYPE_FLOAT = 11,
  FORY_TYPE_DOUBLE = 12,
  FORY_TYPE_STRING = 13,    /* utf8 */
  FORY_TYPE_BINARY = 14,
  FORY_TYPE_DATE32 = 16,
  FORY_TYPE_TIMESTAMP = 18,
  FORY_TYPE_DECIMAL = 23,   /* ArrowType.DECIMAL (= DECIMAL128's id): BigDecimal / BigInteger fields
                               (BigInteger: reserved = FORY_DECIMAL_BIGINTEGER) */
  FORY_TYPE_LIST = 25,
  FORY_TYPE_STRUCT = 26,
  FORY_TYPE_MAP = 30
};

/* One node of the schema, flattened in pre-order. A schema is the sequence of
 * its top-level fields; a STRUCT node is followed by its `num_children` child
 * subtrees, a LIST node by exactly one subtree (the element field "item"), a
 * MAP node by exactly two: the key field (not nullable, DataTypes.mapField
 * DataTypes.java:418-424) and the value field — Arrow's entries struct is
 * elided, as in the schema hash (DataTypes.java:522-527).
 * Order must be the Java schema order: TypeInference.inferSchema
 * (TypeInference.java:68-80,238-247) = fields sorted by name
 * (Descriptor.java:415-423). */
typedef struct fory_field_desc {
  int32_t type_id;       /* enum fory_type_id */
  int32_t nullable;      /* 1 = boxed/String/bean/List (TypeInference.java:182-247) */
  int32_t num_children;  /* STRUCT: >= 0, LIST: 1, MAP: 2, others: 0 */
  int32_t reserved;      /* DECIMAL: the precision (0 = 38, DecimalUtils.MAX_PRECISION), or
                            FORY_DECIMAL_BIGINTEGER; else 0 */
} fory_field_desc;

/* fory_field_desc.reserved of a DECIMAL node whose bean field is java.math.BigInteger
 * (TypeInference.java:203-204 types it Decimal(38, 0), like a BigDecimal's type but scale 0).
 * The codec does not write it with writeDecimal: it writes value.toByteArray()
 * (BaseBinaryEncoderBuilder.java:192-194) through BinaryWriter.write(int, byte[]) ->
 * writeUnaligned (BinaryWriter.java:167-194): the minimal big-endian two's complement,
 * bitLength / 8 + 1 bytes (1..16 for a decimal128 value), zero-padded to 8, behind an
 * (offset, length) slot; and reads it back as new BigInteger(bytes)
 * (BaseBinaryEncoderBuilder.java:559-560). No precision check applies. Its column is a
 * decimal128 column like any DECIMAL's (the value at scale 0); a row whose bytes do not
 * fit one (0 or more than 16 bytes) decodes as FORY_ERR_CORRUPT. The precision bits
 * (low 8) must be 0 or 38 with this flag. */
#define FORY_DECIMAL_BIGINTEGER 0x100

/* Column of one field (index = pre-order index of its fory_field_desc).
 *  fixed-width : values = length * width bytes, little-endian
 *                (BOOL: 1 byte per value, non-zero = true; FLOAT/DOUBLE raw IEEE bits)
 *  STRING/BINARY: offsets = length+1 int32 Arrow offsets into values (bytes)
 *  LIST        : offsets = length+1 int32 Arrow offsets into the child column
 *  MAP         : offsets = length+1 int32 Arrow offsets into the key and value
 *                columns (entries); key/value columns hold one slot per entry
 *  DECIMAL     : values = length * 16 bytes, Arrow decimal128 (the unscaled value,
 *                little-endian two's complement, at the field's scale). A row holds it
 *                out of line as 32 bytes sign-extended behind an (offset, 32) slot
 *                (BinaryWriter.writeDecimal, BinaryWriter.java:214-230,
 *                DecimalUtils.DECIMAL_BYTE_LENGTH = 32); |value| > 10^precision - 1
 *                is FORY_ERR_UNSUPPORTED on encode (DecimalUtility.checkPrecisionAndScale).
 *                BigInteger fields (FORY_DECIMAL_BIGINTEGER): the same column; the row holds
 *                toByteArray()'s bytes instead (see FORY_DECIMAL_BIGINTEGER)
 *  STRUCT      : values/offsets unused; children have the same length
 *  validity    : Arrow validity bitmap, LSB-first, 1 = valid; NULL = all valid.
 *                Only read/written for nullable fields.
 *  length      : number of slots (rows for top-level and struct children,
 *                total items for a list element column).
 *  capacity    : bytes available at `values` (decode outputs; ignored on encode) */
typedef struct fory_column {
  void* values;
  int32_t* offsets;
  uint8_t* validity;
  int64_t length;
  int64_t capacity;
} fory_column;

typedef struct fory_plan fory_plan;

typedef struct fory_plan_info {
  int64_t schema_hash;       /* DataTypes.computeSchemaHash (DataTypes.java:499-544) */
  int32_t num_fields;        /* top-level fields */
  int32_t num_columns;       /* = num_desc (one column per pre-order node) */
  int32_t bitmap_bytes;      /* BitUtils.calculateBitmapWidthInBytes (BitUtils.java:175-177) */
  int32_t fixed_size;        /* bitmap + 8*num_fields (BinaryRowWriter.java:46-52) */
  int32_t fixed_width;       /* 1 if every row has the same size (no varlen/nested fields) */
  int32_t row_size;          /* fixed_size when fixed_width, else -1 */
} fory_plan_info;

/* Framing modes for a batch of N rows:
 *  FORY_FRAME_RAW   : rows back to back; row i = BinaryRowWriter.getRow()
 *                     bytes of object i (BinaryRowWriter.java:131-136,
 *                     BinaryRow.toBytes BinaryRow.java:229-231).
 *  FORY_FRAME_STREAM: frames back to back, exactly what N calls of
 *                     Encoder.encode(MemoryBuffer, T) write into one buffer
 *                     (Encoders.java:213-225):
 *                     [int32 LE 8+rowSize][int64 LE schemaHash][row].     */
enum fory_frame_mode { FORY_FRAME_RAW = 0, FORY_FRAME_STREAM = 1, FORY_FRAME_COLLECTION = 2, FORY_FRAME_HASHED = 3 };
/*  FORY_FRAME_HASHED: N calls of Encoder.encode(T) -> byte[] (Encoders.java:203-210):
 *                     [int64 LE schemaHash][row] per record, back to back; like
 *                     RAW rows they do not delimit themselves, so row offsets
 *                     (encoded_size) locate each byte[]. Decode = N x
 *                     Encoder.decode(byte[]) (Encoders.java:195-197): the hash is
 *                     checked (FORY_ERR_SCHEMA_MISMATCH). The reference points the
 *                     BinaryRow at [8, 8 + bytes.length) — a size 8 bytes too large
 *                     (Encoders.java:191-193); the decoded values do not depend on
 *                     it, and the row's own bytes here are [8, bytes.length). */
/*  FORY_FRAME_COLLECTION: the standalone collection encoders — N calls of
 *                     ArrayEncoder / MapEncoder .encode(MemoryBuffer, T)
 *                     (Encoders.arrayEncoder / mapEncoder, Encoders.java:418-431,
 *                     559-572): [int32 LE size][BinaryArray | BinaryMap].
 *                     Only for plans of exactly one top-level LIST or MAP field
 *                     (the collection); no schema hash. A null collection is
 *                     written from its offsets (empty for Arrow-style nulls);
 *                     decoding yields not-null collections. Decode checks
 *                     size == frame length - 4 (FORY_ERR_CORRUPT otherwise). */

/* --- library / errors --------------------------------------------------- */
int32_t fory_rowfmt_abi_version(void);
const char* fory_rowfmt_last_error(void);   /* thread-local; never NULL */

/* --- plan: replaces TypeInference/BinaryRowWriter(Schema)/computeSchemaHash
 *     done once per bean class in Encoders.bean (Encoders.java:75-78,155). */
int fory_rowfmt_plan_create(const fory_field_desc* fields, int32_t num_desc,
                            fory_plan** out_plan);
void fory_rowfmt_plan_destroy(fory_plan* plan);
int fory_rowfmt_plan_info(const fory_plan* plan, fory_plan_info* out_info);

/* Device workspace (bytes) every call below needs for `num_rows` rows. */
int64_t fory_rowfmt_workspace_bytes(const fory_plan* plan, int64_t num_rows);

/* Workspace (bytes, >= fory_rowfmt_workspace_bytes) with which encoded_size / encode
 * of these columns take the columnar tree engine: plans with list / map nesting beyond
 * the op programs (BaseBinaryEncoderBuilder.serializeFor's arrays and maps,
 * :236-351 / :370-427) are sized node by node and written tile by tile, with per-node
 * temporaries of each column's element count (fory_column.length of list items and map
 * keys / values: their offsets must lie in [0, length]). A smaller workspace keeps the
 * per-record engine; the bytes are identical. The encode that directly follows an
 * encoded_size of the same plan, columns, rows and framing on the same workspace uses the
 * sizes that call left there, once (the columns must not change in between: a string
 * whose length no longer matches is not written and sets FORY_ERR_ENCODER); encode leaves
 * no sizes of its own, and any other call with that workspace discards them. Equals
 * fory_rowfmt_workspace_bytes for every other plan. */
int64_t fory_rowfmt_encode_workspace_bytes(const fory_plan* plan, const fory_column* cols,
                                           int64_t num_rows);

/* Workspace (bytes, >= fory_rowfmt_workspace_bytes) with which decode_sizes / decode of
 * such plans take the columnar decode: per-node passes (rows and beans field by field,
 * lists and maps element by element) with the positions of every bean / list / map
 * instance of the levels allocated so far in out_cols (their fory_column.length) as
 * temporaries. Ask again after allocating a deeper level: the need grows with it. A smaller
 * workspace keeps the per-record decoder; the columns are identical. The positions are
 * state between calls: a decode_sizes of the next level and the final decode read the
 * positions the previous decode_sizes of the same plan, rows and columns left in the
 * workspace, so the workspace must not be written in between. Any other call with that
 * workspace discards them, and the next call starts at level 0. */
int64_t fory_rowfmt_decode_workspace_bytes(const fory_plan* plan, const fory_column* out_cols,
                                           int64_t num_rows);

/* --- encode: replaces N x { writer.reset(); GeneratedRowEncoder.toRow(obj) }
 *     (Encoders.java:92-95 / 213-225, RowEncoderBuilder.java:177-208).
 *
 * fory_rowfmt_encoded_size: writes d_row_offsets[0..N] (int64, device):
 * d_row_offsets[i] = byte offset of row/frame i in the output,
 * d_row_offsets[N] = total bytes. Needed before encode for varlen plans;
 * for fixed-width plans it is i*stride and may be skipped. */
int fory_rowfmt_encoded_size(const fory_plan* plan, const fory_column* cols,
                             int64_t num_rows, int32_t frame_mode,
                             int64_t* d_row_offsets, void* d_workspace,
                             int64_t workspace_bytes, void* stream);

/* Encode N rows into d_out (device, out_capacity bytes, 16-byte aligned for
 * fixed-width plans). d_row_offsets from fory_rowfmt_encoded_size is required
 * for varlen plans, ignored (may be NULL) for fixed-width plans, whose
 * capacity is checked on the host. A varlen row that would end past
 * out_capacity is skipped and sets *d_status = FORY_ERR_CAPACITY (d_status
 * may be NULL). Null slots are written as zeros (the bytes Java produces on
 * a fresh buffer; BinaryWriter.java:123-126). */
int fory_rowfmt_encode(const fory_plan* plan, const fory_column* cols,
                       int64_t num_rows, int32_t frame_mode,
                       const int64_t* d_row_offsets, void* d_out,
                       int64_t out_capacity, int32_t* d_status,
                       void* d_workspace, int64_t workspace_bytes,
                       void* stream);

/* --- decode: replaces N x { Encoder.decode(buffer) | RowEncoder.fromRow(row) }
 *     (Encoders.java:177-195, RowEncoderBuilder.java:215-318, UnsafeTrait.java:68-197).
 *
 * d_row_offsets: N+1 offsets of each row (RAW) or frame (STREAM): required
 * for varlen plans; ignored (may be NULL) for fixed-width plans, whose rows
 * are i*stride (16-byte aligned d_rows).
 *
 * fory_rowfmt_decode_sizes (varlen plans; no-op for fixed-width): writes
 * offsets[num_rows] (the total: bytes, or items for LIST, entries for MAP) of
 * every STRING/BINARY/LIST/MAP output column's `offsets` array (num_rows+1 int32,
 * device), so the caller can size `values` and list element columns. The
 * rest of `offsets` is complete after fory_rowfmt_decode (for plans whose
 * top-level fields are all fixed/string/binary/list, decode_sizes writes
 * tile-start prefixes at offsets[64*k] and decode fills the records in
 * between): pass the same rows, row offsets and column arrays to both calls
 * and do not modify `offsets` in between.
 *
 * Columns under lists / maps (indexed by element) are sized level by level.
 * Level L = the columns with L list/map ancestors; level 0 are the rows' own
 * columns (num_rows positions). A level-(L+1) column has as many positions as
 * its nearest list/map ancestor's total (offsets[length] of that column). Pass
 * the deeper columns with offsets = NULL (skipped) to the first call; after
 * each call allocate the next level's columns (offsets of length+1 int32 for
 * STRING/BINARY/LIST/MAP, `length` = positions) and call decode_sizes again:
 * every call re-sizes each level whose STRING/BINARY/LIST/MAP columns all have
 * offsets, in order, and stops at the first level that does not. Any nesting of
 * struct / list / map fields has a device path (op programs for the common
 * shapes, a tree engine for list<list<...>>, List<Bean> with var fields,
 * Map<K, Bean> and the like).
 *
 * The columnar tree engine (a workspace of fory_rowfmt_decode_workspace_bytes) may also
 * write the values and validity of the levels a decode_sizes call sizes (all but string /
 * binary bytes); pass the same columns to the later calls. On one workspace, a
 * decode_sizes call resumes after the levels the directly preceding decode_sizes ran for
 * the same plan, rows, offsets and columns, and a decode directly after them only copies
 * the string bytes; each call consumes what the previous one left, and any other call on
 * the workspace drops it (the result is the same either way when the rows and columns
 * did not change in between). A list / map item column shorter than its items
 * (fory_column.length) is not written past its length: FORY_ERR_CAPACITY; on encode,
 * offsets past an item column's length are FORY_ERR_INVALID_ARGUMENT.
 *
 * fory_rowfmt_decode: writes values/offsets/validity of out_cols. Null
 * values decode to 0 (RowEncoderBuilder.java:239-246 leaves the Java default).
 * In STREAM mode every frame's int32 size and int64 schema hash are checked
 * (Encoders.java:177-193); a mismatch sets *d_status (device int32) to
 * FORY_ERR_SCHEMA_MISMATCH or FORY_ERR_CORRUPT. d_status may be NULL. */
int fory_rowfmt_decode_sizes(const fory_plan* plan, const void* d_rows,
                             const int64_t* d_row_offsets, int64_t num_rows,
                             int32_t frame_mode, const fory_column* out_cols,
                             int32_t* d_status, void* d_workspace,
                             int64_t workspace_bytes, void* stream);
int fory_rowfmt_decode(const fory_plan* plan, const void* d_rows,
                       const int64_t* d_row_offsets, int64_t num_rows,
                       int32_t frame_mode, const fory_column* out_cols,
                       int32_t* d_status, void* d_workspace,
                       int64_t workspace_bytes, void* stream);

/* --- frame index: the stream alone -> row offsets, on the device.
 * Encoder.decode(MemoryBuffer) reads [i32 size][i64 hash], checks the hash and
 * advances by the frame (Encoders.java:176-193): the frames delimit themselves.
 * A receiver that has only the stream (e.g. from an RPC socket) calls this
 * before fory_rowfmt_decode_sizes / fory_rowfmt_decode: it writes the starts of
 * the first num_rows frames of d_rows (rows_bytes bytes, 4-byte aligned) to
 * d_row_offsets[0..num_rows-1] and the end of frame num_rows-1 (= the bytes the
 * N decodes consume) to d_row_offsets[num_rows]. FORY_FRAME_STREAM only (RAW
 * rows are not self-delimiting; collection frames carry no schema hash to
 * resynchronise on: FORY_ERR_UNSUPPORTED). A size field out of range, or fewer
 * than num_rows frames in rows_bytes, sets *d_status = FORY_ERR_CORRUPT; schema
 * hashes are checked by the decode that follows. Bytes past the last frame are
 * never required to be frames. Workspace: fory_rowfmt_index_workspace_bytes. */
int64_t fory_rowfmt_index_workspace_bytes(const fory_plan* plan, int64_t num_rows, int64_t rows_bytes);
int fory_rowfmt_index_frames(const fory_plan* plan, const void* d_rows, int64_t rows_bytes, int64_t num_rows,
                             int32_t frame_mode, int64_t* d_row_offsets, int32_t* d_status, void* d_workspace,
                             int64_t workspace_bytes, void* stream);

/* Synchronises `stream` and returns the status word written by decode
 * (FORY_OK if none). Sets last_error with the reference's message shape. */
int fory_rowfmt_read_status(const int32_t* d_status, void* stream);

/* --- <= 2 GiB MemoryBuffer windows. A MemoryBuffer is int-sized
 * (java/fory-core/.../memory/MemoryBuffer.java:87), so a JVM receives a big batch
 * as several buffers, each holding whole rows/frames. fory_rowfmt_split_windows
 * splits a batch's output (HOST row_offsets[0..num_rows], or row i at i * stride
 * when row_offsets is NULL) greedily into windows of at most max_window_bytes
 * (2^31 - 1 for a MemoryBuffer): window w = rows [first[w], first[w+1]) = bytes
 * [offsets[first[w]], offsets[first[w+1]]) of the device output, never a row or
 * frame across a boundary. first has room for max_windows + 1 entries;
 * *num_windows receives the count. A row larger than a window, or more than
 * max_windows windows: FORY_ERR_CAPACITY. Host-only (no device work). */
int fory_rowfmt_split_windows(const int64_t* row_offsets, int64_t stride, int64_t num_rows, int64_t max_window_bytes,
                              int32_t max_windows, int64_t* first, int32_t* num_windows);

/* --- host path: replaces N x Encoder.encode(MemoryBuffer, T) /
 *     Encoder.decode(MemoryBuffer) over OFF-HEAP host buffers
 *     (Encoders.java:177-225; MemoryBuffer.getUnsafeAddress,
 *     java/fory-core/.../memory/MemoryBuffer.java:287-297) — the path's real
 *     endpoints (JVM buffers on their way to / from an RPC socket).
 *
 * A host context owns one device, three HIP streams and two sets of device
 * chunk buffers (columns, rows, workspace), allocated once at creation. Each
 * call splits the batch into chunks of chunk_rows records (rounded up to a
 * multiple of 64) and pipelines H2D of chunk k+1 || kernel of chunk k || D2H
 * of chunk k-1. Calls are synchronous: they return when the host output is
 * complete (or with the first error). All pointers are HOST memory; register
 * long-lived buffers (fory_rowfmt_host_register = hipHostRegister) for full
 * PCIe rate. The plan must outlive the context; a context serves one call at
 * a time. Fixed-width plans use the chunk pipeline (host_encode / host_decode);
 * varlen plans the _var entry points below. Output bytes equal
 * fory_rowfmt_encode's / decode's. */
typedef struct fory_host_ctx fory_host_ctx;
int fory_rowfmt_host_ctx_create(const fory_plan* plan, int32_t device, int64_t chunk_rows,
                                fory_host_ctx** out_ctx);
void fory_rowfmt_host_ctx_destroy(fory_host_ctx* ctx);
/* host_cols: values (+ validity for nullable fields) in host memory; rows
 * written back to back into host_out (out_capacity bytes; FORY_ERR_CAPACITY
 * before any work if n * stride does not fit: IndexOutOfBoundsException). */
int fory_rowfmt_host_encode(fory_host_ctx* ctx, const fory_column* host_cols, int64_t num_rows,
                            int32_t frame_mode, void* host_out, int64_t out_capacity);
/* host_rows: rows_bytes of rows/frames; host_out_cols: values (+ validity)
 * targets in host memory. STREAM mode checks every frame's size and schema
 * hash (FORY_ERR_SCHEMA_MISMATCH: ClassNotCompatibleException). */
int fory_rowfmt_host_decode(fory_host_ctx* ctx, const void* host_rows, int64_t rows_bytes,
                            int64_t num_rows, int32_t frame_mode, const fory_column* host_out_cols);
/* Encode into several host windows (e.g. the off-heap addresses of int-sized
 * MemoryBuffers): window w receives whole rows/frames while they fit
 * window_caps[w] bytes (greedy, in order; a window too small for the next row stays
 * empty), then the next window; window_rows / window_bytes (num_windows each,
 * nullable) receive what each holds. Fixed-width and varlen plans. Not enough room
 * in all windows: FORY_ERR_CAPACITY (fixed-width plans: before any row is copied;
 * varlen plans: the chunks before the overflow may already be written). */
int fory_rowfmt_host_encode_windows(fory_host_ctx* ctx, const fory_column* host_cols, int64_t num_rows,
                                    int32_t frame_mode, void* const* windows, const int64_t* window_caps,
                                    int32_t num_windows, int64_t* window_rows, int64_t* window_bytes);
/* Varlen plans (strings, lists, maps, nested structs; also FORY_FRAME_COLLECTION):
 * the context keeps its device buffers and grows them as needed.
 * host_encode_var: host columns (Arrow layout, as fory_rowfmt_encode) -> rows /
 * frames back to back in host_out, pipelined by chunks of chunk_rows records (each
 * chunk's column slices follow its rows' offsets; its rows are sized on the device,
 * then placed after the chunks before); *out_bytes receives the total (also on
 * FORY_ERR_CAPACITY, so the caller can grow its buffer; rows of the chunks before
 * the overflow may already be written), host_row_offsets (n+1, may be NULL) the
 * row/frame starts. */
int fory_rowfmt_host_encode_var(fory_host_ctx* ctx, const fory_column* host_cols, int64_t num_rows,
                                int32_t frame_mode, void* host_out, int64_t out_capacity,
                                int64_t* host_row_offsets, int64_t* out_bytes);
/* Decode of host rows in two calls (the caller allocates in between):
 * host_decode_var_sizes stages the rows (host_row_offsets: n+1 starts, required)
 * on the device and writes per pre-order column its element count
 * (host_counts: rows for top-level fields, items / entries below a list or map)
 * and value bytes (host_bytes: count x width, or the string/binary bytes; 0 for
 * struct/list/map). host_decode_var then decodes that staged batch into
 * host_out_cols: values (>= host_bytes), offsets (count + 1 int32) for
 * string/binary/list/map, validity ((count + 7) / 8 bytes) for nullable fields.
 * Errors as fory_rowfmt_decode (schema hash, corrupt frame). */
int fory_rowfmt_host_decode_var_sizes(fory_host_ctx* ctx, const void* host_rows,
                                      const int64_t* host_row_offsets, int64_t num_rows,
                                      int32_t frame_mode, int64_t* host_counts, int64_t* host_bytes);
/* The same staging for a receiver that has only the frame stream (STREAM mode):
 * the first num_rows frames of host_rows (rows_bytes bytes) are found on the
 * device (fory_rowfmt_index_frames), *consumed_bytes receives the bytes those
 * frames span (Encoder.decode's reader index after num_rows calls), then
 * host_decode_var decodes them. */
int fory_rowfmt_host_decode_stream_sizes(fory_host_ctx* ctx, const void* host_rows, int64_t rows_bytes,
                                         int64_t num_rows, int64_t* host_counts, int64_t* host_bytes,
                                         int64_t* consumed_bytes);
/* Any host_encode_var on the context between the sizes call and this one drops
 * the staged batch (FORY_ERR_INVALID_ARGUMENT: stage it again). */
int fory_rowfmt_host_decode_var(fory_host_ctx* ctx, const fory_column* host_out_cols);
/* One-call decode into caller-sized host columns, pipelined by chunks of chunk_rows
 * records (H2D of chunk k+1 || sizes + decode of chunk k || D2H of chunk k-1): the
 * receiver that keeps (and grows) its Arrow buffers across batches, as host_encode_var
 * does its output. host_out_cols[i].length: element capacity of every column (offsets
 * need length + 1 entries, validity (length + 7) / 8 bytes, fixed values length x
 * width); .capacity: value-byte capacity of string/binary columns. host_counts /
 * host_bytes (num_columns each) receive the batch's element counts and value bytes —
 * also on FORY_ERR_CAPACITY (a column too small; the columns hold a partial decode),
 * so the caller can grow and call again. host_row_offsets (n+1) required. */
int fory_rowfmt_host_decode_var_into(fory_host_ctx* ctx, const void* host_rows, const int64_t* host_row_offsets,
                                     int64_t num_rows, int32_t frame_mode, const fory_column* host_out_cols,
                                     int64_t* host_counts, int64_t* host_bytes);
/* Pins [host_ptr, host_ptr + bytes) (hipHostRegister): copies inside it become direct
 * DMAs (their device mapping comes from the library's registration table, no runtime
 * query per copy); other memory goes through the context's pinned staging. Two live
 * registrations may not overlap (FORY_ERR_INVALID_ARGUMENT; sharing a page is fine).
 * Unregister takes the start of a registered range (else FORY_ERR_INVALID_ARGUMENT) and
 * checks that the runtime no longer maps the range (FORY_ERR_DEVICE otherwise).
 * Unregister before the memory is freed. */
int fory_rowfmt_host_register(void* host_ptr, int64_t bytes);
int fory_rowfmt_host_unregister(void* host_ptr);

#ifdef __cplusplus
}
#endif
#endif /* FORY_ROWFMT_H_ */
