/*
 * MI355X row-format batch path: the batched RowEncoder / Encoder of one bean class,
 * over libfory_rowfmt.so (include/fory_rowfmt.h) through jni/fory_rowfmt_jni.c.
 */
package org.apache.fory.format.encoder;

import java.nio.ByteBuffer;
import java.util.ArrayList;
import java.util.List;
import org.apache.arrow.vector.types.pojo.Schema;
import org.apache.fory.format.type.DataTypes;
import org.apache.fory.format.type.TypeInference;
import org.apache.fory.memory.MemoryBuffer;
import org.apache.fory.util.Preconditions;

/**
 * N x {@code Encoder<T>} calls in one device batch. Bytes are identical to the per-object
 * reference calls on the same values:
 *
 * <ul>
 *   <li>{@link #encode}: N x {@code encode(MemoryBuffer, T)} (Encoders.java:213-225), the
 *       {@code [i32 8+size][i64 hash][row]} frame stream;
 *   <li>{@link #encodeRows}: N x {@code toRow(T).toBytes()} (Encoders.java:92-95), raw rows
 *       back to back, with their offsets;
 *   <li>{@link #encodeEach}: N x {@code encode(T)} (Encoders.java:203-210), {@code [i64
 *       hash][row]} each;
 *   <li>{@link #decode}: N x {@code decode(MemoryBuffer)} (Encoders.java:177-193) from the
 *       frames alone; {@link #decodeInto} when the frame offsets travel with the stream.
 * </ul>
 *
 * The beans cross the boundary as a {@link ColumnBatch} (Arrow layout, off-heap). The
 * schema is {@code TypeInference.inferSchema(beanClass)} (TypeInference.java:58-80), the
 * one {@code Encoders.bean(beanClass)} uses, so field order and schema hash agree. Like a
 * reference encoder, an instance is single-threaded; instances on different threads or
 * devices are independent.
 *
 * <p>The object-level surface is {@code Encoder<T>}'s four methods (Encoder.java:31-39)
 * over a batch of N objects: {@link #encode(MemoryBuffer, List)}, {@link #encode(List)},
 * {@link #decode(MemoryBuffer, int)}, {@link #decode(byte[][])}. The objects become
 * columns through {@link BeanColumns} (the generated codec's per-field conversions), so a
 * caller of {@code Encoders.bean(Foo.class)} swaps one line:
 *
 * <pre>{@code
 * // RowEncoder<Foo> enc = Encoders.bean(Foo.class);  for (Foo f : foos) enc.encode(buf, f);
 * BatchRowEncoder<Foo> enc = new BatchRowEncoder<>(Foo.class);  enc.encode(buf, foos);
 * }</pre>
 */
public final class BatchRowEncoder<T> implements AutoCloseable {
  static {
    System.loadLibrary("fory_rowfmt_jni");
  }

  /** include/fory_rowfmt.h frame modes. */
  public static final int FRAME_RAW = 0;

  public static final int FRAME_STREAM = 1;
  public static final int FRAME_HASHED = 3;

  private final Schema schema;
  private final BeanColumns<T> beans; // objects <-> columns
  private ByteBuffer scratch; // heap MemoryBuffers: staged through this direct buffer
  private final long plan; // fory_plan*
  private final long hostCtx; // fory_host_ctx*: three HIP streams + device chunk slots
  private final long schemaHash;
  private final int rowSize; // fixed-width plans: BinaryRowWriter fixed size, else -1

  public BatchRowEncoder(Class<T> beanClass) {
    this(beanClass, 0, 1 << 20);
  }

  /** @param device HIP device ordinal; @param chunkRows records per pipelined chunk */
  public BatchRowEncoder(Class<T> beanClass, int device, long chunkRows) {
    this.schema = TypeInference.inferSchema(beanClass);
    this.beans = new BeanColumns<>(beanClass, schema);
    // BigInteger fields flagged (FORY_DECIMAL_BIGINTEGER): the row holds toByteArray()
    this.plan = nPlanCreate(DeviceSchemas.flatten(schema, beans.bigIntegerColumns())); // EncoderException / UnsupportedOperation
    this.schemaHash = nSchemaHash(plan);
    this.rowSize = nRowSize(plan);
    Preconditions.checkArgument(
        schemaHash == DataTypes.computeSchemaHash(schema), "device schema hash differs from the reference's");
    this.hostCtx = nHostCtxCreate(plan, device, chunkRows);
  }

  public Schema schema() {
    return schema;
  }

  public long schemaHash() {
    return schemaHash;
  }

  // ------------------------------------------------------------ Encoder<T> over batches

  /**
   * N x {@code encode(MemoryBuffer, T)} (Encoders.java:213-225): the N frames {@code [i32
   * 8+size][i64 hash][row]} appended at the buffer's writerIndex, which ends past them. The
   * buffer grows as a MemoryBuffer does ({@code ensure}); an off-heap buffer receives the
   * frames straight from the device, a heap one through a direct staging buffer.
   * IndexOutOfBoundsException when the frames do not fit an int-sized buffer.
   */
  public void encode(MemoryBuffer buffer, List<T> objs) {
    ColumnBatch cols = new ColumnBatch(schema);
    beans.fill(objs, cols);
    appendFrames(buffer, cols, objs.size(), FRAME_STREAM);
  }

  /** N x {@code encode(T)} (Encoders.java:203-210): one {@code [i64 hash][row]} array each. */
  public byte[][] encode(List<T> objs) {
    ColumnBatch cols = new ColumnBatch(schema);
    beans.fill(objs, cols);
    return encodeEach(cols, objs.size());
  }

  /**
   * N x {@code decode(MemoryBuffer)} (Encoders.java:177-193): N objects from the frames at
   * the buffer's readerIndex, which ends past them. ClassNotCompatibleException on a
   * schema-hash mismatch.
   */
  public List<T> decode(MemoryBuffer buffer, int numRows) {
    ColumnBatch out = new ColumnBatch(schema);
    decode(buffer, numRows, out);
    return beans.read(out, numRows);
  }

  /** N x {@code decode(byte[])} (Encoders.java:195-197), one {@code [i64 hash][row]} each. */
  public List<T> decode(byte[][] each) {
    int n = each.length;
    long[] offs = new long[n + 1];
    for (int i = 0; i < n; i++) offs[i + 1] = offs[i] + each[i].length;
    if (offs[n] > Integer.MAX_VALUE - 16) {
      throw new IndexOutOfBoundsException("decode batch of " + offs[n] + " bytes: split the batch");
    }
    ByteBuffer buf = scratch(offs[n]);
    for (byte[] b : each) buf.put(b);
    long addr = ColumnBatch.baseAddress(buf); // the rows' start (buf's position is past them)
    ColumnBatch out = new ColumnBatch(schema);
    if (rowSize >= 0) {
      for (byte[] b : each) {
        if (b.length != rowSize + 8) throw new EncoderException("row of " + b.length + " bytes, expected " + (rowSize + 8));
      }
      nDecodeFixed(hostCtx, addr, offs[n], n, FRAME_HASHED, out);
    } else {
      nDecodeInto(hostCtx, addr, offs, n, FRAME_HASHED, out);
    }
    return beans.read(out, n);
  }

  /** The bytes of N frames (fixed-width plans: computed; else a sizing pass on the device). */
  private long frameBytes(long[] cols, int numRows, int frame) {
    int hdr = frame == FRAME_STREAM ? 12 : frame == FRAME_HASHED ? 8 : 0;
    return rowSize >= 0 ? (long) numRows * (rowSize + hdr) : nEncodedBytes(hostCtx, cols, numRows, frame);
  }

  private void appendFrames(MemoryBuffer buffer, ColumnBatch columns, int numRows, int frame) {
    long[] cols = columns.addresses();
    long need = frameBytes(cols, numRows, frame);
    int at = buffer.writerIndex();
    if (at + need > Integer.MAX_VALUE - 8) {
      throw new IndexOutOfBoundsException(
          "writerIndex " + at + " + " + need + " bytes of frames exceed an int-sized MemoryBuffer");
    }
    buffer.ensure((int) (at + need));
    long[] bytes = new long[1];
    if (buffer.isOffHeap()) {
      nEncodeWindows(hostCtx, cols, numRows, frame, new long[] {buffer.getUnsafeAddress() + at}, new long[] {need}, bytes);
    } else {
      ByteBuffer tmp = scratch(need);
      long ta = ColumnBatch.baseAddress(tmp);
      nEncodeWindows(hostCtx, cols, numRows, frame, new long[] {ta}, new long[] {need}, bytes);
      buffer.copyFromUnsafe(at, null, ta, need);
    }
    buffer.writerIndex((int) (at + bytes[0]));
  }

  /** A direct staging buffer of at least {@code bytes} (kept, grown), position 0. */
  private ByteBuffer scratch(long bytes) {
    if (bytes > Integer.MAX_VALUE - 16) {
      throw new IndexOutOfBoundsException(bytes + " bytes exceed a direct buffer");
    }
    if (scratch == null || scratch.capacity() < bytes) {
      scratch = ByteBuffer.allocateDirect((int) Math.max(bytes + bytes / 4 + 16, 4096));
    }
    scratch.clear();
    return scratch;
  }

  // ------------------------------------------------------------ column batches

  /**
   * N x encode(MemoryBuffer, T). A MemoryBuffer is int-sized (MemoryBuffer.java:87): the
   * stream lands in as many off-heap buffers of at most 2^31 - 1 bytes as it needs, each
   * holding whole frames (fory_rowfmt_host_encode_windows splits greedily), writerIndex
   * at its end. IndexOutOfBoundsException when a single frame exceeds a window.
   */
  public List<MemoryBuffer> encode(ColumnBatch columns, int numRows) {
    return encodeWindows(columns, numRows, FRAME_STREAM);
  }

  /** N x toRow(T).toBytes() back to back (raw rows), in windows as {@link #encode}. */
  public List<MemoryBuffer> encodeRows(ColumnBatch columns, int numRows) {
    return encodeWindows(columns, numRows, FRAME_RAW);
  }

  private List<MemoryBuffer> encodeWindows(ColumnBatch columns, int numRows, int frame) {
    long[] cols = columns.addresses();
    long[] sizes; // the exact bytes of each window: whole frames, greedily, <= 2^31 - 1 each
    if (rowSize >= 0) {
      long stride = rowSize + (frame == FRAME_STREAM ? 12 : frame == FRAME_HASHED ? 8 : 0);
      long perWindow = Integer.MAX_VALUE / stride;
      int windows = (int) Math.max(1, (numRows + perWindow - 1) / perWindow);
      sizes = new long[windows];
      for (int w = 0; w < windows; w++) sizes[w] = Math.min(perWindow, numRows - w * perWindow) * stride;
    } else { // the device sizes the rows, fory_rowfmt_split_windows places them
      sizes = nWindowBytes(hostCtx, cols, numRows, frame, Integer.MAX_VALUE);
    }
    int windows = sizes.length;
    List<MemoryBuffer> out = new ArrayList<>(windows);
    long[] addrs = new long[windows];
    long[] caps = new long[windows];
    for (int w = 0; w < windows; w++) {
      int cap = (int) Math.max(sizes[w], 1);
      MemoryBuffer b = MemoryBuffer.fromByteBuffer(java.nio.ByteBuffer.allocateDirect(cap));
      out.add(b);
      addrs[w] = b.getUnsafeAddress();
      caps[w] = b.size();
    }
    long[] bytes = new long[windows];
    nEncodeWindows(hostCtx, cols, numRows, frame, addrs, caps, bytes);
    List<MemoryBuffer> used = new ArrayList<>(windows);
    for (int w = 0; w < windows; w++) {
      if (bytes[w] > 0 || w == 0) {
        out.get(w).writerIndex((int) bytes[w]);
        used.add(out.get(w));
      }
    }
    return used;
  }

  /**
   * N x encode(T) -> byte[] (FORY_FRAME_HASHED): one [i64 hash][row] array per object,
   * cut from one device batch at the row offsets the device computed.
   */
  public byte[][] encodeEach(ColumnBatch columns, int numRows) {
    long[] cols = columns.addresses();
    long need =
        rowSize >= 0 ? (long) numRows * (rowSize + 8) : nEncodedBytes(hostCtx, cols, numRows, FRAME_HASHED);
    if (need > Integer.MAX_VALUE) {
      throw new IndexOutOfBoundsException("encodeEach batch of " + need + " bytes: split the batch");
    }
    java.nio.ByteBuffer buf = java.nio.ByteBuffer.allocateDirect((int) Math.max(need, 1));
    MemoryBuffer mb = MemoryBuffer.fromByteBuffer(buf);
    long[] offsets = new long[numRows + 1];
    nEncodeVar(hostCtx, cols, numRows, FRAME_HASHED, mb.getUnsafeAddress(), mb.size(), offsets);
    byte[][] each = new byte[numRows][];
    for (int i = 0; i < numRows; i++) {
      each[i] = new byte[(int) (offsets[i + 1] - offsets[i])];
      mb.get((int) offsets[i], each[i], 0, each[i].length);
    }
    return each;
  }

  /**
   * N x decode(MemoryBuffer) from the frames alone (an RPC receiver has no offsets): the
   * frame starts are found on the device; {@code out} is sized and filled. Advances the
   * buffer's readerIndex past the N frames. ClassNotCompatibleException on a schema-hash
   * mismatch (Encoders.java:182-190).
   */
  public void decode(MemoryBuffer in, int numRows, ColumnBatch out) {
    if (!in.isOffHeap()) { // a heap buffer has no native address: staged through a direct buffer
      int len = in.remaining();
      ByteBuffer tmp = scratch(len);
      in.copyToUnsafe(in.readerIndex(), null, ColumnBatch.baseAddress(tmp), len);
      tmp.limit(len);
      MemoryBuffer staged = MemoryBuffer.fromByteBuffer(tmp);
      decode(staged, numRows, out);
      in.readerIndex(in.readerIndex() + staged.readerIndex());
      return;
    }
    long addr = in.getUnsafeAddress() + in.readerIndex();
    long consumed;
    if (rowSize >= 0) { // fixed width: every frame is rowSize + 12 bytes
      consumed = (long) numRows * (rowSize + 12);
      nDecodeFixed(hostCtx, addr, in.remaining(), numRows, FRAME_STREAM, out);
    } else {
      consumed = nDecodeStream(hostCtx, addr, in.remaining(), numRows, out);
    }
    in.readerIndex(in.readerIndex() + (int) consumed);
  }

  /**
   * N x decode(MemoryBuffer) when the sender's frame offsets travel with the stream: one
   * pipelined call into the receiver's reused columns (grown when a batch does not fit).
   */
  public void decodeInto(MemoryBuffer in, long[] frameOffsets, int numRows, ColumnBatch out) {
    nDecodeInto(hostCtx, in.getUnsafeAddress(), frameOffsets, numRows, FRAME_STREAM, out);
  }

  /** Pins a long-lived off-heap buffer (its copies become direct DMAs). */
  public static void register(MemoryBuffer buffer) {
    nRegister(buffer.getUnsafeAddress(), buffer.size());
  }

  public static void unregister(MemoryBuffer buffer) {
    nUnregister(buffer.getUnsafeAddress());
  }

  @Override
  public void close() {
    nHostCtxDestroy(hostCtx);
    nPlanDestroy(plan);
  }

  private static native long nPlanCreate(int[] desc);

  private static native void nPlanDestroy(long plan);

  private static native long nSchemaHash(long plan);

  private static native int nRowSize(long plan);

  private static native long nHostCtxCreate(long plan, int device, long chunkRows);

  private static native void nHostCtxDestroy(long ctx);

  private static native long nEncodedBytes(long ctx, long[] cols, int n, int frame);

  private static native long[] nWindowBytes(long ctx, long[] cols, int n, int frame, long maxWindow);

  private static native void nEncodeWindows(
      long ctx, long[] cols, int n, int frame, long[] addrs, long[] caps, long[] bytes);

  private static native long nEncodeVar(
      long ctx, long[] cols, int n, int frame, long outAddr, long outCap, long[] rowOffsets);

  private static native long nDecodeStream(long ctx, long inAddr, long inLen, int n, ColumnBatch out);

  private static native void nDecodeFixed(long ctx, long inAddr, long inLen, int n, int frame, ColumnBatch out);

  private static native void nDecodeInto(long ctx, long inAddr, long[] offs, int n, int frame, ColumnBatch out);

  private static native void nRegister(long addr, long bytes);

  private static native void nUnregister(long addr);
}
