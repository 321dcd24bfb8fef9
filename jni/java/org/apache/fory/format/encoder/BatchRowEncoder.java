/*
 * MI355X row-format batch path: the batched RowEncoder / Encoder of one bean class,
 * over libfory_rowfmt.so (include/fory_rowfmt.h) through jni/fory_rowfmt_jni.c.
 */
package org.apache.fory.format.encoder;

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
    this.plan = nPlanCreate(DeviceSchemas.flatten(schema)); // EncoderException / UnsupportedOperation
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
    long need =
        rowSize >= 0
            ? (long) numRows * (rowSize + (frame == FRAME_STREAM ? 12 : frame == FRAME_HASHED ? 8 : 0))
            : nEncodedBytes(hostCtx, cols, numRows, frame); // a sizing pass on the device
    int windows = (int) Math.max(1, (need + Integer.MAX_VALUE - 1) / Integer.MAX_VALUE + 1);
    List<MemoryBuffer> out = new ArrayList<>(windows);
    long[] addrs = new long[windows];
    long[] caps = new long[windows];
    for (int w = 0; w < windows; w++) {
      int cap = (int) Math.min(Integer.MAX_VALUE, Math.max(need, 1));
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
