/*
 * MI355X row-format batch path: off-heap Arrow-layout columns of one batch.
 */
package org.apache.fory.format.encoder;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import org.apache.arrow.vector.types.pojo.Field;
import org.apache.arrow.vector.types.pojo.Schema;
import org.apache.fory.format.type.DataTypes;
import org.apache.fory.memory.MemoryBuffer;

/**
 * The columns of a batch of N beans in Arrow layout, one per pre-order schema node (the
 * columnar view vectorized/ArrowWriter.java:55-99 builds): fixed-width values, int32
 * offsets for strings / binary / lists / maps, validity bitmaps (1 = valid) for nullable
 * nodes. Buffers are direct (off-heap) so their addresses can cross JNI and be pinned
 * once (BatchRowEncoder.register). A receiver keeps one ColumnBatch across batches: the
 * JNI shim calls {@link #allocate} when a batch needs more room.
 */
public final class ColumnBatch {
  static final int FIELDS_PER_COLUMN = 5; // values, offsets, validity, length, value capacity

  private final int[] typeIds;
  private final int[] widths; // fixed width in bytes, or -1 (string/binary/list/map/struct)
  private final boolean[] nullable;
  private final ByteBuffer[] values;
  private final ByteBuffer[] offsets;
  private final ByteBuffer[] validity;
  private final long[] length;

  public ColumnBatch(Schema schema) {
    int n = DeviceSchemas.columns(schema);
    typeIds = new int[n];
    widths = new int[n];
    nullable = new boolean[n];
    values = new ByteBuffer[n];
    offsets = new ByteBuffer[n];
    validity = new ByteBuffer[n];
    length = new long[n];
    int at = 0;
    for (Field f : schema.getFields()) {
      at = describe(f, at);
    }
  }

  private int describe(Field f, int at) {
    typeIds[at] = DataTypes.getTypeIdValue(f.getType());
    widths[at] = DataTypes.getTypeWidth(f.getType()); // DataTypes.java:225-227 (-1: variable)
    nullable[at] = f.isNullable();
    at++;
    for (Field c : DeviceSchemas.deviceChildren(f)) {
      at = describe(c, at);
    }
    return at;
  }

  public int numColumns() {
    return typeIds.length;
  }

  private boolean hasOffsets(int i) {
    // utf8 / binary / list / map (ArrowType ordinals of DataTypes.getTypeIdValue)
    int t = typeIds[i];
    return t == ArrowTypeIds.UTF8 || t == ArrowTypeIds.BINARY || t == ArrowTypeIds.LIST || t == ArrowTypeIds.MAP;
  }

  private boolean hasValues(int i) {
    // decimal: Arrow decimal128, 16 bytes per value (getTypeWidth says -1: 32 bytes out of line in a row)
    return widths[i] > 0 || typeIds[i] == ArrowTypeIds.UTF8 || typeIds[i] == ArrowTypeIds.BINARY
        || typeIds[i] == ArrowTypeIds.DECIMAL;
  }

  /**
   * Sizes the columns for per-column element counts and value bytes (string/binary
   * columns: payload bytes), growing any buffer that is too small; lengths become the
   * counts. Called by the JNI shim after a sizes pass (fory_rowfmt_host_decode_*).
   */
  public void allocate(long[] counts, long[] bytes) {
    for (int i = 0; i < typeIds.length; i++) {
      long k = counts[i];
      if (hasValues(i)) {
        long need = widths[i] > 0 ? k * widths[i] : typeIds[i] == ArrowTypeIds.DECIMAL ? 16 * k : bytes[i];
        values[i] = grow(values[i], need);
      }
      if (hasOffsets(i)) {
        offsets[i] = grow(offsets[i], 4 * (k + 1));
      }
      if (nullable[i]) {
        validity[i] = grow(validity[i], ((k + 7) / 8 + 3) / 4 * 4);
      }
      length[i] = k;
    }
  }

  private static ByteBuffer grow(ByteBuffer b, long need) {
    if (need > Integer.MAX_VALUE) {
      throw new IndexOutOfBoundsException("column of " + need + " bytes exceeds a direct buffer");
    }
    if (b != null && b.capacity() >= need) {
      return b;
    }
    return ByteBuffer.allocateDirect((int) Math.max(need, 16)).order(ByteOrder.LITTLE_ENDIAN);
  }

  /**
   * Column i's buffers and slot count, as BeanColumns built them from beans (direct,
   * little-endian; validity with at least 4 bytes of slack past its last bit, the device
   * path reads whole dwords). Buffers a column does not use are dropped.
   */
  void set(int i, ByteBuffer v, ByteBuffer o, ByteBuffer valid, long len) {
    values[i] = hasValues(i) ? v : null;
    offsets[i] = hasOffsets(i) ? o : null;
    validity[i] = nullable[i] ? valid : null;
    length[i] = len;
  }

  /** Per column {values, offsets, validity, length, value capacity}: native addresses (0 = none). */
  public long[] addresses() {
    long[] a = new long[FIELDS_PER_COLUMN * typeIds.length];
    for (int i = 0; i < typeIds.length; i++) {
      a[FIELDS_PER_COLUMN * i] = address(values[i]);
      a[FIELDS_PER_COLUMN * i + 1] = address(offsets[i]);
      a[FIELDS_PER_COLUMN * i + 2] = address(validity[i]);
      a[FIELDS_PER_COLUMN * i + 3] = length[i];
      a[FIELDS_PER_COLUMN * i + 4] = values[i] == null ? 0 : values[i].capacity();
    }
    return a;
  }

  private static long address(ByteBuffer b) {
    return b == null ? 0 : baseAddress(b);
  }

  /**
   * The native address of a direct buffer's byte 0, whatever its position: {@code
   * MemoryBuffer.fromByteBuffer(b).getUnsafeAddress()} adds {@code b.position()}
   * (MemoryBuffer.java:2639-2640), and buffers that were just written hold their position
   * at the end of the data.
   */
  static long baseAddress(ByteBuffer b) {
    ByteBuffer at0 = b.duplicate();
    at0.clear(); // position 0 (a duplicate: b's own position and limit are kept)
    return MemoryBuffer.fromByteBuffer(at0).getUnsafeAddress(); // MemoryBuffer.java:295
  }

  /** The direct buffer of column i's values (null for struct / list / map nodes). */
  public ByteBuffer values(int i) {
    return values[i];
  }

  public ByteBuffer offsets(int i) {
    return offsets[i];
  }

  public ByteBuffer validity(int i) {
    return validity[i];
  }

  public long length(int i) {
    return length[i];
  }

  /** ArrowType ordinals (org.apache.fory.format.type.ArrowType, ArrowType.java:25-160). */
  static final class ArrowTypeIds {
    static final int UTF8 = 13;
    static final int BINARY = 14;
    static final int LIST = 25;
    static final int MAP = 30;
    static final int DECIMAL = 23;
  }
}
