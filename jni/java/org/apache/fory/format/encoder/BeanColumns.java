/*
 * MI355X row-format batch path: beans <-> the Arrow-layout columns of a ColumnBatch.
 */
package org.apache.fory.format.encoder;

import java.lang.reflect.Array;
import java.math.BigDecimal;
import java.math.BigInteger;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.Collection;
import java.util.HashMap;
import java.util.HashSet;
import java.util.LinkedHashMap;
import java.util.List;
import java.util.Map;
import java.util.Optional;
import java.util.Set;
import org.apache.arrow.vector.types.pojo.ArrowType;
import org.apache.arrow.vector.types.pojo.Field;
import org.apache.arrow.vector.types.pojo.Schema;
import org.apache.fory.collection.Tuple2;
import org.apache.fory.memory.Platform;
import org.apache.fory.reflect.FieldAccessor;
import org.apache.fory.reflect.TypeRef;
import org.apache.fory.type.Descriptor;
import org.apache.fory.type.TypeUtils;
import org.apache.fory.util.DateTimeUtils;
import org.apache.fory.util.Preconditions;

/**
 * The bean side of {@link BatchRowEncoder}: N objects of a bean class as the columns the
 * device encodes (one per pre-order node of {@code TypeInference.inferSchema(beanClass)},
 * the layout {@link ColumnBatch} holds), and the columns the device decodes back as N
 * objects. The per-field value conversions are the generated codec's
 * (BaseBinaryEncoderBuilder.serializeFor, :149-271, and deserializeFor, :540-600):
 *
 * <ul>
 *   <li>primitives and boxed values as themselves; a null boxed value is a null slot
 *       (setNullAt);
 *   <li>{@code BigDecimal} as Arrow decimal128: its unscaled value at the field's scale
 *       (DecimalUtils.MAX_SCALE); another scale is an UnsupportedOperationException, as
 *       DecimalUtility.checkPrecisionAndScale throws in BinaryWriter.writeDecimal
 *       (BinaryWriter.java:214-225);
 *   <li>{@code BigInteger} as decimal128 at scale 0 (TypeInference.java:203-204), its column
 *       flagged FORY_DECIMAL_BIGINTEGER in the plan ({@link #bigIntegerColumns}), so the device
 *       writes {@code toByteArray()} into the row (BaseBinaryEncoderBuilder.java:192-194) and
 *       reads it back as {@code new BigInteger(bytes)} (:559-560); a value beyond 128 bits has
 *       no decimal128 column value (UnsupportedOperationException);
 *   <li>{@code LocalDate} / {@code java.sql.Date} as days ({@code
 *       DateTimeUtils.localDateToDays / fromJavaDate}), {@code Timestamp} / {@code Instant} as
 *       microseconds ({@code fromJavaTimestamp / instantToMicros}), enums by {@code name()},
 *       Strings as UTF-8, {@code Optional} unwrapped (:195-230, :171-181);
 *   <li>arrays and Iterables as lists, Maps as maps, beans as structs (:231-271).
 * </ul>
 *
 * Decoded collections are ArrayList / HashSet / HashMap (LinkedHashMap for a declared
 * LinkedHashMap), arrays of the declared component type, beans built by {@code
 * Platform.newInstance} and filled through {@code FieldAccessor}, as fory-core does.
 */
final class BeanColumns<T> {
  static final int FIXED = 0;
  static final int BOOL = 1;
  static final int STRING = 2;
  static final int BINARY = 3;
  static final int DECIMAL = 4;
  static final int BIGINT = 5;
  static final int LIST = 6;
  static final int MAP = 7;
  static final int STRUCT = 8;

  // value conversions of FIXED / STRING nodes
  static final int AS_IS = 0;
  static final int LOCAL_DATE = 1;
  static final int SQL_DATE = 2;
  static final int TIMESTAMP = 3;
  static final int INSTANT = 4;
  static final int ENUM = 5;
  static final int CHAR = 6;

  /** One pre-order schema node (= one ColumnBatch column) with its Java type. */
  static final class Node {
    int column;
    int kind;
    int width; // FIXED: 1/2/4/8
    int conv;
    int scale; // DECIMAL
    boolean nullable;
    boolean optional; // the Java value is an Optional of this type
    Class<?> raw; // declared type (decode: what to build)
    FieldAccessor accessor; // a bean's field (children of STRUCT nodes)
    Node[] children = new Node[0];
  }

  private final Class<T> beanClass;
  private final Node[] top;
  private final int numColumns;

  BeanColumns(Class<T> beanClass, Schema schema) {
    this.beanClass = beanClass;
    int[] next = {0};
    this.top = beanFields(beanClass, schema.getFields(), next);
    this.numColumns = next[0];
    Preconditions.checkArgument(numColumns == DeviceSchemas.columns(schema), "bean / schema node count differ");
  }

  int numColumns() {
    return numColumns;
  }

  /** Per pre-order column: a BigInteger field (DeviceSchemas.flatten flags its descriptor). */
  boolean[] bigIntegerColumns() {
    boolean[] out = new boolean[numColumns];
    for (Node f : top) markBigInteger(f, out);
    return out;
  }

  private static void markBigInteger(Node f, boolean[] out) {
    if (f.kind == BIGINT) out[f.column] = true;
    for (Node c : f.children) markBigInteger(c, out);
  }

  // ---------------------------------------------------------------- schema walk
  private static Node[] beanFields(Class<?> cls, List<Field> fields, int[] next) {
    List<Descriptor> ds = Descriptor.getDescriptors(cls); // TypeInference.java:238-247 order
    Preconditions.checkArgument(ds.size() == fields.size(), "descriptors / schema fields differ for " + cls);
    Node[] out = new Node[fields.size()];
    for (int k = 0; k < out.length; k++) {
      Descriptor d = ds.get(k);
      out[k] = node(d.getTypeRef(), fields.get(k), next);
      java.lang.reflect.Field jf = d.getField();
      Preconditions.checkArgument(jf != null, "bean field without a java.lang.reflect.Field: " + d.getName());
      out[k].accessor = FieldAccessor.createAccessor(jf);
    }
    return out;
  }

  private static Node node(TypeRef<?> type, Field f, int[] next) {
    Node n = new Node();
    n.column = next[0]++;
    n.nullable = f.isNullable();
    Class<?> raw = type.getRawType();
    if (raw == Optional.class) {
      n.optional = true;
      type = TypeUtils.getTypeArguments(type).get(0);
      raw = type.getRawType();
    }
    n.raw = raw;
    ArrowType at = f.getType();
    if (raw.isEnum()) {
      n.kind = STRING;
      n.conv = ENUM;
    } else if (at instanceof ArrowType.Utf8) {
      n.kind = STRING;
    } else if (at instanceof ArrowType.Binary) {
      n.kind = BINARY;
    } else if (at instanceof ArrowType.Decimal) {
      n.kind = raw == BigInteger.class ? BIGINT : DECIMAL;
      n.scale = ((ArrowType.Decimal) at).getScale();
    } else if (at instanceof ArrowType.Bool) {
      n.kind = BOOL;
      n.width = 1;
    } else if (at instanceof ArrowType.Struct) {
      n.kind = STRUCT;
      n.children = beanFields(raw, f.getChildren(), next);
    } else if (at instanceof ArrowType.List) {
      n.kind = LIST;
      TypeRef<?> elem = raw.isArray() ? TypeRef.of(raw.getComponentType()) : TypeUtils.getElementType(type);
      n.children = new Node[] {node(elem, f.getChildren().get(0), next)};
    } else if (at instanceof ArrowType.Map) {
      n.kind = MAP;
      Tuple2<TypeRef<?>, TypeRef<?>> kv = TypeUtils.getMapKeyValueType(type);
      List<Field> entries = DeviceSchemas.deviceChildren(f); // key, value (entries struct elided)
      Node key = node(kv.f0, entries.get(0), next);
      Node value = node(kv.f1, entries.get(1), next);
      n.children = new Node[] {key, value};
    } else {
      n.kind = FIXED;
      n.width = org.apache.fory.format.type.DataTypes.getTypeWidth(at); // DataTypes.java:225-227
      if (raw == java.time.LocalDate.class) n.conv = LOCAL_DATE;
      else if (raw == java.sql.Date.class) n.conv = SQL_DATE;
      else if (raw == java.sql.Timestamp.class) n.conv = TIMESTAMP;
      else if (raw == java.time.Instant.class) n.conv = INSTANT;
      else if (raw == char.class || raw == Character.class) n.conv = CHAR;
    }
    return n;
  }

  // ---------------------------------------------------------------- beans -> columns
  /** Growable little-endian direct buffers of one column. */
  private static final class Col {
    ByteBuffer values = alloc(64);
    ByteBuffer offsets = alloc(64);
    ByteBuffer validity = alloc(64);
    long length; // slots appended
    int items; // list / map: items so far (its offsets' running value)

    Col() {
      offsets.putInt(0);
    }

    static ByteBuffer alloc(int cap) {
      return ByteBuffer.allocateDirect(cap).order(ByteOrder.LITTLE_ENDIAN);
    }

    static ByteBuffer room(ByteBuffer b, int more) {
      if (b.remaining() >= more) return b;
      long need = (long) b.position() + more;
      if (need > Integer.MAX_VALUE - 16) {
        throw new IndexOutOfBoundsException("column of " + need + " bytes exceeds a direct buffer");
      }
      ByteBuffer g = alloc((int) Math.min(Integer.MAX_VALUE - 16, Math.max(need, 2L * b.capacity())));
      b.flip();
      g.put(b);
      return g;
    }

    void bit(boolean valid) {
      int byteIndex = (int) (length >>> 3);
      if (byteIndex >= validity.position()) {
        validity = room(validity, 1);
        validity.put((byte) 0);
      }
      if (valid) validity.put(byteIndex, (byte) (validity.get(byteIndex) | (1 << (length & 7))));
    }

    void fixed(int width, long v) {
      values = room(values, 8);
      switch (width) {
        case 8: values.putLong(v); break;
        case 4: values.putInt((int) v); break;
        case 2: values.putShort((short) v); break;
        default: values.put((byte) v); break;
      }
    }

    void bytes(byte[] b) {
      values = room(values, b.length);
      values.put(b);
      offsets = room(offsets, 4);
      offsets.putInt(values.position());
    }

    void count(int n) {
      items += n;
      offsets = room(offsets, 4);
      offsets.putInt(items);
    }
  }

  /** The columns of {@code beans}, in {@code out} (its buffers replaced). */
  void fill(List<T> beans, ColumnBatch out) {
    Col[] cols = new Col[numColumns];
    for (int i = 0; i < numColumns; i++) cols[i] = new Col();
    for (T bean : beans) {
      Preconditions.checkNotNull(bean, "a null bean in the batch");
      for (Node f : top) put(cols, f, f.accessor.get(bean), true);
    }
    for (int i = 0; i < numColumns; i++) {
      Col c = cols[i];
      // slack past the data: the device path reads whole dwords of validity and offsets
      c.validity = Col.room(c.validity, 8);
      c.offsets = Col.room(c.offsets, 8);
      c.values = Col.room(c.values, 16);
      // (ColumnBatch takes each buffer's byte 0 as the column start: their positions are
      // past the data here)
      out.set(i, c.values, c.offsets, c.validity, c.length);
    }
  }

  private void put(Col[] cols, Node f, Object v, boolean present) {
    if (f.optional && v != null) v = ((Optional<?>) v).orElse(null);
    Col c = cols[f.column];
    boolean valid = present && v != null;
    if (f.nullable) c.bit(valid);
    switch (f.kind) {
      case FIXED:
      case BOOL:
        c.fixed(f.width, valid ? fixedBits(f, v) : 0);
        break;
      case STRING:
        c.bytes(valid ? (f.conv == ENUM ? ((Enum<?>) v).name() : (String) v).getBytes(StandardCharsets.UTF_8)
                      : new byte[0]);
        break;
      case BINARY:
        c.bytes(valid ? (byte[]) v : new byte[0]);
        break;
      case DECIMAL:
      case BIGINT:
        putDecimal(c, f, valid ? v : null);
        break;
      case STRUCT:
        for (Node ch : f.children) put(cols, ch, valid ? ch.accessor.get(v) : null, valid);
        break;
      case LIST: {
        int n = 0;
        if (valid) {
          if (v.getClass().isArray()) {
            n = Array.getLength(v);
            for (int j = 0; j < n; j++) put(cols, f.children[0], Array.get(v, j), true);
          } else {
            for (Object e : (Iterable<?>) v) {
              put(cols, f.children[0], e, true);
              n++;
            }
          }
        }
        c.count(n);
        break;
      }
      case MAP: {
        int n = 0;
        if (valid) {
          for (Map.Entry<?, ?> e : ((Map<?, ?>) v).entrySet()) {
            put(cols, f.children[0], e.getKey(), true);
            put(cols, f.children[1], e.getValue(), true);
            n++;
          }
        }
        c.count(n);
        break;
      }
      default:
        throw new IllegalStateException("node kind " + f.kind);
    }
    c.length++;
  }

  private static long fixedBits(Node f, Object v) {
    switch (f.conv) {
      case LOCAL_DATE: return DateTimeUtils.localDateToDays((java.time.LocalDate) v);
      case SQL_DATE: return DateTimeUtils.fromJavaDate((java.sql.Date) v);
      case TIMESTAMP: return DateTimeUtils.fromJavaTimestamp((java.sql.Timestamp) v);
      case INSTANT: return DateTimeUtils.instantToMicros((java.time.Instant) v);
      case CHAR: return (Character) v;
      default: break;
    }
    if (v instanceof Boolean) return ((Boolean) v) ? 1 : 0;
    if (v instanceof Float) return Float.floatToRawIntBits((Float) v) & 0xffffffffL;
    if (v instanceof Double) return Double.doubleToRawLongBits((Double) v);
    return ((Number) v).longValue();
  }

  /** decimal128: the unscaled value, 16 bytes little-endian two's complement. */
  private static void putDecimal(Col c, Node f, Object v) {
    BigInteger u = BigInteger.ZERO;
    if (v != null) {
      if (f.kind == BIGINT) {
        u = (BigInteger) v;
      } else {
        BigDecimal d = (BigDecimal) v;
        if (d.scale() != f.scale) { // DecimalUtility.checkPrecisionAndScale
          throw new UnsupportedOperationException(
              "BigDecimal scale must equal that in the Arrow vector: " + d.scale() + " != " + f.scale);
        }
        u = d.unscaledValue();
      }
      if (u.bitLength() > 127) {
        throw new UnsupportedOperationException("decimal value does not fit decimal128: " + v);
      }
    }
    byte[] be = u.toByteArray(); // big-endian, minimal
    byte[] le = new byte[16];
    byte ext = (byte) (u.signum() < 0 ? 0xff : 0);
    for (int k = 0; k < 16; k++) le[k] = k < be.length ? be[be.length - 1 - k] : ext;
    c.values = Col.room(c.values, 16);
    c.values.put(le);
  }

  // ---------------------------------------------------------------- columns -> beans
  /** N beans from the columns of {@code in} (as the device decoded them). */
  List<T> read(ColumnBatch in, int n) {
    List<T> out = new ArrayList<>(n);
    for (int i = 0; i < n; i++) {
      T bean = Platform.newInstance(beanClass);
      for (Node f : top) f.accessor.set(bean, get(in, f, i));
      out.add(bean);
    }
    return out;
  }

  private static boolean valid(ColumnBatch in, Node f, long i) {
    if (!f.nullable) return true;
    ByteBuffer v = in.validity(f.column);
    return v == null || ((v.get((int) (i >>> 3)) >>> (i & 7)) & 1) != 0;
  }

  private Object get(ColumnBatch in, Node f, long i) {
    Object v = valid(in, f, i) ? value(in, f, i) : null;
    return f.optional ? Optional.ofNullable(v) : v;
  }

  private Object value(ColumnBatch in, Node f, long i) {
    ByteBuffer vals = in.values(f.column);
    switch (f.kind) {
      case BOOL:
        return vals.get((int) i) != 0;
      case FIXED:
        return boxFixed(f, vals, (int) i);
      case STRING: {
        String s = new String(slice(in, f, i), StandardCharsets.UTF_8);
        return f.conv == ENUM ? enumOf(f.raw, s) : s;
      }
      case BINARY:
        return slice(in, f, i);
      case DECIMAL:
      case BIGINT: {
        byte[] be = new byte[16];
        for (int k = 0; k < 16; k++) be[15 - k] = vals.get((int) (16 * i + k));
        BigInteger u = new BigInteger(be);
        return f.kind == BIGINT ? u : new BigDecimal(u, f.scale);
      }
      case STRUCT: {
        Object bean = Platform.newInstance(f.raw);
        for (Node ch : f.children) ch.accessor.set(bean, get(in, ch, i));
        return bean;
      }
      case LIST: {
        ByteBuffer off = in.offsets(f.column);
        int a = off.getInt((int) (4 * i)), b = off.getInt((int) (4 * i + 4));
        Node it = f.children[0];
        if (f.raw.isArray()) {
          Object arr = Array.newInstance(f.raw.getComponentType(), b - a);
          for (int j = a; j < b; j++) Array.set(arr, j - a, get(in, it, j));
          return arr;
        }
        Collection<Object> coll = Set.class.isAssignableFrom(f.raw) ? new HashSet<>() : new ArrayList<>(b - a);
        for (int j = a; j < b; j++) coll.add(get(in, it, j));
        return coll;
      }
      case MAP: {
        ByteBuffer off = in.offsets(f.column);
        int a = off.getInt((int) (4 * i)), b = off.getInt((int) (4 * i + 4));
        Map<Object, Object> m = LinkedHashMap.class.isAssignableFrom(f.raw) ? new LinkedHashMap<>() : new HashMap<>();
        for (int j = a; j < b; j++) m.put(get(in, f.children[0], j), get(in, f.children[1], j));
        return m;
      }
      default:
        throw new IllegalStateException("node kind " + f.kind);
    }
  }

  private static byte[] slice(ColumnBatch in, Node f, long i) {
    ByteBuffer off = in.offsets(f.column);
    int a = off.getInt((int) (4 * i)), b = off.getInt((int) (4 * i + 4));
    byte[] out = new byte[b - a];
    ByteBuffer v = in.values(f.column).duplicate();
    v.position(a);
    v.get(out);
    return out;
  }

  @SuppressWarnings({"unchecked", "rawtypes"})
  private static Object enumOf(Class<?> cls, String name) {
    return Enum.valueOf((Class) cls, name);
  }

  private static Object boxFixed(Node f, ByteBuffer v, int i) {
    switch (f.conv) {
      case LOCAL_DATE: return DateTimeUtils.daysToLocalDate(v.getInt(4 * i));
      case SQL_DATE: return DateTimeUtils.toJavaDate(v.getInt(4 * i));
      case TIMESTAMP: return DateTimeUtils.toJavaTimestamp(v.getLong(8 * i));
      case INSTANT: return DateTimeUtils.microsToInstant(v.getLong(8 * i));
      case CHAR: return (char) v.getShort(2 * i);
      default: break;
    }
    Class<?> r = f.raw;
    if (r == int.class || r == Integer.class) return v.getInt(4 * i);
    if (r == long.class || r == Long.class) return v.getLong(8 * i);
    if (r == double.class || r == Double.class) return v.getDouble(8 * i);
    if (r == float.class || r == Float.class) return v.getFloat(4 * i);
    if (r == short.class || r == Short.class) return v.getShort(2 * i);
    if (r == byte.class || r == Byte.class) return v.get(i);
    throw new UnsupportedOperationException("fixed-width field of type " + r);
  }
}
