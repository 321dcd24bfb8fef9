/*
 * MI355X row-format batch path: the schema a BatchRowEncoder hands to
 * fory_rowfmt_plan_create (include/fory_rowfmt.h, fory_field_desc).
 */
package org.apache.fory.format.encoder;

import java.util.List;
import org.apache.arrow.vector.types.pojo.Field;
import org.apache.arrow.vector.types.pojo.Schema;
import org.apache.fory.format.type.DataTypes;

/**
 * Flattens an inferred row schema into the pre-order {@code fory_field_desc[]} the C-ABI
 * takes: four ints per node, {@code {typeId, nullable, numChildren, reserved}}. The schema comes
 * from {@code TypeInference.inferSchema(beanClass)} (TypeInference.java:58-80), so the
 * field order (Descriptor order, names sorted) and the schema hash
 * (DataTypes.computeSchemaHash, DataTypes.java:499-544) are the reference's own.
 */
public final class DeviceSchemas {
  private DeviceSchemas() {}

  /** include/fory_rowfmt.h: reserved word of a decimal node that is a java.math.BigInteger field. */
  static final int FORY_DECIMAL_BIGINTEGER = 0x100;

  /** Pre-order {typeId, nullable, numChildren, 0} of every field node. */
  public static int[] flatten(Schema schema) {
    return flatten(schema, null);
  }

  /**
   * Pre-order {typeId, nullable, numChildren, reserved} of every field node; reserved is
   * FORY_DECIMAL_BIGINTEGER for the columns {@code bigInteger} marks (decimal(38, 0) nodes of
   * BigInteger fields, which the codec writes as toByteArray(), BaseBinaryEncoderBuilder.java:192-194,
   * not with writeDecimal), else 0 (a decimal's precision 0 = 38). The Arrow schema alone
   * cannot tell a BigInteger from a BigDecimal of scale 0: the bean class does
   * (BeanColumns.bigIntegerColumns).
   */
  public static int[] flatten(Schema schema, boolean[] bigInteger) {
    int nodes = 0;
    for (Field f : schema.getFields()) {
      nodes += count(f);
    }
    int[] out = new int[4 * nodes];
    int at = 0;
    for (Field f : schema.getFields()) {
      at = visit(f, out, at);
    }
    if (bigInteger != null) {
      for (int i = 0; i < nodes && i < bigInteger.length; i++) {
        if (bigInteger[i]) out[4 * i + 3] = FORY_DECIMAL_BIGINTEGER;
      }
    }
    return out;
  }

  /** Number of pre-order nodes (= columns of a ColumnBatch) of the schema. */
  public static int columns(Schema schema) {
    int nodes = 0;
    for (Field f : schema.getFields()) {
      nodes += count(f);
    }
    return nodes;
  }

  /**
   * Children as the C-ABI numbers them: a map's entries struct is elided (key, value are
   * the map node's two children), as the schema hash elides it (DataTypes.java:522-527).
   */
  static List<Field> deviceChildren(Field f) {
    List<Field> children = f.getChildren();
    if (DataTypes.getTypeIdValue(f.getType()) == ColumnBatch.ArrowTypeIds.MAP && children.size() == 1) {
      return children.get(0).getChildren(); // entries: {key, value}
    }
    return children;
  }

  private static int count(Field f) {
    int n = 1;
    for (Field c : deviceChildren(f)) {
      n += count(c);
    }
    return n;
  }

  private static int visit(Field f, int[] out, int at) {
    List<Field> children = deviceChildren(f);
    // ArrowType ordinal, the id the schema hash folds in (DataTypes.java:233-235, 510-530)
    out[at] = DataTypes.getTypeIdValue(f.getType());
    out[at + 1] = f.isNullable() ? 1 : 0;
    out[at + 2] = children.size(); // list: 1 ("item"), map: 2 (key, value), struct: n
    out[at + 3] = 0;
    at += 4;
    for (Field c : children) {
      at = visit(c, out, at);
    }
    return at;
  }
}
