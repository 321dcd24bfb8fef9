"""Schema types — a Python mirror of the reference's row-format type layer.

Mirrors (reference paths relative to java/fory-format/src/main/java/org/apache/fory/format):
  ArrowType ids                         type/ArrowType.java:25-160
  DataTypes.getTypeWidth                type/DataTypes.java:68-133,225-227
  DataTypes.arrayField / structField    type/DataTypes.java:360-379
  DataTypes.computeSchemaHash           type/DataTypes.java:499-544 (computed by the
                                        native plan, fory_rowfmt_plan_info)
Arrow-Java's pojo ``Field``/``Schema`` are used by the reference as pure
metadata; ``Field``/``Schema`` here carry exactly that metadata (name, type,
nullable, children) and flatten it into the C-ABI's pre-order
``fory_field_desc`` array.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field as dc_field
from typing import List, Optional, Sequence


class ArrowType:
    """Ordinals of org.apache.fory.format.type.ArrowType (ArrowType.java:25-160)."""
    NA = 0
    BOOL = 1
    UINT8 = 2
    INT8 = 3
    UINT16 = 4
    INT16 = 5
    UINT32 = 6
    INT32 = 7
    UINT64 = 8
    INT64 = 9
    HALF_FLOAT = 10
    FLOAT = 11
    DOUBLE = 12
    STRING = 13
    BINARY = 14
    FIXED_SIZE_BINARY = 15
    DATE32 = 16
    DATE64 = 17
    TIMESTAMP = 18
    TIME32 = 19
    TIME64 = 20
    INTERVAL_MONTHS = 21
    INTERVAL_DAY_TIME = 22
    DECIMAL128 = 23
    DECIMAL256 = 24
    LIST = 25
    STRUCT = 26
    SPARSE_UNION = 27
    DENSE_UNION = 28
    DICTIONARY = 29
    MAP = 30


_WIDTH = {
    ArrowType.BOOL: 1, ArrowType.INT8: 1, ArrowType.INT16: 2, ArrowType.INT32: 4,
    ArrowType.INT64: 8, ArrowType.FLOAT: 4, ArrowType.DOUBLE: 8, ArrowType.DATE32: 4,
    ArrowType.TIMESTAMP: 8,
}

_NAMES = {v: k.lower() for k, v in vars(ArrowType).items() if not k.startswith("_")}


@dataclass(frozen=True)
class DataType:
    id: int
    precision: int = 0  # DECIMAL128 only (Arrow Decimal(precision, scale)); neither enters the hash
    scale: int = 0
    # DECIMAL128 only: the bean field is java.math.BigInteger (Decimal(38, 0),
    # TypeInference.java:203-204), which the codec writes as toByteArray() bytes
    # (BaseBinaryEncoderBuilder.java:192-194), not with writeDecimal. Not in the hash.
    big_integer: bool = False

    @property
    def width(self) -> int:
        """DataTypes.getTypeWidth: byte width, -1 for variable-width types."""
        return _WIDTH.get(self.id, -1)

    @property
    def column_width(self) -> int:
        """Bytes per element of the Arrow column (decimal128: 16), -1 for var-length."""
        return 16 if self.id == ArrowType.DECIMAL128 else self.width

    def __repr__(self) -> str:
        if self.id == ArrowType.DECIMAL128:
            return "biginteger" if self.big_integer else f"decimal({self.precision}, {self.scale})"
        return _NAMES.get(self.id, str(self.id))


@dataclass
class Field:
    name: str
    type: DataType
    nullable: bool = True
    children: List["Field"] = dc_field(default_factory=list)

    def __repr__(self) -> str:
        kids = f", children={self.children}" if self.children else ""
        null = "" if self.nullable else " not null"
        return f"{self.name}: {self.type!r}{null}{kids}"


@dataclass
class Schema:
    fields: List[Field]

    def __len__(self) -> int:
        return len(self.fields)

    def __iter__(self):
        return iter(self.fields)

    def __getitem__(self, i) -> Field:
        return self.fields[i]

    def names(self) -> List[str]:
        return [f.name for f in self.fields]


class DataTypes:
    """Factory/helper mirror of type/DataTypes.java."""

    @staticmethod
    def bool_() -> DataType:
        return DataType(ArrowType.BOOL)

    @staticmethod
    def int8() -> DataType:
        return DataType(ArrowType.INT8)

    @staticmethod
    def int16() -> DataType:
        return DataType(ArrowType.INT16)

    @staticmethod
    def int32() -> DataType:
        return DataType(ArrowType.INT32)

    @staticmethod
    def int64() -> DataType:
        return DataType(ArrowType.INT64)

    @staticmethod
    def float32() -> DataType:
        return DataType(ArrowType.FLOAT)

    @staticmethod
    def float64() -> DataType:
        return DataType(ArrowType.DOUBLE)

    @staticmethod
    def utf8() -> DataType:
        return DataType(ArrowType.STRING)

    @staticmethod
    def binary() -> DataType:
        return DataType(ArrowType.BINARY)

    @staticmethod
    def date32() -> DataType:
        return DataType(ArrowType.DATE32)

    @staticmethod
    def timestamp() -> DataType:
        return DataType(ArrowType.TIMESTAMP)

    @staticmethod
    def decimal(precision: int = 38, scale: int = 18) -> DataType:
        """DataTypes.decimal (DataTypes.java:291-298): Decimal(MAX_PRECISION 38, MAX_SCALE 18)
        by default; DataTypes.bigintDecimal = decimal(38, 0)."""
        return DataType(ArrowType.DECIMAL128, precision, scale)

    @staticmethod
    def big_integer() -> DataType:
        """The type of a java.math.BigInteger bean field: DataTypes.bigintDecimal() =
        decimal(38, 0) (DataTypes.java:300-302, TypeInference.java:203-204), marked as a
        BigInteger so the row holds value.toByteArray() (BaseBinaryEncoderBuilder.java:192-194)."""
        return DataType(ArrowType.DECIMAL128, 38, 0, True)

    @staticmethod
    def field(name: str, type_: DataType, nullable: bool = True,
              children: Optional[Sequence[Field]] = None) -> Field:
        return Field(name, type_, nullable, list(children or []))

    @staticmethod
    def array_field(name: str, item: Field) -> Field:
        """DataTypes.arrayField (DataTypes.java:364-379): nullable list, child "item"."""
        item = Field("item", item.type, item.nullable, item.children)
        return Field(name, DataType(ArrowType.LIST), True, [item])

    @staticmethod
    def map_field(name: str, key: Field, value: Field) -> Field:
        """DataTypes.mapField (DataTypes.java:404-424): nullable map, key not nullable. The
        entries struct of Arrow's map type is elided: children are [key, value], the
        fields the schema hash visits (DataTypes.java:522-527)."""
        if key.nullable:
            from .errors import IllegalArgumentException
            raise IllegalArgumentException("Map's keys must be non-nullable")
        return Field(name, DataType(ArrowType.MAP), True,
                     [Field("key", key.type, False, key.children), Field("value", value.type, value.nullable,
                                                                          value.children)])

    @staticmethod
    def struct_field(name: str, nullable: bool, children: Sequence[Field]) -> Field:
        return Field(name, DataType(ArrowType.STRUCT), nullable, list(children))

    @staticmethod
    def schema(fields: Sequence[Field]) -> Schema:
        return Schema(list(fields))

    @staticmethod
    def get_type_width(type_: DataType) -> int:
        return type_.width

    @staticmethod
    def compute_schema_hash(schema: Schema) -> int:
        """DataTypes.computeSchemaHash, computed by the native layout planner."""
        from .native import NativePlan
        return NativePlan(schema).schema_hash

    @staticmethod
    def get_bitmap_bytes(num_fields: int) -> int:
        """BitUtils.calculateBitmapWidthInBytes (BitUtils.java:175-177)."""
        return ((num_fields + 63) // 64) * 8


def flatten(schema: Schema):
    """Pre-order ``fory_field_desc`` array for the C-ABI (and the oracle)."""
    from .._lib import FieldDesc
    out: List[tuple] = []

    def visit(f: Field):
        out.append((f.type.id, 1 if f.nullable else 0, len(f.children), desc_reserved(f.type)))
        for c in f.children:
            visit(c)

    for f in schema.fields:
        visit(f)
    arr = (FieldDesc * max(1, len(out)))()
    for i, (t, n, k, r) in enumerate(out):
        arr[i].type_id = t
        arr[i].nullable = n
        arr[i].num_children = k
        arr[i].reserved = r
    return arr, len(out)


FORY_DECIMAL_BIGINTEGER = 0x100  # include/fory_rowfmt.h


def desc_reserved(t: DataType) -> int:
    """fory_field_desc.reserved: a decimal's precision (0 = 38), FORY_DECIMAL_BIGINTEGER for
    a BigInteger field, else 0."""
    if t.id != ArrowType.DECIMAL128:
        return 0
    return FORY_DECIMAL_BIGINTEGER if t.big_integer else (t.precision or 38)


def preorder(schema: Schema) -> List[Field]:
    """Fields in the pre-order used for column indices."""
    out: List[Field] = []

    def visit(f: Field):
        out.append(f)
        for c in f.children:
            visit(c)

    for f in schema.fields:
        visit(f)
    return out
