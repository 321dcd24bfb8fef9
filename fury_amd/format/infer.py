"""TypeInference mirror: Python bean classes -> row-format Schema.

Restates org.apache.fory.format.type.TypeInference.inferField
(java/fory-format/src/main/java/org/apache/fory/format/type/TypeInference.java:141-254)
for Python classes whose annotations name Java field types:

  primitives (not null):  jboolean jbyte jshort jint jlong jfloat jdouble
  boxed (nullable):       Boolean Byte Short Integer Long Float Double
  nullable other:         String (utf8), LocalDate (date32), Timestamp / Instant
                          (timestamp), Binary (binary), BigDecimal (decimal(38, 18)),
                          BigInteger (decimal(38, 0))  (TypeInference.java:198-204)
  List[X] / X[]           list (nullable) with element field "item"
  Dict[K, V] / Map<K,V>   map (nullable): key field "key" forced not-null, value "value"
                          (TypeInference.java:228-237, DataTypes.mapField :404-424)
  any annotated class     nested bean -> nullable struct

Field order = names sorted with String.compareTo (Descriptor.java:415-423);
field names = StringUtils.lowerCamelToLowerUnderscore (StringUtils.java:252-271).
"""
from __future__ import annotations

import typing
from typing import Dict, List

from .types import DataType, DataTypes, Field, Schema, ArrowType


class _JavaType:
    type_id: int = ArrowType.NA
    nullable: bool = True


def _jt(name: str, type_id: int, nullable: bool):
    return type(name, (_JavaType,), {"type_id": type_id, "nullable": nullable})


# primitives: DataTypes.notNullFieldType (TypeInference.java:164-181)
jboolean = _jt("jboolean", ArrowType.BOOL, False)
jbyte = _jt("jbyte", ArrowType.INT8, False)
jshort = _jt("jshort", ArrowType.INT16, False)
jint = _jt("jint", ArrowType.INT32, False)
jlong = _jt("jlong", ArrowType.INT64, False)
jfloat = _jt("jfloat", ArrowType.FLOAT, False)
jdouble = _jt("jdouble", ArrowType.DOUBLE, False)
# boxed: FieldType.nullable (TypeInference.java:182-197)
Boolean = _jt("Boolean", ArrowType.BOOL, True)
Byte = _jt("Byte", ArrowType.INT8, True)
Short = _jt("Short", ArrowType.INT16, True)
Integer = _jt("Integer", ArrowType.INT32, True)
Long = _jt("Long", ArrowType.INT64, True)
Float = _jt("Float", ArrowType.FLOAT, True)
Double = _jt("Double", ArrowType.DOUBLE, True)
# TypeInference.java:205-218
String = _jt("String", ArrowType.STRING, True)
LocalDate = _jt("LocalDate", ArrowType.DATE32, True)
Timestamp = _jt("Timestamp", ArrowType.TIMESTAMP, True)
Instant = _jt("Instant", ArrowType.TIMESTAMP, True)
Binary = _jt("Binary", ArrowType.BINARY, True)
# TypeInference.java:198-204: Decimal(DecimalUtils.MAX_PRECISION 38, MAX_SCALE 18) /
# Decimal(38, 0), nullable
BigDecimal = type("BigDecimal", (_JavaType,), {"type_id": ArrowType.DECIMAL128, "nullable": True,
                                               "precision": 38, "scale": 18})
BigInteger = type("BigInteger", (_JavaType,), {"type_id": ArrowType.DECIMAL128, "nullable": True,
                                               "precision": 38, "scale": 0, "big_integer": True})


def lower_camel_to_lower_underscore(s: str) -> str:
    """StringUtils.lowerCamelToLowerUnderscore (StringUtils.java:252-271)."""
    out = []
    start = 0
    for i, ch in enumerate(s):
        if "A" <= ch <= "Z":
            out.append(s[start:i])
            out.append("_")
            out.append(ch.lower())
            start = i + 1
    if start < len(s):
        out.append(s[start:])
    return "".join(out)


def _java_compare_key(name: str):
    # String.compareTo compares UTF-16 code units.
    return name.encode("utf-16-be")


def _bean_fields(cls) -> List[str]:
    hints = typing.get_type_hints(cls)
    return sorted(hints.keys(), key=_java_compare_key)


def _infer_field(name: str, tp, walked: List[type]) -> Field:
    origin = typing.get_origin(tp)
    if origin in (list, List):
        (elem,) = typing.get_args(tp)
        item = _infer_field("item", elem, walked)
        return DataTypes.array_field(name, item)
    if origin in (dict, Dict):
        kt, vt = typing.get_args(tp)
        key = _infer_field("key", kt, walked)
        key = Field(key.name, key.type, False, key.children)  # Map's keys must be non-nullable
        return DataTypes.map_field(name, key, _infer_field("value", vt, walked))
    if isinstance(tp, type) and issubclass(tp, _JavaType):
        if tp.type_id == ArrowType.DECIMAL128:
            if getattr(tp, "big_integer", False):  # toByteArray() bytes (BaseBinaryEncoderBuilder.java:192-194)
                return Field(name, DataTypes.big_integer(), tp.nullable)
            return Field(name, DataTypes.decimal(tp.precision, tp.scale), tp.nullable)
        return Field(name, DataType(tp.type_id), tp.nullable)
    if isinstance(tp, type) and getattr(tp, "__annotations__", None):
        if tp in walked:  # TypeResolutionContext.checkNoCycle
            raise ValueError(f"circular references in bean class are not allowed: {tp}")
        hints = typing.get_type_hints(tp)
        children = [
            _infer_field(lower_camel_to_lower_underscore(n), hints[n], walked + [tp])
            for n in _bean_fields(tp)
        ]
        return DataTypes.struct_field(name, True, children)
    raise NotImplementedError(
        f"Unsupported type {tp} for field {name}, seen type set is {walked}")


def infer_schema(cls) -> Schema:
    """TypeInference.inferSchema(Class) (TypeInference.java:68-80)."""
    f = _infer_field("", cls, [])
    if f.type.id != ArrowType.STRUCT:
        raise ValueError(f"{cls} is not a bean class")
    return Schema(f.children)


def field_names(cls) -> Dict[str, str]:
    """schema field name -> Python attribute name, in schema order."""
    return {lower_camel_to_lower_underscore(n): n for n in _bean_fields(cls)}
