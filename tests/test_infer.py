"""CPU: TypeInference mirror (fury_amd.format.infer) against the reference's rules
(TypeInference.java:141-254, Descriptor.java:415-423, StringUtils.java:252-271) and
the reference Python infer_schema field order (tests/golden)."""
from typing import List

import pytest

from fury_amd.format import infer as I
from fury_amd.format.types import ArrowType
from fury_amd import workloads as W


def make_struct_class():
    ann = {}
    kinds = {ArrowType.INT32: I.jint, ArrowType.INT64: I.jlong, ArrowType.FLOAT: I.jfloat,
             ArrowType.DOUBLE: I.jdouble}
    for name, k in W.struct_decl(100):
        ann[name] = kinds[k]
    return type("Struct", (), {"__annotations__": ann})


def test_struct_inference_matches_reference(golden):
    s = I.infer_schema(make_struct_class())
    assert s.names() == golden["struct104_field_order"]
    assert [f.type.id for f in s] == [f.type.id for f in W.struct_schema()]
    assert not any(f.nullable for f in s)
    from fury_amd.format.native import NativePlan
    assert NativePlan(s).schema_hash == golden["struct104_inferred_hash"]


def test_names_and_nullability():
    class Inner:
        x: I.jint
        y: I.Long
        z: List[I.Long]

    class Bean:
        someLongField: I.jlong
        aString: I.String
        inner: Inner
        boxedInt: I.Integer
        flag: I.jboolean

    s = I.infer_schema(Bean)
    assert s.names() == ["a_string", "boxed_int", "flag", "inner", "some_long_field"]
    by = {f.name: f for f in s}
    assert by["a_string"].nullable and by["a_string"].type.id == ArrowType.STRING
    assert not by["flag"].nullable and by["flag"].type.id == ArrowType.BOOL
    assert by["inner"].type.id == ArrowType.STRUCT and by["inner"].nullable
    z = by["inner"].children[2]
    assert z.name == "z" and z.type.id == ArrowType.LIST and z.children[0].name == "item"
    assert z.children[0].nullable


def test_lower_camel_to_lower_underscore():
    assert I.lower_camel_to_lower_underscore("variableName") == "variable_name"
    assert I.lower_camel_to_lower_underscore("f100") == "f100"
    assert I.lower_camel_to_lower_underscore("aBC") == "a_b_c"


def test_unsupported_and_cycles():
    class Bad:
        m: dict

    with pytest.raises(NotImplementedError):
        I.infer_schema(Bad)

    class Node:
        pass

    Node.__annotations__ = {"next": Node, "v": I.jint}
    with pytest.raises(ValueError):
        I.infer_schema(Node)


def test_encoders_bean_wraps_errors():
    pytest.importorskip("torch")
    from fury_amd.format import EncoderException, Encoders

    class Bad:
        m: dict

    with pytest.raises(EncoderException):
        Encoders.bean(Bad)


def test_infer_map_field(golden):
    """Dict[K, V] infers a map with a not-null key (TypeInference.java:228-237) and hashes
    like the reference's map schema."""
    import typing

    from fury_amd.format import infer
    from fury_amd.format.native import NativePlan
    from fury_amd.format.types import ArrowType

    class S:
        flags: typing.Dict[infer.Long, infer.Boolean]
        w: infer.jshort

    class Maps:
        a: infer.jint
        counts: typing.Dict[infer.Integer, infer.Long]
        s: S
        scores: typing.Dict[infer.Short, infer.jdouble]

    schema = infer.infer_schema(Maps)
    m = schema.fields[1]
    assert m.type.id == ArrowType.MAP and m.nullable
    assert [c.name for c in m.children] == ["key", "value"] and not m.children[0].nullable
    assert NativePlan(schema).schema_hash == golden["schema_hash"]["maps"]


def test_infer_list_of_beans(golden):
    """List[Bean] infers a list whose item is a nullable struct (TypeInference.java:222-227,
    DataTypes.arrayField); the device plan accepts beans of fixed-width fields."""
    import typing

    from fury_amd.format import infer
    from fury_amd.format.native import NativePlan
    from fury_amd.format.types import ArrowType

    class Item:
        a: infer.jint
        b: infer.Long
        c: infer.jboolean
        d: infer.jfloat

    class Holder:
        id: infer.jlong
        items: typing.List[Item]
        tag: infer.String

    schema = infer.infer_schema(Holder)
    lst = schema.fields[1]
    assert lst.type.id == ArrowType.LIST and lst.children[0].type.id == ArrowType.STRUCT
    assert NativePlan(schema).schema_hash == golden["schema_hash"]["list_struct"]
