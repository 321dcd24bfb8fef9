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


# --- type trees against the reference's Python infer_schema (tests/golden) ----------
def _java_classes():
    """Java-typed mirrors of the golden classes (primitives where the Java beans have them:
    Mixed / Nested fields, RowEncoderTest.Bar.f1 / Foo.f1 are int/long/double)."""
    from typing import Dict
    kinds = {ArrowType.INT32: I.jint, ArrowType.INT64: I.jlong, ArrowType.DOUBLE: I.jdouble,
             ArrowType.STRING: I.String}
    mixed = type("Mixed", (), {"__annotations__": {n: kinds[k] for n, k in W.mixed_decl()}})
    inner = type("Inner", (), {"__annotations__": {"x": I.jint, "y": I.jlong, "z": List[I.Long]}})
    nested = type("Nested", (), {"__annotations__": {"a": I.jlong, "b": I.jdouble, "c": inner}})
    bar = type("Bar", (), {"__annotations__": {"f1": I.jint, "f2": I.String}})
    foo = type("Foo", (), {"__annotations__": {"f1": I.jint, "f2": I.String, "f3": List[I.String],
                                               "f4": Dict[I.String, I.Integer], "f5": bar}})
    colls = type("Colls", (), {"__annotations__": {
        "double2d": List[List[I.Double]], "bars": List[bar], "bar_map": Dict[I.String, bar],
        "nest": List[List[List[bar]]], "counts": Dict[I.Integer, I.Long], "blobs": List[I.Binary]}})
    return {"mixed40": mixed, "nested": nested, "bar": bar, "foo": foo, "collections": colls}


def _tree(f):
    return {"name": f.name, "type_id": int(f.type.id), "nullable": bool(f.nullable),
            "children": [_tree(c) for c in f.children]}


def _strip_nullable(t, primitive_ids):
    """The reference Python marks every field nullable; Java primitives are not-null
    (TypeInference.java:164-181): compare nullability only for non-primitive fields."""
    out = dict(t)
    if t["type_id"] in primitive_ids and not t["nullable"]:
        out["nullable"] = None
    out["children"] = [_strip_nullable(c, primitive_ids) for c in t["children"]]
    return out


@pytest.mark.parametrize("name", ["mixed40", "nested", "bar", "foo", "collections"])
def test_type_trees_match_reference_infer_schema(golden, name):
    from fury_amd.format.native import NativePlan
    want = golden["inferred"][name]
    s = I.infer_schema(_java_classes()[name])
    got = [_tree(f) for f in s]
    prim = {ArrowType.BOOL, ArrowType.INT8, ArrowType.INT16, ArrowType.INT32, ArrowType.INT64,
            ArrowType.FLOAT, ArrowType.DOUBLE}
    g = [_strip_nullable(t, prim) for t in got]

    def relax(w, gg):  # where ours is a not-null primitive, accept the reference's nullable=True
        return {**w, "nullable": gg["nullable"] if gg["nullable"] is None else w["nullable"],
                "children": [relax(a, b) for a, b in zip(w["children"], gg["children"])]}

    assert [relax(w, x) for w, x in zip(want["fields"], g)] == g
    from oracle import oracle
    assert oracle.schema_hash(s) == want["hash"]
    assert NativePlan(s).schema_hash == want["hash"]
    if name in ("mixed40", "nested"):  # the bench's hand-built schemas are the inferred ones
        ref = W.mixed_schema() if name == "mixed40" else W.nested_schema()
        assert [_tree(f) for f in ref] == got
