"""Generates tests/golden/schema_hashes.json from the REFERENCE's own Python code.

Runs only in the build container (needs /root/reference; the GPU box never
runs it). It loads python/pyfory/type.py and python/pyfory/format/infer.py
from the reference tree as plain modules (without executing pyfory/__init__.py,
which needs the unbuilt Cython extension) and records:
  - compute_schema_hash (infer.py:160-190) of the S / M / N schemas and of a
    few edge schemas, built as pyarrow schemas mirroring the Java inferred
    schemas (pyarrow type ids == Java ArrowType ordinals, ArrowType.java:25-160);
  - the field order infer_schema produces for the benchmark Struct (infer.py:94-106);
  - infer_schema's type trees (names, type ids, nullability, children) of Python
    classes mirroring the Mixed / Nested / RowEncoderTest.Foo, Bar / collection
    beans (infer.py:94-145).
No reference source is copied; only the resulting numbers are committed.

Usage: python tests/golden/make_golden.py [/root/reference]
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def load_reference(ref: str):
    sys.dont_write_bytecode = True  # never write into the read-only reference tree
    pkg_dir = os.path.join(ref, "python", "pyfory")
    pyfory = types.ModuleType("pyfory")
    pyfory.__path__ = [pkg_dir]
    sys.modules["pyfory"] = pyfory
    fmt = types.ModuleType("pyfory.format")
    fmt.__path__ = [os.path.join(pkg_dir, "format")]
    sys.modules["pyfory.format"] = fmt

    def load(name, path):
        spec = importlib.util.spec_from_file_location(name, path)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
        return mod

    ptype = load("pyfory.type", os.path.join(pkg_dir, "type.py"))
    infer = load("pyfory.format.infer", os.path.join(pkg_dir, "format", "infer.py"))
    return ptype, infer


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    import pyarrow as pa

    ptype, infer = load_reference(ref)
    sys.path.insert(0, REPO)
    from fury_amd import workloads as W
    from fury_amd.format.types import ArrowType

    def to_pa(f):
        t = f.type.id
        simple = {ArrowType.BOOL: pa.bool_(), ArrowType.INT8: pa.int8(), ArrowType.INT16: pa.int16(),
                  ArrowType.INT32: pa.int32(), ArrowType.INT64: pa.int64(),
                  ArrowType.FLOAT: pa.float32(), ArrowType.DOUBLE: pa.float64(),
                  ArrowType.STRING: pa.utf8(), ArrowType.BINARY: pa.binary(),
                  ArrowType.DATE32: pa.date32(), ArrowType.TIMESTAMP: pa.timestamp("us")}
        if t in simple:
            typ = simple[t]
        elif t == ArrowType.LIST:
            typ = pa.list_(to_pa(f.children[0]))
        elif t == ArrowType.STRUCT:
            typ = pa.struct([to_pa(c) for c in f.children])
        elif t == ArrowType.MAP:
            typ = pa.map_(to_pa(f.children[0]).type, to_pa(f.children[1]).type)
        elif t == ArrowType.DECIMAL128:  # pa.decimal128's id == ArrowType.DECIMAL (DECIMAL128) = 23
            typ = pa.decimal128(f.type.precision or 38, f.type.scale)
        else:
            raise ValueError(t)
        return pa.field(f.name, typ, nullable=f.nullable)

    from fury_amd.format.types import DataType, DataTypes, Field, Schema
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from helpers import deep_nested_schema, list_struct_schema, maps_schema, nested_schemas, string_elems_schema

    edge = {
        "empty": Schema([]),
        "one_int": Schema([Field("f", DataType(ArrowType.INT32), False)]),
        "all_types": Schema([Field(f"t{k}", DataType(k), True) for k in
                             (1, 3, 5, 7, 9, 11, 12, 13, 14, 16, 18)]),
        "list_of_string": Schema([DataTypes.array_field("l", Field("item", DataType(ArrowType.STRING)))]),
        "deep": Schema([DataTypes.struct_field("s", True, [DataTypes.struct_field("t", True, [
            Field("u", DataType(ArrowType.INT64))])])]),
        "wide_300": Schema([Field(f"c{i:03d}", DataType(ArrowType.INT64), False) for i in range(300)]),
        "struct_boxed": W.struct_schema(100, boxed=True),
        "maps": maps_schema(),
        "deep_nested": deep_nested_schema(),
        "list_struct": list_struct_schema(),
        "string_elems": string_elems_schema(),
        "decimals": nested_schemas()["decimals"],  # BigDecimal / BigInteger fields (decimal128 ids)
        "bean_a": nested_schemas()["bean_a"],      # BeanA incl. f16 (BigDecimal)
    }
    schemas = {"struct104": W.struct_schema(), "mixed40": W.mixed_schema(),
               "nested": W.nested_schema(), **edge}
    out = {"generator": "tests/golden/make_golden.py", "reference": "python/pyfory/format/infer.py:160-190",
           "schema_hash": {}, "type_ids": {}}
    for name, s in schemas.items():
        pas = pa.schema([to_pa(f) for f in s.fields])
        out["schema_hash"][name] = int(infer.compute_schema_hash(pas))
        out["type_ids"][name] = [int(f.type.id) for f in pas]

    # infer_schema field order for the benchmark Struct (sorted names, infer.py:97)
    ann = {}
    for name, kind in W.struct_decl(100):
        ann[name] = {ArrowType.INT32: pa.int32, ArrowType.INT64: pa.int64,
                     ArrowType.FLOAT: pa.float32, ArrowType.DOUBLE: pa.float64}[kind]
    cls = type("Struct", (), {"__annotations__": ann, "__module__": "golden"})
    inferred = infer.infer_schema(cls)
    out["struct104_field_order"] = [f.name for f in inferred]
    out["struct104_inferred_hash"] = int(infer.compute_schema_hash(inferred))

    # infer_schema type trees of Python classes mirroring the configs' Java beans:
    # field names (sorted), type ids and children, recursively (infer.py:94-106,
    # ArrowTypeVisitor :109-145). The reference's Python marks every field
    # nullable (pa.field default); Java's TypeInference makes primitives not-null
    # (TypeInference.java:164-181) — nullability is recorded as produced.
    import typing

    def tree(field):
        t = field.type
        kids = []
        if isinstance(t, pa.ListType):
            kids = [tree(t.value_field)]
        elif isinstance(t, pa.StructType):
            kids = [tree(t.field(i)) for i in range(t.num_fields)]
        elif isinstance(t, pa.MapType):
            kids = [tree(t.key_field), tree(t.item_field)]
        return {"name": field.name, "type_id": int(t.id), "nullable": bool(field.nullable), "children": kids}

    def cls(name, ann):
        return type(name, (), {"__annotations__": ann, "__module__": "golden"})

    pa_of = {ArrowType.INT32: pa.int32, ArrowType.INT64: pa.int64, ArrowType.DOUBLE: pa.float64,
             ArrowType.STRING: str}
    mixed = cls("Mixed", {n: pa_of[k] for n, k in W.mixed_decl()})
    inner = cls("Inner", {"x": pa.int32, "y": pa.int64, "z": typing.List[pa.int64]})
    nested = cls("Nested", {"a": pa.int64, "b": pa.float64, "c": inner})
    bar = cls("Bar", {"f1": pa.int32, "f2": str})
    foo = cls("Foo", {"f1": pa.int32, "f2": str, "f3": typing.List[str], "f4": typing.Dict[str, pa.int32],
                      "f5": bar})
    colls = cls("Colls", {"double2d": typing.List[typing.List[pa.float64]], "bars": typing.List[bar],
                          "bar_map": typing.Dict[str, bar], "nest": typing.List[typing.List[typing.List[bar]]],
                          "counts": typing.Dict[pa.int32, pa.int64], "blobs": typing.List[bytes]})
    out["inferred"] = {}
    for name, c in (("mixed40", mixed), ("nested", nested), ("bar", bar), ("foo", foo), ("collections", colls)):
        sch = infer.infer_schema(c)
        out["inferred"][name] = {"fields": [tree(f) for f in sch], "hash": int(infer.compute_schema_hash(sch))}

    path = os.path.join(HERE, "schema_hashes.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    main()
