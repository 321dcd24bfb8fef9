"""Shared test helpers: schema catalog and column comparison."""
from __future__ import annotations

from typing import List

import numpy as np

from fury_amd import workloads as W
from fury_amd.format.columns import HostColumn, build_columns, unpack_validity
from fury_amd.format.types import ArrowType, DataType, DataTypes, Field, Schema, preorder


def all_types_schema() -> Schema:
    """Every fixed-width type, nullable (boxed) and not (primitive)."""
    fields = []
    for k, name in [(ArrowType.BOOL, "b"), (ArrowType.INT8, "i8"), (ArrowType.INT16, "i16"),
                    (ArrowType.INT32, "i32"), (ArrowType.INT64, "i64"), (ArrowType.FLOAT, "f32"),
                    (ArrowType.DOUBLE, "f64"), (ArrowType.DATE32, "d32"), (ArrowType.TIMESTAMP, "ts")]:
        fields.append(Field(name + "_boxed", DataType(k), True))
        fields.append(Field(name + "_prim", DataType(k), False))
    return Schema(sorted(fields, key=lambda f: f.name))


def random_fixed_columns(schema: Schema, n: int, seed: int, null_rate: float = 0.3) -> List[HostColumn]:
    from fury_amd.format.columns import NP_DTYPE, pack_validity
    rng = np.random.default_rng(seed)
    cols = []
    for f in schema.fields:
        dt = NP_DTYPE[f.type.id]
        raw = rng.integers(0, 256, size=n * np.dtype(dt).itemsize, dtype=np.uint8)
        v = raw.view(dt).copy()
        if f.type.id == ArrowType.BOOL:
            v = (rng.random(n) < 0.5).astype(np.uint8) * rng.integers(1, 255, size=n).astype(np.uint8)
        valid = None
        if f.nullable:
            valid = pack_validity(rng.random(n) >= null_rate)
        cols.append(HostColumn(v, None, valid, n))
    return cols


def wide_schema(n: int = 300) -> Schema:
    return Schema([Field(f"c{i:04d}", DataType([ArrowType.INT64, ArrowType.INT32, ArrowType.INT16,
                                                 ArrowType.INT8][i % 4]), i % 3 == 0) for i in range(n)])


def string_list_rows(n: int, seed: int):
    """Python rows for a schema with strings (incl. unicode/empty/null) and a list<int32>."""
    rng = np.random.default_rng(seed)
    alphabet = ["a", "bc", "é", "中文", "😀", "", "xyz" * 5]
    rows = []
    for i in range(n):
        s = None if rng.random() < 0.2 else "".join(rng.choice(alphabet, size=rng.integers(0, 6)))
        b = None if rng.random() < 0.2 else bytes(rng.integers(0, 256, size=rng.integers(0, 20), dtype=np.uint8))
        lst = None if rng.random() < 0.2 else [None if rng.random() < 0.1 else int(x)
                                               for x in rng.integers(-1000, 1000, size=rng.integers(0, 70))]
        rows.append({"id": int(i), "name": s, "payload": b, "vals": lst,
                     "score": None if rng.random() < 0.3 else float(rng.standard_normal())})
    return rows


def string_list_schema() -> Schema:
    return Schema([
        Field("id", DataType(ArrowType.INT64), False),
        Field("name", DataType(ArrowType.STRING), True),
        Field("payload", DataType(ArrowType.BINARY), True),
        Field("score", DataType(ArrowType.DOUBLE), True),
        DataTypes.array_field("vals", Field("item", DataType(ArrowType.INT32), True)),
    ])


def columns_equal(schema: Schema, a: List[HostColumn], b: List[HostColumn]) -> List[str]:
    """Semantic equality of two pre-order column sets (values compared only where valid)."""
    errs = []
    fields = preorder(schema)
    parent = _struct_parents(schema)
    eff = {}
    for i, f in enumerate(fields):
        ca, cb = a[i], b[i]
        n = ca.length
        if ca.length != cb.length:
            errs.append(f"{i}:{f.name} length {ca.length} != {cb.length}")
            continue
        va = unpack_validity(ca.validity if f.nullable else None, n)
        vb = unpack_validity(cb.validity if f.nullable else None, n)
        if i in parent:  # a child of a null struct is absent: compare under the parent's validity
            pv = eff.get(parent[i])
            if pv is not None:
                va, vb = va & pv, vb & pv
        eff[i] = va
        if not np.array_equal(va, vb):
            errs.append(f"{i}:{f.name} validity differs at {np.nonzero(va != vb)[0][:5]}")
            continue
        t = f.type.id
        if ca.values is not None and t not in (ArrowType.STRING, ArrowType.BINARY):
            xa = np.asarray(ca.values)[:n].view(np.uint8).reshape(n, -1) if n else np.zeros((0, 1), np.uint8)
            xb = np.asarray(cb.values)[:n].view(np.uint8).reshape(n, -1) if n else np.zeros((0, 1), np.uint8)
            if t == ArrowType.BOOL:
                xa, xb = (xa != 0), (xb != 0)
            bad = np.nonzero(np.any(xa != xb, axis=1) & va)[0]
            if len(bad):
                errs.append(f"{i}:{f.name} values differ at rows {bad[:5]}")
        if t in (ArrowType.STRING, ArrowType.BINARY, ArrowType.LIST, ArrowType.MAP):
            oa = np.asarray(ca.offsets)[: n + 1].astype(np.int64)
            ob = np.asarray(cb.offsets)[: n + 1].astype(np.int64)
            la, lb = np.diff(oa), np.diff(ob)
            bad = np.nonzero((la != lb) & va)[0]
            if len(bad):
                errs.append(f"{i}:{f.name} lengths differ at rows {bad[:5]}")
                continue
            if t not in (ArrowType.LIST, ArrowType.MAP):
                for r in np.nonzero(va)[0]:
                    if bytes(np.asarray(ca.values)[oa[r]:oa[r + 1]]) != bytes(np.asarray(cb.values)[ob[r]:ob[r + 1]]):
                        errs.append(f"{i}:{f.name} bytes differ at row {r}")
                        break
    return errs


def flat_mix_rows(n: int, seed: int):
    """Flat varlen rows: short and long strings (spans beyond one staging buffer),
    list<int64>/list<int16> with not-null items, list<bool>, bool / int8 fields."""
    rng = np.random.default_rng(seed)
    rows = []
    for i in range(n):
        long_len = int(rng.integers(0, 300)) if rng.random() < 0.5 else int(rng.integers(0, 8))
        rows.append({
            "a": bool(rng.random() < 0.5),
            "b": int(rng.integers(-128, 128)),
            "c": None if rng.random() < 0.1 else "".join(chr(int(x)) for x in rng.integers(97, 123, size=rng.integers(0, 12))),
            "d": "".join(chr(int(x)) for x in rng.integers(65, 91, size=long_len)),
            "e": None if rng.random() < 0.15 else [int(x) for x in rng.integers(-2**62, 2**62, size=rng.integers(0, 20))],
            "f": [int(x) for x in rng.integers(-30000, 30000, size=rng.integers(0, 9))],
            "g": [bool(x) for x in rng.integers(0, 2, size=rng.integers(0, 5))],
            "h": int(rng.integers(-2**31, 2**31)),
        })
    return rows


def flat_mix_schema() -> Schema:
    return Schema([
        Field("a", DataType(ArrowType.BOOL), False),
        Field("b", DataType(ArrowType.INT8), False),
        Field("c", DataType(ArrowType.STRING), True),
        Field("d", DataType(ArrowType.STRING), False),
        DataTypes.array_field("e", Field("item", DataType(ArrowType.INT64), False)),
        Field("f", DataType(ArrowType.LIST), False, [Field("item", DataType(ArrowType.INT16), False)]),
        Field("g", DataType(ArrowType.LIST), False, [Field("item", DataType(ArrowType.BOOL), False)]),
        Field("h", DataType(ArrowType.INT32), False),
    ])


def deep_nested_rows(n: int, seed: int):
    """Rows of deep_nested_schema: null structs at two levels, strings and lists
    inside child rows, an all-fixed child struct, empty strings/lists."""
    rng = np.random.default_rng(seed)
    rows = []

    def s(k):
        return "".join(chr(int(x)) for x in rng.integers(97, 123, size=rng.integers(0, k)))

    for i in range(n):
        q = None if rng.random() < 0.2 else {
            "s": s(20),
            "v": None if rng.random() < 0.2 else [None if rng.random() < 0.1 else int(x)
                                                  for x in rng.integers(-9999, 9999, size=rng.integers(0, 40))],
            "w": None if rng.random() < 0.3 else int(rng.integers(-30000, 30000)),
        }
        p = None if rng.random() < 0.15 else {
            "k": bool(rng.random() < 0.5),
            "name": None if rng.random() < 0.2 else s(12),
            "q": q,
        }
        rows.append({
            "id": int(rng.integers(-2**62, 2**62)),
            "p": p,
            "r": {"x": float(rng.standard_normal()),
                  "y": [int(x) for x in rng.integers(-2**62, 2**62, size=rng.integers(0, 10))]},
            "t": {"u": int(rng.integers(-2**31, 2**31)), "z": float(rng.standard_normal())},
            "tag": s(30),
        })
    return rows


def deep_nested_schema() -> Schema:
    q = DataTypes.struct_field("q", True, [
        Field("s", DataType(ArrowType.STRING), False),
        DataTypes.array_field("v", Field("item", DataType(ArrowType.INT32), True)),
        Field("w", DataType(ArrowType.INT16), True),
    ])
    p = DataTypes.struct_field("p", True, [
        Field("k", DataType(ArrowType.BOOL), False),
        Field("name", DataType(ArrowType.STRING), True),
        q,
    ])
    r = DataTypes.struct_field("r", False, [
        Field("x", DataType(ArrowType.DOUBLE), False),
        Field("y", DataType(ArrowType.LIST), False, [Field("item", DataType(ArrowType.INT64), False)]),
    ])
    t = DataTypes.struct_field("t", False, [
        Field("u", DataType(ArrowType.INT32), False),
        Field("z", DataType(ArrowType.FLOAT), False),
    ])
    return Schema([Field("id", DataType(ArrowType.INT64), False), p, r, t,
                   Field("tag", DataType(ArrowType.STRING), False)])


def maps_rows(n: int, seed: int):
    """Rows of maps_schema: null / empty / up to 70 entries (bitmap beyond one word),
    null values, bool values, a map inside a nullable struct."""
    rng = np.random.default_rng(seed)
    rows = []
    for i in range(n):
        def m(k, null_p=0.1, vals=lambda: int(rng.integers(-2**62, 2**62))):
            if rng.random() < null_p:
                return None
            keys = rng.choice(10**6, size=int(rng.integers(0, k)), replace=False)
            return {int(x): (None if rng.random() < 0.15 else vals()) for x in keys}
        s = None if rng.random() < 0.2 else {
            "flags": m(6, vals=lambda: bool(rng.random() < 0.5)),
            "w": int(rng.integers(-999, 999)),
        }
        rows.append({
            "a": int(rng.integers(-2**31, 2**31)),
            "counts": m(70),
            "s": s,
            "scores": None if rng.random() < 0.1 else {int(x): float(rng.standard_normal())
                                                       for x in rng.choice(1000, size=rng.integers(0, 5),
                                                                           replace=False)},
        })
    return rows


def maps_schema() -> Schema:
    return Schema([
        Field("a", DataType(ArrowType.INT32), False),
        DataTypes.map_field("counts", Field("key", DataType(ArrowType.INT32), False),
                            Field("value", DataType(ArrowType.INT64), True)),
        DataTypes.struct_field("s", True, [
            DataTypes.map_field("flags", Field("key", DataType(ArrowType.INT64), False),
                                Field("value", DataType(ArrowType.BOOL), True)),
            Field("w", DataType(ArrowType.INT16), False),
        ]),
        DataTypes.map_field("scores", Field("key", DataType(ArrowType.INT16), False),
                            Field("value", DataType(ArrowType.DOUBLE), False)),
    ])


def list_struct_rows(n: int, seed: int):
    """Rows of list_struct_schema: List<Bean> with null elements, null / empty lists,
    more than 64 elements (element bitmap beyond one word), nullable bean fields."""
    rng = np.random.default_rng(seed)
    rows = []
    for i in range(n):
        items = None
        if rng.random() >= 0.15:
            k = int(rng.integers(0, 70)) if rng.random() < 0.1 else int(rng.integers(0, 6))
            items = [None if rng.random() < 0.1 else {
                "a": int(rng.integers(-2**31, 2**31)),
                "b": None if rng.random() < 0.3 else int(rng.integers(-2**62, 2**62)),
                "c": bool(rng.random() < 0.5),
                "d": float(rng.standard_normal()),
            } for _ in range(k)]
        rows.append({"id": int(rng.integers(-2**62, 2**62)), "items": items,
                     "tag": "".join(chr(int(x)) for x in rng.integers(97, 123, size=rng.integers(0, 10)))})
    return rows


def string_elems_schema() -> Schema:
    """List<String>, List<byte[]>, Map<String, String>, Map<String, Integer> inside a
    nullable bean, Map<Long, byte[]>: string/binary array elements and map keys/values
    (BinaryArrayWriter with 8-byte (offset, size) element slots)."""
    return Schema([
        Field("id", DataType(ArrowType.INT64), False),
        DataTypes.array_field("names", Field("item", DataType(ArrowType.STRING), True)),
        DataTypes.array_field("blobs", Field("item", DataType(ArrowType.BINARY), False)),
        DataTypes.map_field("attrs", Field("key", DataType(ArrowType.STRING), False),
                            Field("value", DataType(ArrowType.STRING), True)),
        DataTypes.struct_field("s", True, [
            DataTypes.map_field("idx", Field("key", DataType(ArrowType.STRING), False),
                                Field("value", DataType(ArrowType.INT32), True)),
            Field("z", DataType(ArrowType.INT16), False),
        ]),
        DataTypes.map_field("codes", Field("key", DataType(ArrowType.INT64), False),
                            Field("value", DataType(ArrowType.BINARY), True)),
    ])


def string_elems_rows(n: int, seed: int):
    """Rows of string_elems_schema: null / empty containers, null elements and values,
    empty and multi-byte UTF-8 strings, one container in ten beyond 64 elements."""
    rng = np.random.default_rng(seed)
    alphabet = "abcdefghijklmnopqrstuvwxyz0123456789 éü中文"

    def text(k=20):
        return "".join(alphabet[int(x)] for x in rng.integers(0, len(alphabet), size=rng.integers(0, k)))

    def count():
        return int(rng.integers(0, 70)) if rng.random() < 0.1 else int(rng.integers(0, 6))

    def smap(val, null_p=0.1):
        if rng.random() < null_p:
            return None
        return {f"{text(6)}#{j}": (None if rng.random() < 0.15 else val()) for j in range(count())}

    rows = []
    for _ in range(n):
        rows.append({
            "id": int(rng.integers(-2**62, 2**62)),
            "names": None if rng.random() < 0.1 else [None if rng.random() < 0.15 else text() for _ in range(count())],
            "blobs": None if rng.random() < 0.1 else [bytes(rng.integers(0, 256, size=rng.integers(0, 30),
                                                                         dtype=np.uint8)) for _ in range(count())],
            "attrs": smap(lambda: text(40)),
            "s": None if rng.random() < 0.2 else {"idx": smap(lambda: int(rng.integers(-2**31, 2**31))),
                                                  "z": int(rng.integers(-999, 999))},
            "codes": None if rng.random() < 0.1 else {
                int(k): (None if rng.random() < 0.2 else bytes(rng.integers(0, 256, size=rng.integers(0, 12),
                                                                             dtype=np.uint8)))
                for k in rng.choice(10**6, size=count(), replace=False)},
        })
    return rows


def list_struct_schema() -> Schema:
    bean = DataTypes.struct_field("item", True, [
        Field("a", DataType(ArrowType.INT32), False),
        Field("b", DataType(ArrowType.INT64), True),
        Field("c", DataType(ArrowType.BOOL), False),
        Field("d", DataType(ArrowType.FLOAT), False),
    ])
    return Schema([Field("id", DataType(ArrowType.INT64), False),
                   Field("items", DataType(ArrowType.LIST), True, [bean]),
                   Field("tag", DataType(ArrowType.STRING), True)])


def catalog():
    """name -> (schema, host column factory(n, seed))."""
    return {
        "struct104": (W.struct_schema(), lambda n, s: W.struct_host_columns(n, seed_base=17 + s)),
        "struct104_boxed": (W.struct_schema(boxed=True),
                            lambda n, s: random_fixed_columns(W.struct_schema(boxed=True), n, s)),
        "all_types": (all_types_schema(), lambda n, s: random_fixed_columns(all_types_schema(), n, s)),
        "wide300": (wide_schema(), lambda n, s: random_fixed_columns(wide_schema(), n, s)),
        "mixed40": (W.mixed_schema(), lambda n, s: W.mixed_host_columns(n, seed=23 + s)),
        "mixed40_nulls": (W.mixed_schema(), lambda n, s: W.mixed_host_columns(n, seed=23 + s, null_rate=0.2)),
        "nested": (W.nested_schema(), lambda n, s: W.nested_host_columns(n, seed=29 + s)),
        "nested_nulls": (W.nested_schema(), lambda n, s: W.nested_host_columns(n, seed=29 + s, null_rate=0.25)),
        "strings_lists": (string_list_schema(),
                          lambda n, s: build_columns(string_list_schema(), string_list_rows(n, s))),
        "flat_mix": (flat_mix_schema(), lambda n, s: build_columns(flat_mix_schema(), flat_mix_rows(n, s))),
        "deep_nested": (deep_nested_schema(),
                        lambda n, s: build_columns(deep_nested_schema(), deep_nested_rows(n, s))),
        "maps": (maps_schema(), lambda n, s: build_columns(maps_schema(), maps_rows(n, s))),
        "list_struct": (list_struct_schema(),
                        lambda n, s: build_columns(list_struct_schema(), list_struct_rows(n, s))),
        "string_elems": (string_elems_schema(),
                         lambda n, s: build_columns(string_elems_schema(), string_elems_rows(n, s))),
    }


def _struct_parents(schema: Schema):
    """pre-order index -> index of its parent STRUCT (struct children only)."""
    out = {}
    pos = [0]

    def visit(f, par):
        me = pos[0]
        pos[0] += 1
        if par is not None:
            out[me] = par
        for c in f.children:
            visit(c, me if f.type.id == ArrowType.STRUCT else None)

    for f in schema.fields:
        visit(f, None)
    return out


def collection_cases(n=300, seed=5):
    """One-field schemas of the standalone collection encoders (Encoders.arrayEncoder /
    mapEncoder) and their rows: list<Long>, List<Bean>, Map<Integer, Long>, List<String>,
    Map<String, String>."""
    rng = np.random.default_rng(seed)

    def bean():
        return {"a": int(rng.integers(-2**31, 2**31)), "b": None if rng.random() < 0.3 else int(rng.integers(-2**62, 2**62)),
                "c": bool(rng.random() < 0.5), "d": float(np.float32(rng.standard_normal()))}

    longs = Schema([DataTypes.array_field("", Field("item", DataType(ArrowType.INT64), True))])
    beans = Schema([list_struct_schema().fields[1]])
    amap = Schema([maps_schema().fields[1]])
    names = Schema([string_elems_schema().fields[1]])
    attrs = Schema([string_elems_schema().fields[3]])
    out = []
    for schema, gen in [
        (longs, lambda: {"": [None if rng.random() < 0.1 else int(x) for x in rng.integers(-9, 9, size=rng.integers(0, 70))]}),
        (beans, lambda: {"items": [None if rng.random() < 0.2 else bean() for _ in range(int(rng.integers(0, 5)))]}),
        (amap, lambda: {"counts": {int(k): (None if rng.random() < 0.2 else int(k) * 3)
                                   for k in rng.choice(1000, size=rng.integers(0, 9), replace=False)}}),
    ]:
        rows = [gen() for _ in range(n)]
        out.append((schema, build_columns(schema, rows)))
    # List<String> / Map<String, String> collections
    for schema, key in ((names, "names"), (attrs, "attrs")):
        empty = [] if key == "names" else {}
        rows = [{key: empty if r[key] is None else r[key]} for r in string_elems_rows(n, seed)]
        out.append((schema, build_columns(schema, rows)))
    return out


# --- nested collections (the tree engine's shapes) -----------------------------------
# Mirrors of the reference's test beans, inferred like Encoders.bean does
# (TypeInference.java:141-254): RowEncoderTest.Foo / Bar (RowEncoderTest.java:66-95),
# BeanA / BeanB (fory-test-core .../bean/BeanA.java:34-53, BeanB.java:29-36) without
# the transient f13 (f16 is a BigDecimal: decimal(38, 18)). Java arrays are
# lists of not-null elements (int[] -> list<int32>, byte[] -> list<int8>,
# Iterable<BeanB> -> list<struct>).
def reference_beans():
    from typing import Dict, List as L
    from fury_amd.format import infer as I
    bar = type("Bar", (), {"__annotations__": {"f1": I.jint, "f2": I.String}})
    foo = type("Foo", (), {"__annotations__": {"f1": I.jint, "f2": I.String, "f3": L[I.String],
                                               "f4": Dict[I.String, I.Integer], "f5": bar}})
    bean_b = type("BeanB", (), {"__annotations__": {
        "f1": I.jshort, "f2": I.Integer, "f3": I.jlong, "f4": I.Float, "f5": I.jdouble,
        "intArr": L[I.jint], "intList": L[I.Integer]}})
    bean_a = type("BeanA", (), {"__annotations__": {
        "f1": I.jshort, "f2": I.Integer, "f3": I.jlong, "f4": I.Float, "f5": I.jdouble, "beanB": bean_b,
        "intArray": L[I.jint], "bytes": L[I.jbyte], "f12": I.jboolean, "f15": I.Integer, "f16": I.BigDecimal, "f17": I.String,
        "longStringField": I.String, "doubleList": L[I.Double], "beanBIterable": L[bean_b],
        "beanBList": L[bean_b], "stringBeanBMap": Dict[I.String, bean_b], "int2DArray": L[L[I.jint]],
        "double2DList": L[L[I.Double]]}})
    return {"Bar": bar, "Foo": foo, "BeanA": bean_a, "BeanB": bean_b}


def nested_schemas():
    """name -> schema of nestings the op programs do not cover (plus Foo, which they do)."""
    from typing import Dict, List as L
    from fury_amd.format import infer as I
    B = reference_beans()
    bar, foo = B["Bar"], B["Foo"]
    holder = type("Holder", (), {"__annotations__": {
        "id": I.jlong, "bars": L[bar], "barMap": Dict[I.String, bar], "tag": I.String}})
    lists = type("Lists", (), {"__annotations__": {
        "longs2d": L[L[I.Long]], "names2d": L[L[I.String]], "shorts3d": L[L[L[I.jshort]]], "x": I.jint}})
    maps = type("Maps", (), {"__annotations__": {
        "fooBars": Dict[foo, L[bar]], "nest": Dict[I.String, L[L[bar]]], "ints": Dict[I.String, L[I.Integer]],
        "k": I.Byte}})
    deep = DataTypes.array_field("deep", DataTypes.map_field(
        "item", Field("key", DataType(ArrowType.STRING), False),
        DataTypes.array_field("value", DataTypes.struct_field("item", True, [
            Field("s", DataType(ArrowType.STRING), True),
            DataTypes.array_field("l", DataTypes.array_field("item", Field("item", DataType(ArrowType.INT16), True))),
            Field("b", DataType(ArrowType.BOOL), False)]))))
    # BigDecimal / BigInteger fields (TypeInference.java:198-204) in rows, child rows,
    # lists and map values; one decimal of precision 10 (out-of-range values are errors)
    decimals = type("Decimals", (), {"__annotations__": {
        "amount": I.BigDecimal, "count": I.BigInteger, "prices": L[I.BigDecimal],
        "byName": Dict[I.String, I.BigDecimal], "inner": type("Inner", (), {"__annotations__": {
            "d": I.BigDecimal, "n": I.jint}}), "id": I.jlong}})
    dec_schema = I.infer_schema(decimals)
    dec_schema.fields.append(Field("small", DataTypes.decimal(10, 2), True))
    chain = Field("item", DataType(ArrowType.INT32), True)
    for k in range(9):  # list^9<int32>: 10 schema levels (the 18-frame instantiation)
        chain = DataTypes.array_field("item" if k < 8 else "chain", chain)
    return {
        "holder": I.infer_schema(holder),
        "lists": I.infer_schema(lists),
        "maps_nested": I.infer_schema(maps),
        "foo": I.infer_schema(foo),
        "bean_a": I.infer_schema(B["BeanA"]),
        "decimals": dec_schema,
        "deep": Schema([Field("id", DataType(ArrowType.INT32), False), deep]),
        "chain": Schema([chain, Field("z", DataType(ArrowType.INT64), True)]),
    }


def random_value(f: Field, rng, depth: int = 0, null_p: float = 0.12):
    """A random Python value of field f (None for nulls): containers hold 0-4 elements,
    one in twelve near the top holds up to 70 (element bitmaps beyond one word)."""
    if f.nullable and rng.random() < null_p:
        return None
    t = f.type.id
    if t == ArrowType.STRUCT:
        return {c.name: random_value(c, rng, depth + 1, null_p) for c in f.children}
    if t in (ArrowType.LIST, ArrowType.MAP):
        k = int(rng.integers(0, 70)) if depth < 2 and rng.random() < 1 / 12 else int(rng.integers(0, 5))
        if t == ArrowType.LIST:
            return [random_value(f.children[0], rng, depth + 1, null_p) for _ in range(k)]
        return [(random_value(f.children[0], rng, depth + 1, null_p), random_value(f.children[1], rng, depth + 1, null_p))
                for _ in range(k)]
    if t == ArrowType.DECIMAL128 and f.type.big_integer:  # any int128: toByteArray() of 1..16 bytes
        r = rng.random()
        if r < 0.25:  # the length boundaries of toByteArray() and the int128 extremes
            edges = (0, -1, 127, 128, -128, -129, 255, 256, 32767, 32768, -32769, 2 ** 63, -(2 ** 63) - 1,
                     2 ** 127 - 1, -(2 ** 127), 2 ** 119, -(2 ** 119) - 1)
            return edges[int(rng.integers(0, len(edges)))]
        bits = int(rng.integers(1, 128))
        u = int.from_bytes(rng.bytes(16), "little") & ((1 << bits) - 1)
        return -u - 1 if rng.random() < 0.5 else u
    if t == ArrowType.DECIMAL128:  # the unscaled value: up to `precision` digits, either sign
        p = f.type.precision or 38
        r = rng.random()
        if r < 0.1:  # the extremes of the precision
            u = 10 ** p - 1
        elif r < 0.3:
            u = int(rng.integers(0, 1000))
        else:
            digits = int(rng.integers(1, p + 1))
            u = int("".join(str(int(x)) for x in rng.integers(0, 10, size=digits)))
        return -u if rng.random() < 0.5 else u
    if t == ArrowType.STRING:
        alphabet = "abcdefghij0123456789 éü中文😀"
        return "".join(alphabet[int(x)] for x in rng.integers(0, len(alphabet), size=rng.integers(0, 24)))
    if t == ArrowType.BINARY:
        return bytes(rng.integers(0, 256, size=rng.integers(0, 24), dtype=np.uint8))
    if t == ArrowType.BOOL:
        return bool(rng.random() < 0.5)
    if t in (ArrowType.FLOAT, ArrowType.DOUBLE):
        return float(np.float32(rng.standard_normal())) if t == ArrowType.FLOAT else float(rng.standard_normal())
    bits = {ArrowType.INT8: 8, ArrowType.INT16: 16, ArrowType.INT32: 32, ArrowType.DATE32: 32}.get(t, 64)
    return int(rng.integers(-2 ** (bits - 1), 2 ** (bits - 1) - 1, dtype=np.int64))


def random_rows(schema: Schema, n: int, seed: int, null_p: float = 0.12):
    rng = np.random.default_rng(seed)
    return [{f.name: random_value(f, rng, 0, null_p) for f in schema.fields} for _ in range(n)]


def nested_columns(name: str, n: int, seed: int):
    schema = nested_schemas()[name]
    return schema, build_columns(schema, random_rows(schema, n, seed))


def knob_key():
    """The FORY_ROWFMT_* launch knobs in the environment: a plan reads them once, when it
    is created, so encoder caches in the tests are keyed by them too."""
    import os
    return tuple(sorted((k, v) for k, v in os.environ.items() if k.startswith("FORY_ROWFMT_") and k != "FORY_ROWFMT_LIB"))
