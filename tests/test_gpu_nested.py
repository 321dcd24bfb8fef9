"""GPU: nested collections on the device (the tree engine, fury_amd/csrc/generic.hip).

Shapes the op programs do not cover — list<list<...>>, List<Bean with strings>,
Map<String, Bean>, Map<Bean, List<Bean>>, BeanA (with its BigDecimal), decimal
fields in rows / child rows / lists / map values, a list^9 chain — are encoded on the device byte-identically to the oracle in every
framing, decoded back (with and without row offsets), and the reference's own
ArrayEncoderTest / MapEncoderTest values produce the byte lengths those tests
assert (ArrayEncoderTest.java:56,90,124).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import oracle  # noqa: E402
from fury_amd.format import CorruptRowException, errors  # noqa: E402
from fury_amd.format.columns import build_columns, to_device, to_host  # noqa: E402
from fury_amd.format.encoder import CollectionEncoder, EncodedRows, RowEncoder  # noqa: E402
from fury_amd.format.types import DataTypes, Schema  # noqa: E402
from fury_amd.format import infer as I  # noqa: E402

from helpers import columns_equal, nested_columns, nested_schemas, random_rows, reference_beans, knob_key  # noqa: E402

pytestmark = pytest.mark.gpu

_ENC = {}


def encoder_for(name):
    key = (name, knob_key())  # a plan reads the launch knobs when it is created
    if key not in _ENC:
        _ENC[key] = RowEncoder(nested_schemas()[name])
    return _ENC[key]


def check(schema, enc, cols, n, frame):
    expect, offs = oracle.encode(schema, cols, n, frame)
    rows = enc.encode(to_device(cols), n, frame)
    got = rows.buffer.cpu().numpy()
    assert got.nbytes == expect.nbytes
    bad = np.nonzero(got != expect)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"
    assert np.array_equal(rows.offsets.cpu().numpy(), offs)
    dec = to_host(enc.decode(rows))
    assert columns_equal(schema, cols, dec) == []
    if frame == 1:  # self-delimiting: the device frame index instead of offsets
        dec = to_host(enc.decode(rows.buffer, n, frame, None))
        assert columns_equal(schema, cols, dec) == []
    # the oracle's bytes decode to the oracle's columns
    ref = oracle.decode(schema, expect, offs, n, frame)
    buf = torch.from_numpy(np.concatenate([expect, np.zeros(16, np.uint8)])).cuda()
    dec = to_host(enc.decode(buf, n, frame, torch.from_numpy(offs).cuda()))
    assert columns_equal(schema, ref, dec) == []


NAMES = list(nested_schemas())


@pytest.mark.parametrize("engine", ["columnar", "per_lane"])
@pytest.mark.parametrize("frame", [0, 1, 3])
@pytest.mark.parametrize("n", [0, 1, 65, 700])
@pytest.mark.parametrize("name", NAMES)
def test_nested_parity(name, n, frame, engine, monkeypatch):
    """Both encode engines: the columnar one (treecol.hip, the default when the
    workspace is sized by encode_workspace_bytes) and the per-record one
    (FORY_ROWFMT_TREECOL=0)."""
    if engine == "per_lane":
        monkeypatch.setenv("FORY_ROWFMT_TREECOL", "0")
    if name == "chain" and n > 65:
        n = 120  # ~20 KiB per record
    schema, cols = nested_columns(name, n, 100 + n + frame)
    check(schema, encoder_for(name), cols, n, frame)


@pytest.mark.parametrize("name", ["holder", "lists", "maps_nested", "bean_a", "deep", "decimals"])
def test_nested_all_null_and_empty(name):
    """Every nullable value null; then every container empty."""
    schema = nested_schemas()[name]
    n = 300
    rows = random_rows(schema, n, 5, null_p=1.0)
    check(schema, encoder_for(name), build_columns(schema, rows), n, 1)
    rng = np.random.default_rng(0)

    def empty(f, v):
        if isinstance(v, dict):
            return {c.name: empty(c, v[c.name]) for c in f.children}
        if isinstance(v, list):
            return []
        return v
    rows = [{f.name: empty(f, r[f.name]) for f in schema.fields} for r in random_rows(schema, n, int(rng.integers(99)))]
    check(schema, encoder_for(name), build_columns(schema, rows), n, 0)


def test_nested_large_batch():
    """100k BeanA-shaped records: one launch of each kernel, round trip + oracle bytes."""
    schema, cols = nested_columns("holder", 100_000, 9)
    check(schema, encoder_for("holder"), cols, 100_000, 1)


# --- the reference's own collection tests --------------------------------------------
def _bar(f1=1, f2="str"):  # RowEncoderTest.Bar(): f1 = 1, f2 = "str" (RowEncoderTest.java:84-95)
    return {"f1": f1, "f2": f2}


def _foo():  # RowEncoderTest.Foo() (RowEncoderTest.java:67-82); HashMap iteration k1, k2
    return {"f1": 2, "f2": "str", "f3": ["a", "b", "c"], "f4": [("k1", 1), ("k2", 2)], "f5": _bar()}


def _array_encoder(elem_type):
    item = I._infer_field("item", elem_type, [])
    return CollectionEncoder(Schema([DataTypes.array_field("", item)]))


def _map_encoder(key_type, value_type):
    key = I._infer_field("key", key_type, [])
    key = type(key)(key.name, key.type, False, key.children)
    return CollectionEncoder(Schema([DataTypes.map_field("", key, I._infer_field("value", value_type, []))]))


def _collection_round_trip(enc, values):
    schema = enc.schema()
    n = len(values)
    cols = build_columns(schema, [{"": v} for v in values])
    expect, offs = oracle.encode(schema, cols, n, 2)
    rows = enc.encode(to_device(cols), n)
    got = rows.buffer.cpu().numpy()
    assert np.array_equal(got, expect)
    assert np.array_equal(rows.offsets.cpu().numpy(), offs)
    assert columns_equal(schema, cols, to_host(enc.decode(rows))) == []
    return [int(got[o:o + 4].view(np.int32)[0]) for o in offs[:-1]]


def test_reference_array_encoder_lengths():
    from typing import Dict, List
    B = reference_beans()
    bar, foo = B["Bar"], B["Foo"]
    # testListEncoder: 5 Bars (k, "i" + k) -> encode(bars).length == 224 (= 8 + array bytes)
    sizes = _collection_round_trip(_array_encoder(bar), [[_bar(k, f"i{k}") for k in range(5)]])
    assert sizes[0] + 8 == 224
    # testNestListEncoder: list i holds i lists of 3 Bars (k, "s" + k) -> 1576
    nest = [[[_bar(k, f"s{k}") for k in range(3)] for _ in range(i)] for i in range(5)]
    sizes = _collection_round_trip(_array_encoder(List[List[bar]]), [nest])
    assert sizes[0] + 8 == 1576
    # testNestArrayWithMapEncoder: 10 x 3 x {Foo(): [Bar(j, "x" + j)]} -> 10824
    lmap = [[[(_foo(), [_bar(j, f"x{j}")])] for j in range(3)] for _ in range(10)]
    sizes = _collection_round_trip(_array_encoder(List[Dict[foo, List[bar]]]), [lmap])
    assert sizes[0] + 8 == 10824
    # the three as one batch of collection frames, plus 500 random ones
    enc = _array_encoder(List[List[bar]])
    rows = random_rows(enc.schema(), 500, 3)
    _collection_round_trip(enc, [nest] + [r[""] if r[""] is not None else [] for r in rows])


def test_reference_map_encoder_shapes():
    from typing import List
    B = reference_beans()
    bar, foo = B["Bar"], B["Foo"]
    # testMapEncoder: Map<String, Bar>, 5 entries
    _collection_round_trip(_map_encoder(I.String, bar), [[(f"i{k}", _bar(k, f"i{k}")) for k in range(5)]])
    # testNestListEncoder: Map<String, List<List<Bar>>>
    nest = [(str(i), [[_bar(k, f"s{k}") for k in range(3)] for _ in range(i)]) for i in range(5)]
    _collection_round_trip(_map_encoder(I.String, List[List[bar]]), [nest])
    # testSimpleNestArrayWithMapEncoder1 / 2, testSimpleStructWithMapEncoder2 (Map<String, Foo>)
    _collection_round_trip(_map_encoder(I.String, List[I.Integer]), [[("k1", [1, 2])]])
    _collection_round_trip(_map_encoder(I.String, List[List[I.Integer]]), [[("k1", [[1, 2], [1, 2]])]])
    _collection_round_trip(_map_encoder(I.String, foo), [[("k1", _foo())]])
    enc = _map_encoder(foo, List[bar])  # random batch, nulls inside
    rows = random_rows(enc.schema(), 400, 8)
    _collection_round_trip(enc, [r[""] if r[""] is not None else [] for r in rows])


def test_nested_corrupt_rows_are_reported_not_faulted():
    """Flipped bytes in nested rows: decode raises CorruptRowException (or decodes
    different values) and never reads or writes outside its buffers; the device stays
    healthy for the next batch."""
    schema, cols = nested_columns("maps_nested", 400, 21)
    enc = encoder_for("maps_nested")
    rows = enc.encode(to_device(cols), 400, 0)
    rng = np.random.default_rng(4)
    raised = 0
    for trial in range(24):
        bad = rows.buffer.clone()
        pos = rng.integers(0, bad.numel(), size=8)
        bad[torch.from_numpy(pos).cuda()] ^= torch.from_numpy(rng.integers(1, 256, size=8).astype(np.uint8)).cuda()
        try:
            enc.decode(EncodedRows(bad, rows.offsets, 400, 0))
        except (CorruptRowException, errors.IndexOutOfBoundsException, errors.EncoderException):
            raised += 1
    assert raised > 0
    assert columns_equal(schema, cols, to_host(enc.decode(rows))) == []


# --- decimal fields (BinaryWriter.writeDecimal, BinaryWriter.java:214-230) ------------
def test_decimal_precision_is_checked_on_the_device():
    """|unscaled| > 10^precision - 1 is the reference's UnsupportedOperationException
    (DecimalUtility.checkPrecisionAndScale inside writeDecimal); the oracle agrees."""
    from fury_amd.format import UnsupportedOperationException
    from fury_amd.format.types import DataTypes, Field
    schema = Schema([Field("d", DataTypes.decimal(10, 2), True), Field("id", DataTypes.int64(), False)])
    rows = [{"d": v, "id": i} for i, v in enumerate([1, 10 ** 10 - 1, -(10 ** 10 - 1), None, 5])]
    enc = RowEncoder(schema)
    cols = build_columns(schema, rows)
    check(schema, enc, cols, len(rows), 1)  # in range: bytes == oracle
    rows[2]["d"] = -(10 ** 10)  # 11 digits
    cols = build_columns(schema, rows)
    with pytest.raises(UnsupportedOperationException):
        enc.encode(to_device(cols), len(rows), 1)
    with pytest.raises(oracle.OracleUnsupported):
        oracle.encode(schema, cols, len(rows), 1)


def test_decimal_beyond_decimal128_is_corrupt():
    """32 row bytes that are not a sign-extended decimal128 cannot land in an Arrow
    decimal128 column: CorruptRowException (the oracle reports the same)."""
    schema, cols = nested_columns("decimals", 64, 3)
    enc = encoder_for("decimals")
    expect, offs = oracle.encode(schema, cols, 64, 0)
    bad = expect.copy()
    # the first non-null top-level decimal of record 0 ("amount", ordinal 0)
    slot = int.from_bytes(bad[8:16].tobytes(), "little")
    assert slot & 0xFFFFFFFF == 32 or slot == 0
    if slot == 0:
        pytest.skip("record 0's amount is null")
    at = slot >> 32
    bad[at + 24] ^= 0x01
    buf = torch.from_numpy(np.concatenate([bad, np.zeros(16, np.uint8)])).cuda()
    with pytest.raises(CorruptRowException):
        enc.decode(buf, 64, 0, torch.from_numpy(offs).cuda())
    with pytest.raises(oracle.OracleError):
        oracle.decode(schema, bad, offs, 64, 0)
