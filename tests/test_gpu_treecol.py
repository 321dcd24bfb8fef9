"""GPU: the columnar tree engine (fury_amd/csrc/treecol.hip) at its edges.

Nested shapes are sized node by node and written node by node (rows, then each var
node's instances at the positions their parents handed down); these tests take it to
rows of ~100 KiB among small ones, containers of thousands of items, collection
frames, the workspace contract (encode_workspace_bytes vs workspace_bytes) and the
sizes encode reuses from encoded_size (and must not reuse after another call wrote the
workspace). Every output is compared byte for byte with the
oracle (oracle/rowfmt_oracle.c, BaseBinaryEncoderBuilder.serializeFor's layout).
"""
from typing import Dict, List

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import oracle  # noqa: E402
from fury_amd.format import errors, native  # noqa: E402
from fury_amd.format.columns import build_columns, to_device  # noqa: E402
from fury_amd.format.encoder import CollectionEncoder, RowEncoder  # noqa: E402
from fury_amd.format.types import DataTypes, Schema  # noqa: E402
from fury_amd.format import infer as I  # noqa: E402

from helpers import nested_columns, nested_schemas, random_rows, reference_beans  # noqa: E402

pytestmark = pytest.mark.gpu


def oracle_equal(schema, cols, n, frame, rows):
    expect, offs = oracle.encode(schema, cols, n, frame)
    got = rows.buffer.cpu().numpy()
    assert got.nbytes == expect.nbytes
    bad = np.nonzero(got != expect)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"
    assert np.array_equal(rows.offsets.cpu().numpy(), offs)


def _big_rows_schema():
    return I.infer_schema(type("Big", (), {"__annotations__": {
        "id": I.jint, "names": List[I.String], "grid": List[List[I.jshort]], "tag": I.String}}))


@pytest.mark.parametrize("frame", [0, 1, 3])
def test_rows_of_100k_among_small_ones(frame):
    """A few rows of ~100 KiB (3000 strings) among small ones (one workgroup's items
    span thousands of elements); oracle bytes."""
    schema = _big_rows_schema()
    rng = np.random.default_rng(1)
    rows = []
    for i in range(600):
        big = i % 97 == 5
        k = 3000 if big else int(rng.integers(0, 4))
        rows.append({"id": i, "names": [("s%d" % j) * int(rng.integers(1, 8)) for j in range(k)],
                     "grid": [[int(x) for x in rng.integers(-9, 9, size=int(rng.integers(0, 4)))]
                              for _ in range(int(rng.integers(0, 3)))],
                     "tag": None if i % 5 == 0 else "t%d" % i})
    cols = build_columns(schema, rows)
    enc = RowEncoder(schema)
    oracle_equal(schema, cols, len(rows), frame, enc.encode(to_device(cols), len(rows), frame))


def test_rows_of_thousands_of_lists():
    """Rows of ~6000 short lists each (inner lists of one item, 6000 per outer list)."""
    schema = _big_rows_schema()
    rows = [{"id": i, "names": [], "grid": [[i % 7] for _ in range(6000 if i % 3 == 0 else 2)], "tag": "x"}
            for i in range(40)]
    cols = build_columns(schema, rows)
    enc = RowEncoder(schema)
    oracle_equal(schema, cols, len(rows), 1, enc.encode(to_device(cols), len(rows), 1))


def test_collection_frames_columnar():
    """ArrayEncoder / MapEncoder frames of nested collections (List<List<String>>,
    Map<String, List<Bar>>) at 3000 records."""
    B = reference_beans()
    for schema in (
        Schema([DataTypes.array_field("", I._infer_field("item", List[I.String], []))]),
        Schema([DataTypes.map_field("", type(k := I._infer_field("key", I.String, []))(k.name, k.type, False, k.children),
                                    I._infer_field("value", List[B["Bar"]], []))]),
    ):
        enc = CollectionEncoder(schema)
        rows = random_rows(schema, 3000, 7)
        for r in rows:  # collection frames encode a null collection from its (empty) offsets
            if r[""] is None:
                r[""] = []
        cols = build_columns(schema, rows)
        oracle_equal(schema, cols, 3000, 2, enc.encode(to_device(cols), 3000))


def _native_encode(enc, dcols, n, frame, ws, offs_from=None):
    p = enc.plan
    arr = native.column_array(dcols)
    offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    if offs_from is None:
        native.encoded_size(p, arr, n, frame, offs, ws)
    else:
        offs.copy_(offs_from)
    total = int(offs[n].item())
    out = torch.empty(max(16, total), dtype=torch.uint8, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    native.encode(p, arr, n, frame, offs, out, status, ws)
    native.read_status(status)
    return out[:total], offs


@pytest.mark.parametrize("name", ["holder", "bean_a", "maps_nested"])
def test_workspace_contract_selects_the_engine(name):
    """workspace_bytes keeps the per-record engine, encode_workspace_bytes enables the
    columnar one (larger: per-node temporaries); both give the oracle's bytes."""
    schema, cols = nested_columns(name, 900, 3)
    enc = RowEncoder(schema)
    dcols = to_device(cols)
    arr = native.column_array(dcols)
    small, big = enc.plan.workspace_bytes(900), enc.plan.encode_workspace_bytes(arr, 900)
    assert big > small
    expect, offs = oracle.encode(schema, cols, 900, 1)
    for nbytes in (small, big):
        ws = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        out, got_offs = _native_encode(enc, dcols, 900, 1, ws)
        assert np.array_equal(out.cpu().numpy(), expect)
        assert np.array_equal(got_offs.cpu().numpy(), offs)


def test_encode_does_not_reuse_sizes_another_call_overwrote():
    """encoded_size(A); encoded_size(B) on the same workspace; encode(A) with A's
    offsets: the sizes in the workspace are B's, so encode recomputes A's. Likewise
    after a decode wrote the workspace."""
    schema = nested_schemas()["holder"]
    enc = RowEncoder(schema)
    _, ca = nested_columns("holder", 500, 11)
    _, cb = nested_columns("holder", 500, 12)
    da, db = to_device(ca), to_device(cb)
    arr_a = native.column_array(da)
    ws = torch.empty(enc.plan.encode_workspace_bytes(arr_a, 500) * 2, dtype=torch.uint8, device="cuda")
    expect_a, offs_a = oracle.encode(schema, ca, 500, 0)
    _, offs = _native_encode(enc, da, 500, 0, ws)
    _native_encode(enc, db, 500, 0, ws)  # B's sizes now in the workspace
    out, _ = _native_encode(enc, da, 500, 0, ws, offs_from=offs)
    assert np.array_equal(out.cpu().numpy(), expect_a)
    # encoded_size(A), then a decode through the same workspace, then encode(A)
    _, offs = _native_encode(enc, da, 500, 0, ws)
    rows = enc.encode(db, 500, 0)
    p = enc.plan
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    outc = enc.decode(rows)  # output columns of the right shape; then a decode_sizes through ws
    native.decode_sizes(p, rows.buffer, rows.offsets, 500, 0, native.column_array(outc), status, ws)
    out, _ = _native_encode(enc, da, 500, 0, ws, offs_from=offs)
    assert np.array_equal(out.cpu().numpy(), expect_a)


def test_capacity_short_by_one_row_is_reported():
    schema, cols = nested_columns("bean_a", 300, 4)
    enc = RowEncoder(schema)
    dcols = to_device(cols)
    p = enc.plan
    arr = native.column_array(dcols)
    ws = torch.empty(p.encode_workspace_bytes(arr, 300), dtype=torch.uint8, device="cuda")
    offs = torch.empty(301, dtype=torch.int64, device="cuda")
    native.encoded_size(p, arr, 300, 1, offs, ws)
    total = int(offs[300].item())
    out = torch.empty(total, dtype=torch.uint8, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    native.encode(p, arr, 300, 1, offs, out, status, ws, capacity=total - 8)
    with pytest.raises(errors.IndexOutOfBoundsException):
        native.read_status(status)


@pytest.mark.parametrize("name", ["holder", "lists", "maps_nested", "bean_a", "deep", "decimals", "chain"])
def test_columnar_large_batch(name):
    """20k records per shape (thousands of tiles) in STREAM frames."""
    n = 2000 if name == "chain" else 20_000
    schema, cols = nested_columns(name, n, 21)
    enc = RowEncoder(schema)
    oracle_equal(schema, cols, n, 1, enc.encode(to_device(cols), n, 1))


@pytest.mark.parametrize("name", ["holder", "lists", "maps_nested", "bean_a", "chain"])
def test_decode_levels_resume_from_the_previous_call(name):
    """decode_sizes sizes one level per call; on one workspace a call resumes after the
    levels the previous call ran (same plan, rows and columns). The columns equal the
    input with: one big workspace (every call resumes), a fresh workspace per call (none
    does), and a decode of other rows through the same workspace between the levels (its
    positions must not be taken for these rows')."""
    from helpers import columns_equal
    from fury_amd.format.columns import to_host
    n = 60 if name == "chain" else 700
    schema, cols = nested_columns(name, n, 31)
    _, other = nested_columns(name, n, 32)
    enc = RowEncoder(schema)
    rows = enc.encode(to_device(cols), n, 1)
    rows_b = enc.encode(to_device(other), n, 1)
    enc._ws = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
    assert columns_equal(schema, cols, to_host(enc.decode(rows))) == []
    keep = []

    def fresh(m, c=None, decode=False):
        need = enc.plan.decode_workspace_bytes(c, m) if decode else enc.plan.workspace_bytes(m)
        keep.append(torch.empty(max(256, need), dtype=torch.uint8, device="cuda"))
        return keep[-1]

    big = enc._ws
    enc.workspace = fresh
    assert columns_equal(schema, cols, to_host(enc.decode(rows))) == []
    calls = []

    def interleaved(m, c=None, decode=False):  # every other call: a full decode of rows_b first
        calls.append(1)
        if decode and len(calls) % 2 == 0:
            enc.workspace = lambda *a, **k: big
            enc.decode(rows_b)
            enc.workspace = interleaved
        return big

    enc.workspace = interleaved
    assert columns_equal(schema, cols, to_host(enc.decode(rows))) == []


@pytest.mark.parametrize("frame", [0, 1])
def test_long_strings_decode_both_copy_paths(frame):
    """String columns whose 256-value workgroups span more than the LDS image (values of
    100-300 bytes: the dword-by-dword copy) next to short ones (the staged copy), with
    nulls and empty strings; encode bytes and the decoded columns equal the oracle's."""
    from helpers import columns_equal
    from fury_amd.format.columns import to_host
    schema = I.infer_schema(type("LongStrings", (), {"__annotations__": {
        "id": I.jint, "long": List[List[I.String]], "short": List[I.String], "tag": I.String}}))  # (list<list<>>: the tree engine)
    rng = np.random.default_rng(7)
    rows = []
    for i in range(1500):
        rows.append({"id": i,
                     "long": [[None if rng.random() < 0.1 else "x" * int(rng.integers(100, 300))
                               for _ in range(int(rng.integers(0, 4)))] for _ in range(int(rng.integers(0, 3)))],
                     "short": ["" if rng.random() < 0.2 else "s%d" % int(rng.integers(0, 999))
                               for _ in range(int(rng.integers(0, 9)))],
                     "tag": None if i % 7 == 0 else "t" * (i % 300)})
    cols = build_columns(schema, rows)
    enc = RowEncoder(schema)
    encoded = enc.encode(to_device(cols), len(rows), frame)
    oracle_equal(schema, cols, len(rows), frame, encoded)
    assert columns_equal(schema, cols, to_host(enc.decode(encoded))) == []


def _refilled(rows, seed):
    """The same rows with every string replaced by one of another length (list / map
    lengths unchanged, so every column keeps its length)."""
    import copy
    rng = np.random.default_rng(seed)

    def walk(v):
        if isinstance(v, str):
            return "r" * int(rng.integers(0, 40))
        if isinstance(v, list):
            return [walk(x) for x in v]
        if isinstance(v, tuple):  # map entries
            return tuple(walk(x) for x in v)
        if isinstance(v, dict):
            return {k: walk(x) for k, x in v.items()}
        if hasattr(v, "__dict__"):
            o = copy.copy(v)
            o.__dict__.update({k: walk(x) for k, x in v.__dict__.items()})
            return o
        return v

    return [walk(r) for r in rows]


def test_encode_after_in_place_refill_uses_current_sizes():
    """encode(A, ws); A refilled in place (same pointers and lengths, other string sizes);
    encoded_size on another workspace; encode(A, ws): the bytes are the refilled rows'
    (encode leaves no sizes of its own for a later encode to reuse)."""
    schema = nested_schemas()["holder"]
    enc = RowEncoder(schema)
    rows_a = random_rows(schema, 400, 41)
    rows_b = _refilled(rows_a, 42)
    ca, cb = build_columns(schema, rows_a), build_columns(schema, rows_b)
    for a, b in zip(ca, cb):
        assert a.length == b.length
    # device buffers big enough for either contents: pad every values array to the larger
    for a, b in zip(ca, cb):
        if a.values is not None and b.values is not None and b.values.nbytes > a.values.nbytes:
            a.values = np.concatenate([a.values, np.zeros(b.values.nbytes - a.values.nbytes, np.uint8).view(a.values.dtype)])
    da = to_device(ca)
    arr = native.column_array(da)
    ws = torch.empty(enc.plan.encode_workspace_bytes(arr, 400), dtype=torch.uint8, device="cuda")
    ws2 = torch.empty_like(ws)
    out, _ = _native_encode(enc, da, 400, 1, ws)
    expect_a, _ = oracle.encode(schema, ca, 400, 1)
    assert np.array_equal(out.cpu().numpy(), expect_a)
    # refill A in place with B's contents
    for d, b in zip(da, cb):
        for name in ("values", "offsets", "validity"):
            t, h = getattr(d, name), getattr(b, name)
            if t is not None and h is not None:
                src = torch.from_numpy(np.ascontiguousarray(h).view(np.uint8).copy()).cuda()
                t.view(torch.uint8)[:src.numel()].copy_(src)
    _, offs_b = _native_encode(enc, da, 400, 1, ws2)  # sizes of the refilled columns, elsewhere
    out, _ = _native_encode(enc, da, 400, 1, ws, offs_from=offs_b)
    expect_b, _ = oracle.encode(schema, cb, 400, 1)
    assert np.array_equal(out.cpu().numpy(), expect_b)


def test_short_item_column_is_an_error_not_a_shorter_array():
    """An item column whose fory_column.length is shorter than its list's offsets reach:
    encode reports FORY_ERR_INVALID_ARGUMENT (the items were dropped with
    FORY_OK), decode reports FORY_ERR_CAPACITY and writes nothing past the column."""
    schema = nested_schemas()["holder"]
    enc = RowEncoder(schema)
    rows = random_rows(schema, 300, 43)
    cols = build_columns(schema, rows)
    dcols = to_device(cols)
    p = enc.plan
    # the deepest list-item column with items: shorten its length by one
    kinds = [f for f in _preorder_fields(schema)]
    items = [i for i, f in enumerate(kinds) if i > 0 and kinds[i - 1].type.id == 25 and cols[i].length > 1]
    assert items
    it = items[0]
    short = [native.DeviceColumn(c.values, c.offsets, c.validity, c.length) for c in dcols]
    short[it] = native.DeviceColumn(dcols[it].values, dcols[it].offsets, dcols[it].validity, cols[it].length - 1)
    arr = native.column_array(short)
    ws = torch.empty(p.encode_workspace_bytes(arr, 300), dtype=torch.uint8, device="cuda")
    offs = torch.empty(301, dtype=torch.int64, device="cuda")
    native.encoded_size(p, arr, 300, 0, offs, ws)
    total = int(offs[300].item())
    out = torch.empty(max(16, total), dtype=torch.uint8, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    native.encode(p, arr, 300, 0, offs, out, status, ws)
    with pytest.raises(errors.IllegalArgumentException):  # FORY_ERR_INVALID_ARGUMENT
        native.read_status(status)
    # decode into output columns whose item column is one short, with a guard behind it
    good = enc.encode(dcols, 300, 0)
    outc = enc.decode(good)
    guard = torch.full((4096,), 0x5A, dtype=torch.uint8, device="cuda")
    oc = list(outc)
    w = outc[it].values.element_size() if outc[it].values is not None else 0
    if w:
        buf = torch.cat([outc[it].values.view(torch.uint8)[:(cols[it].length - 1) * w], guard])
        oc[it] = native.DeviceColumn(buf.view(outc[it].values.dtype) if w in (1, 2, 4, 8) else buf, outc[it].offsets,
                                     outc[it].validity, cols[it].length - 1)
    else:
        oc[it] = native.DeviceColumn(outc[it].values, outc[it].offsets, outc[it].validity, cols[it].length - 1)
    darr = native.column_array(oc)
    dws = torch.empty(max(p.decode_workspace_bytes(darr, 300), 1 << 20), dtype=torch.uint8, device="cuda")
    status.zero_()
    native.decode_sizes(p, good.buffer, good.offsets, 300, 0, darr, status, dws)
    native.decode(p, good.buffer, good.offsets, 300, 0, darr, status, dws)
    with pytest.raises(errors.IndexOutOfBoundsException):  # FORY_ERR_CAPACITY
        native.read_status(status)
    if w:
        assert bool((buf[(cols[it].length - 1) * w:] == 0x5A).all())


def _preorder_fields(schema):
    out = []

    def walk(f):
        out.append(f)
        for c in f.children:
            walk(c)

    for f in schema.fields:
        walk(f)
    return out
