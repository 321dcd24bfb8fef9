"""GPU: encode v9 at the edges the benchmark plans do not reach — fixed
columns with validity (its NUL template bit 1), plans without any validity (NUL 0), two
var fields (two waves per tile), strings longer than the 32 bytes it carries in flight
(the chunk loop), binary values, empty and all-null strings — against the oracle, forced
(FORY_ROWFMT_VARENC=9) and by default, raw rows and frame streams, tile-boundary sizes."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import oracle  # noqa: E402
from fury_amd.format.columns import build_columns, to_device, to_host  # noqa: E402
from fury_amd.format.encoder import RowEncoder  # noqa: E402
from fury_amd.format.types import ArrowType, DataType, Field, Schema  # noqa: E402

from helpers import columns_equal  # noqa: E402

pytestmark = pytest.mark.gpu


def _schema(kind):
    if kind == "nullable_fixed":  # NUL = 3: fixed and var validity
        return Schema([Field("a", DataType(ArrowType.INT32), True), Field("b", DataType(ArrowType.INT64), True),
                       Field("c", DataType(ArrowType.DOUBLE), False), Field("d", DataType(ArrowType.INT8), True),
                       Field("e", DataType(ArrowType.BOOL), True), Field("f", DataType(ArrowType.STRING), True),
                       Field("g", DataType(ArrowType.BINARY), False), Field("h", DataType(ArrowType.INT16), False),
                       Field("i", DataType(ArrowType.STRING), True)])
    if kind == "no_validity":  # NUL = 0
        return Schema([Field("a", DataType(ArrowType.INT64), False), Field("s", DataType(ArrowType.STRING), False),
                       Field("t", DataType(ArrowType.STRING), False), Field("u", DataType(ArrowType.FLOAT), False)])
    # two var fields, long strings: two waves per tile
    return Schema([Field("k", DataType(ArrowType.INT32), False), Field("x", DataType(ArrowType.STRING), True),
                   Field("y", DataType(ArrowType.STRING), True)])


def _rows(schema, n, seed):
    rng = np.random.default_rng(seed)
    rows = []
    for _ in range(n):
        r = {}
        for f in schema.fields:
            t = f.type.id
            null = f.nullable and rng.random() < 0.2
            if t == ArrowType.STRING:
                ln = int(rng.integers(0, 200)) if rng.random() < 0.4 else int(rng.integers(0, 33))
                v = "".join(chr(int(c)) for c in rng.integers(32, 127, size=ln))
            elif t == ArrowType.BINARY:
                v = bytes(int(c) for c in rng.integers(0, 256, size=int(rng.integers(0, 70))))
            elif t == ArrowType.BOOL:
                v = bool(rng.random() < 0.5)
            elif t == ArrowType.DOUBLE or t == ArrowType.FLOAT:
                v = float(rng.standard_normal())
            else:
                bits = {ArrowType.INT8: 7, ArrowType.INT16: 15, ArrowType.INT32: 31, ArrowType.INT64: 62}[t]
                v = int(rng.integers(-2**bits, 2**bits))
            r[f.name] = None if null else v
        rows.append(r)
    return rows


@pytest.mark.parametrize("forced", [True, False])
@pytest.mark.parametrize("frame", [0, 1])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 128, 129, 1000, 4097])
@pytest.mark.parametrize("kind", ["nullable_fixed", "no_validity", "two_long"])
def test_v9_edges(kind, n, frame, forced, monkeypatch):
    if forced:
        monkeypatch.setenv("FORY_ROWFMT_VARENC", "9")
    schema = _schema(kind)
    cols = build_columns(schema, _rows(schema, n, 11 + n))
    expect, offs = oracle.encode(schema, cols, n, frame)
    enc = RowEncoder(schema)
    rows = enc.encode(to_device(cols), n, frame)
    got = rows.buffer.cpu().numpy()
    assert got.nbytes == expect.nbytes
    bad = np.nonzero(got != expect)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"
    assert columns_equal(schema, cols, to_host(enc.decode(rows))) == []


def test_v9_all_null_and_empty_strings(monkeypatch):
    monkeypatch.setenv("FORY_ROWFMT_VARENC", "9")
    schema = _schema("two_long")
    n = 300
    rows = [{"k": i, "x": None if i % 2 else "", "y": None} for i in range(n)]
    cols = build_columns(schema, rows)
    expect, _ = oracle.encode(schema, cols, n, 0)
    enc = RowEncoder(schema)
    got = enc.encode(to_device(cols), n, 0).buffer.cpu().numpy()
    assert np.array_equal(got, expect)


@pytest.mark.parametrize("kind", ["nullable_fixed", "no_validity", "two_long"])
def test_v9_is_the_kernel_that_ran(kind, monkeypatch, capfd):
    """These plans take encode v9 by default (FORY_ROWFMT_VARDIAG names the launch)."""
    monkeypatch.setenv("FORY_ROWFMT_VARDIAG", "1")
    schema = _schema(kind)
    n = 4097
    cols = build_columns(schema, _rows(schema, n, 5))
    RowEncoder(schema).encode(to_device(cols), n, 0)
    torch.cuda.synchronize()
    assert "encode v9 tile kernel" in capfd.readouterr().err


@pytest.mark.parametrize("delta", [+24, -8, +300])
def test_v9_offsets_from_other_columns_are_an_encoder_error(delta):
    """encode with row offsets that encoded_size computed for other contents (a string's
    length changed since): the record's bytes would overrun its row. v9 writes nothing of
    it, does not store its tile and reports FORY_ERR_ENCODER; the other tiles are intact
    and nothing lands outside the rows."""
    from fury_amd.format import native
    from fury_amd.format.errors import EncoderException
    schema = _schema("no_validity")
    n = 1000
    rows = _rows(schema, n, 3)
    rows[500]["s"] = "q" * 40
    cols_a = build_columns(schema, rows)
    changed = [dict(r) for r in rows]
    changed[500]["s"] = "q" * (40 + delta)
    cols_b = build_columns(schema, changed)
    expect, offs = oracle.encode(schema, cols_a, n, 0)
    total = int(offs[n])
    enc = RowEncoder(schema)
    dev_b = to_device(cols_b)
    arr = native.column_array(dev_b)
    d_offs = torch.from_numpy(offs).cuda()
    out = torch.full((total + 4096,), 0xAB, dtype=torch.uint8, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    native.encode(enc.plan, arr, n, 0, d_offs, out, status, enc.workspace(n, arr))
    with pytest.raises(EncoderException):
        native.read_status(status)
    got = out.cpu().numpy()
    assert (got[total:] == 0xAB).all()
    t0, t1 = int(offs[448]), int(offs[512])  # record 500's tile: not stored
    assert (got[t0:t1] == 0xAB).all()
    assert np.array_equal(got[:t0], expect[:t0]) and np.array_equal(got[t1:total], expect[t1:total])
