"""GPU: the HIP path (through the C-ABI) is byte-identical to the oracle.

Encode: device bytes == oracle bytes (raw rows and Encoder.encode(MemoryBuffer,T)
frame streams). Decode: device columns == oracle-decoded columns == inputs.
Edge cases follow the reference tests (RowEncoderTest / BinaryRowTest /
CodecBuilderTest): empty batch, single row, tile-boundary sizes, nulls
everywhere, empty strings/lists, schema-hash mismatch, corrupt frames,
undersized buffers. Full-size configs are checked through size-independent
properties (round trip, sampled rows against the oracle).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import oracle  # noqa: E402
from fury_amd import workloads as W  # noqa: E402
from fury_amd.format import (ClassNotCompatibleException, CorruptRowException,  # noqa: E402
                             IndexOutOfBoundsException)
from fury_amd.format.columns import to_device, to_host  # noqa: E402
from fury_amd.format.encoder import CollectionEncoder, EncodedRows, Encoders, RowEncoder  # noqa: E402
from fury_amd.format import native  # noqa: E402
from fury_amd.format.types import ArrowType  # noqa: E402

from helpers import catalog, collection_cases, columns_equal, knob_key  # noqa: E402

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 7, 63, 64, 65, 1000, 4097]
_ENC = {}


def encoder_for(name):
    key = (name, knob_key())  # a plan reads the launch knobs when it is created
    if key not in _ENC:
        _ENC[key] = RowEncoder(catalog()[name][0])
    return _ENC[key]


VARLEN = [k for k, (sch, _) in catalog().items()
          if any(f.type.id in (ArrowType.STRING, ArrowType.BINARY, ArrowType.LIST, ArrowType.STRUCT, ArrowType.MAP)
                 for f in sch.fields)]
FIXED = [k for k in catalog() if k not in VARLEN]


@pytest.fixture(params=["flat", "flat_stg256", "flat_r3enc", "flat_v7", "flat_v9", "flat_v9_nocap", "tile", "global",
                        "spill", "nocap", "tile_nocap", "waves2", "waves4"])
def varlen_engine(request, monkeypatch):
    """Varlen engines: flat cooperative tile kernels (default for flat plans), the
    generic one-wave tile interpreter (FORY_ROWFMT_VARFLAT=0), the per-record global
    interpreter (FORY_ROWFMT_VARTILE=0); a 2 KiB LDS image so tiles spill to the second
    (big-image) launch; 2 KiB for both launches so tiles take the per-record global path
    inside the tile kernels (flat and generic); flat with a 256-byte staging buffer
    (most spans take the per-lane copy); cooperative tiles of 2 / 4 waves forced; flat
    plans encoded by the round-3 tile kernel (FORY_ROWFMT_VARENC=1), encode v7 (=7) and encode
    v9 (=9; with 2 KiB images: its spill and per-record paths)."""
    env = {"flat": {}, "flat_stg256": {"FORY_ROWFMT_VARSTG": "256"}, "flat_r3enc": {"FORY_ROWFMT_VARENC": "1"},
           "flat_v7": {"FORY_ROWFMT_VARENC": "7"}, "flat_v9": {"FORY_ROWFMT_VARENC": "9"},
           "flat_v9_nocap": {"FORY_ROWFMT_VARENC": "9", "FORY_ROWFMT_VARCAP": "2048", "FORY_ROWFMT_SPILLCAP": "2048"},
           "tile": {"FORY_ROWFMT_VARFLAT": "0"}, "global": {"FORY_ROWFMT_VARTILE": "0"},
           "spill": {"FORY_ROWFMT_VARCAP": "2048"},
           "nocap": {"FORY_ROWFMT_VARCAP": "2048", "FORY_ROWFMT_SPILLCAP": "2048"},
           "tile_nocap": {"FORY_ROWFMT_VARFLAT": "0", "FORY_ROWFMT_VARCAP": "2048",
                          "FORY_ROWFMT_SPILLCAP": "2048"},
           "waves2": {"FORY_ROWFMT_VARNW": "2"}, "waves4": {"FORY_ROWFMT_VARNW": "4"}}[request.param]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    return request.param


def check_parity(name, n, frame):
    schema, make = catalog()[name]
    cols = make(n, n)
    expect, offs = oracle.encode(schema, cols, n, frame)
    enc = encoder_for(name)
    rows = enc.encode(to_device(cols), n, frame)
    got = rows.buffer.cpu().numpy()
    assert got.nbytes == expect.nbytes
    if got.nbytes:
        bad = np.nonzero(got != expect)[0]
        assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"
    if rows.offsets is not None:
        assert np.array_equal(rows.offsets.cpu().numpy(), offs)
    dec = to_host(enc.decode(rows))
    assert columns_equal(schema, cols, dec) == []
    # decode of oracle-produced bytes, compared with the oracle's own decode
    ref = oracle.decode(schema, expect, offs, n, frame)
    buf = torch.from_numpy(np.concatenate([expect, np.zeros(16, np.uint8)])).cuda()
    d_offs = None if rows.offsets is None else torch.from_numpy(offs).cuda()
    dec2 = to_host(enc.decode(buf, n, frame, d_offs))
    assert columns_equal(schema, ref, dec2) == []


@pytest.mark.parametrize("frame", [0, 1, 3])
@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("name", FIXED)
def test_encode_decode_parity(name, n, frame):
    check_parity(name, n, frame)


@pytest.mark.parametrize("frame", [0, 1, 3])
@pytest.mark.parametrize("n", SIZES + [5000])
@pytest.mark.parametrize("name", VARLEN)
def test_varlen_parity(name, n, frame, varlen_engine):
    check_parity(name, n, frame)


@pytest.mark.parametrize("n", [0, 1, 63, 65, 4097])
def test_collection_frame_parity(n, varlen_engine):
    """ArrayEncoder / MapEncoder frames (Encoders.java:418-431, 559-572): device bytes ==
    oracle bytes for list<Long>, List<Bean> and Map<Integer, Long>, and both decode back."""
    for schema, cols in collection_cases(n, 7 + n):
        f = schema.fields[0]
        if f.type.id == ArrowType.MAP:
            enc = Encoders.map_encoder(f.children[0], f.children[1])
        else:
            enc = Encoders.array_encoder(f.children[0])
        assert enc.plan.schema_hash == CollectionEncoder(schema).plan.schema_hash  # names do not hash
        expect, offs = oracle.encode(schema, cols, n, 2)
        rows = enc.encode(to_device(cols), n)
        got = rows.buffer.cpu().numpy()
        assert got.nbytes == expect.nbytes
        bad = np.nonzero(got != expect)[0]
        assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"
        assert np.array_equal(rows.offsets.cpu().numpy(), offs)
        assert columns_equal(schema, cols, to_host(enc.decode(rows))) == []
        buf = torch.from_numpy(np.concatenate([expect, np.zeros(16, np.uint8)])).cuda()
        dec = to_host(enc.decode(buf, n, None, torch.from_numpy(offs).cuda()))
        assert columns_equal(schema, cols, dec) == []


@pytest.mark.parametrize("shift", [4, 8, 12])
@pytest.mark.parametrize("name", ["mixed40_nulls", "flat_mix", "nested_nulls", "deep_nested", "maps", "list_struct",
                                  "string_elems"])
def test_varlen_unaligned_buffers(name, shift, varlen_engine):
    """Rows written to / read from buffers at a 4-byte (not 16-byte) aligned address."""
    schema, make = catalog()[name]
    n = 777
    cols = make(n, 11)
    enc = encoder_for(name)
    dcols = to_device(cols)
    arr = native.column_array(dcols)
    ws = enc.workspace(n)
    for frame in (0, 1, 3):
        expect, offs = oracle.encode(schema, cols, n, frame)
        d_offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        native.encoded_size(enc.plan, arr, n, frame, d_offs, ws)
        big = torch.zeros(expect.nbytes + 64, dtype=torch.uint8, device="cuda")
        out = big[shift:]
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        native.encode(enc.plan, arr, n, frame, d_offs, out, status, ws)
        native.read_status(status)
        got = out[:expect.nbytes].cpu().numpy()
        assert np.array_equal(got, expect), frame
        assert int(big[:shift].sum().item()) == 0 and int(big[shift + expect.nbytes:].sum().item()) == 0
        dec = to_host(enc.decode(out[:expect.nbytes], n, frame, d_offs))
        assert columns_equal(schema, cols, dec) == []


def test_schema_mismatch_raises():
    enc = encoder_for("struct104")
    schema, make = catalog()["struct104"]
    cols = make(100, 0)
    rows = enc.encode(to_device(cols), 100, 1)
    bad = rows.buffer.clone()
    bad[860 * 37 + 4] ^= 0x40  # flip a bit of frame 37's schema hash
    with pytest.raises(ClassNotCompatibleException):
        enc.decode(EncodedRows(bad, None, 100, 1, 860))
    bad = rows.buffer.clone()
    bad[860 * 5] = 3  # frame size field
    with pytest.raises(CorruptRowException):
        enc.decode(EncodedRows(bad, None, 100, 1, 860))


def test_varlen_schema_mismatch_raises():
    enc = encoder_for("mixed40")
    schema, make = catalog()["mixed40"]
    cols = make(300, 0)
    rows = enc.encode(to_device(cols), 300, 1)
    bad = rows.buffer.clone()
    o = int(rows.offsets[123].item())
    bad[o + 6] ^= 1
    with pytest.raises(ClassNotCompatibleException):
        enc.decode(EncodedRows(bad, rows.offsets, 300, 1))


def test_capacity_errors():
    enc = encoder_for("struct104")
    schema, make = catalog()["struct104"]
    n = 10
    dcols = to_device(make(n, 0))
    arr = native.column_array(dcols)
    ws = enc.workspace(n)
    out = torch.empty(848 * n - 8, dtype=torch.uint8, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    with pytest.raises(IndexOutOfBoundsException):
        native.encode(enc.plan, arr, n, 0, None, out, status, ws)
    # varlen: device-side capacity check
    enc = encoder_for("mixed40")
    schema, make = catalog()["mixed40"]
    dcols = to_device(make(n, 0))
    arr = native.column_array(dcols)
    ws = enc.workspace(n)
    offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    native.encoded_size(enc.plan, arr, n, 1, offs, ws)
    total = int(offs[n].item())
    out = torch.zeros(total - 1, dtype=torch.uint8, device="cuda")
    native.encode(enc.plan, arr, n, 1, offs, out, status, ws)
    with pytest.raises(IndexOutOfBoundsException):
        native.read_status(status)


def test_struct_large_round_trip_and_sampled_parity():
    """S at 2M rows: device-generated java.util.Random values, round trip exact,
    and 4 sampled tiles compared byte-for-byte with the oracle."""
    n = 2 * 1024 * 1024 + 3
    schema = W.struct_schema()
    enc = encoder_for("struct104")
    vals = W.gen_struct_device(n)
    dcols = [native.DeviceColumn(v, None, None, n) for v in vals]
    for frame in (0, 1, 3):
        rows = enc.encode(dcols, n, frame)
        stride = 848 + {0: 0, 1: 12, 3: 8}[frame]
        for r0 in (0, 12345, n // 2, n - 70):
            cnt = min(64, n - r0)
            host = W.struct_host_columns(cnt, row0=r0)
            expect, _ = oracle.encode(schema, host, cnt, frame)
            got = rows.buffer[r0 * stride:(r0 + cnt) * stride].cpu().numpy()
            assert np.array_equal(got, expect), (frame, r0)
        dec = enc.decode(rows)
        for a, b in zip(dec, dcols):
            assert torch.equal(a.values[:n].view(torch.uint8), b.values.view(torch.uint8))


@pytest.mark.parametrize("name", ["struct104_boxed", "all_types"])
def test_nullable_fixed_many_tiles_parity(name):
    """Nullable fixed-width schemas on the persistent v5 kernels: 200K records are
    several tiles per workgroup, so the per-tile re-zeroing of the LDS null bitmaps
    (encode) and the validity words of later tiles (decode) are exercised; every frame
    mode byte-identical to the oracle, oracle bytes decode to the oracle's columns."""
    schema, make = catalog()[name]
    n = 200_000 + 37
    cols = make(n, 11)
    enc = encoder_for(name)
    for frame in (0, 1, 3):
        expect, offs = oracle.encode(schema, cols, n, frame)
        rows = enc.encode(to_device(cols), n, frame)
        got = rows.buffer.cpu().numpy()
        bad = np.nonzero(got != expect)[0]
        assert len(bad) == 0, f"frame {frame}: {len(bad)} bytes differ, first at {bad[:8]}"
        assert columns_equal(schema, cols, to_host(enc.decode(rows))) == []
        buf = torch.from_numpy(np.concatenate([expect, np.zeros(16, np.uint8)])).cuda()
        ref = oracle.decode(schema, expect, offs, n, frame)
        assert columns_equal(schema, ref, to_host(enc.decode(buf, n, frame, None))) == []


@pytest.mark.parametrize("shift", [1, 4])
def test_nullable_fixed_unaligned_validity(shift):
    """Validity buffers at odd / 4-byte offsets (the NUL v5 encode reads each chunk's
    validity byte(s) at any alignment): bytes still equal the oracle's."""
    schema, make = catalog()["struct104_boxed"]
    n = 64 * 40 + 9
    cols = make(n, 13)
    enc = encoder_for("struct104_boxed")
    dcols, keep = [], []
    for c in to_device(cols):
        if c.validity is not None:
            big = torch.zeros(c.validity.numel() + 16, dtype=torch.uint8, device="cuda")
            big[shift:shift + c.validity.numel()] = c.validity
            keep.append(big)
            c.validity = big[shift:shift + c.validity.numel()]
        dcols.append(c)
    for frame in (0, 1):
        expect, _ = oracle.encode(schema, cols, n, frame)
        got = enc.encode(dcols, n, frame).buffer.cpu().numpy()
        assert np.array_equal(got, expect), frame


def test_mixed_and_nested_large_round_trip(varlen_engine):
    for name, n in (("mixed40_nulls", 300_000), ("nested_nulls", 300_000), ("flat_mix", 100_000)):
        schema, make = catalog()[name]
        cols = make(n, 5)
        enc = encoder_for(name)
        rows = enc.encode(to_device(cols), n, 1)
        dec = to_host(enc.decode(rows))
        assert columns_equal(schema, cols, dec) == []
        expect, offs = oracle.encode(schema, cols, n, 1)
        assert np.array_equal(rows.buffer.cpu().numpy(), expect)


def test_hashed_frames_schema_mismatch_raises():
    """Encoder.decode(byte[]) checks the [i64 hash] prefix (Encoders.java:181-190, 195-197)."""
    for name in ("struct104", "mixed40", "nested"):
        enc = encoder_for(name)
        schema, make = catalog()[name]
        cols = make(200, 1)
        rows = enc.encode(to_device(cols), 200, 3)
        bad = rows.buffer.clone()
        o = 0 if rows.offsets is None else int(rows.offsets[77].item())
        if rows.offsets is None:
            o = 77 * rows.stride
        bad[o + 3] ^= 0x04
        with pytest.raises(ClassNotCompatibleException):
            enc.decode(EncodedRows(bad, rows.offsets, 200, 3, rows.stride))


@pytest.mark.parametrize("shift", [0, 8, 24])
def test_fixed_decode_into_unaligned_columns(shift):
    """Decode v5 stores 16-B column chunks: output columns that are not 16-byte aligned
    take the one-tile kernel; both give the input columns back (tail tile included)."""
    schema, make = catalog()["struct104"]
    n = 64 * 37 + 5
    cols = make(n, 3)
    enc = encoder_for("struct104")
    rows = enc.encode(to_device(cols), n, 0)
    outs, backing = [], []
    for c in enc.alloc_fixed_outputs(n):
        k = c.values.element_size()
        big = torch.empty(n * k + 64, dtype=torch.uint8, device="cuda")
        backing.append(big)
        c.values = big[shift:shift + n * k].view(c.values.dtype)
        outs.append(c)
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    native.decode(enc.plan, rows.buffer, None, n, 0, native.column_array(outs), status, enc.workspace(n))
    native.read_status(status)
    assert columns_equal(schema, cols, to_host(outs)) == []
