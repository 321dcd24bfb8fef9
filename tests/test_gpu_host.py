"""GPU: the host-memory path (fory_rowfmt_host_*, C++ chunk pipeline over three HIP
streams) produces the oracle's bytes from host columns and decodes host rows back,
across chunk boundaries (partial last chunk), both framings, nullable fields, and
reports the reference's errors (schema-hash mismatch, capacity)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import oracle  # noqa: E402
from fury_amd.format import ClassNotCompatibleException, IndexOutOfBoundsException  # noqa: E402
from fury_amd.format.columns import HostColumn, NP_DTYPE, validity_bytes  # noqa: E402
from fury_amd.format.native import HostPipeline, NativePlan, host_register, host_unregister  # noqa: E402
from fury_amd.format.types import preorder  # noqa: E402

from helpers import catalog, collection_cases, columns_equal  # noqa: E402

pytestmark = pytest.mark.gpu


def empty_like(schema, n):
    out = []
    for f in preorder(schema):
        out.append(HostColumn(np.zeros(max(1, n), NP_DTYPE[f.type.id]), None,
                              np.zeros(validity_bytes(n), np.uint8) if f.nullable else None, n))
    return out


@pytest.mark.parametrize("frame", [0, 1])
@pytest.mark.parametrize("n", [1, 63, 1024, 5000])
@pytest.mark.parametrize("name", ["struct104", "all_types", "struct104_boxed"])
def test_host_pipeline_parity(name, n, frame):
    schema, make = catalog()[name]
    cols = make(n, n + 7)
    expect, _ = oracle.encode(schema, cols, n, frame)
    plan = NativePlan(schema)
    hp = HostPipeline(plan, chunk_rows=1000)  # rounds to 1024: several chunks + a partial one
    out = np.zeros(expect.nbytes, np.uint8)
    hp.encode(cols, n, frame, out)
    bad = np.nonzero(out != expect)[0]
    if len(bad):
        stride = expect.nbytes // n
        rows = np.unique(bad // stride)
        r0 = rows[0]
        rb = bad[bad // stride == r0] - r0 * stride
        detail = (f"rows {rows[:6]}..{rows[-3:]} ({len(rows)}), zeros in out: {int((out[bad] == 0).sum())}, "
                  f"row {r0} bad byte offsets {rb[:64].tolist()}, got {out[bad[:8]]}, expected {expect[bad[:8]]}")
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}: {detail}"
    dec = empty_like(schema, n)
    hp.decode(expect, n, frame, dec)
    assert columns_equal(schema, cols, dec) == []
    hp.close()


def test_host_pipeline_registered_buffers_and_errors():
    schema, make = catalog()["struct104"]
    n = 3000
    cols = make(n, 3)
    plan = NativePlan(schema)
    hp = HostPipeline(plan, chunk_rows=512)
    out = np.zeros(n * plan.stride(1), np.uint8)
    host_register(out)
    try:
        hp.encode(cols, n, 1, out)
        expect, _ = oracle.encode(schema, cols, n, 1)
        assert np.array_equal(out, expect)
        with pytest.raises(IndexOutOfBoundsException):
            hp.encode(cols, n, 1, out[:-1])
        bad = out.copy()
        bad[4 + 2000 * plan.stride(1)] ^= 1  # schema hash of frame 2000 (Encoders.java:182-190)
        with pytest.raises(ClassNotCompatibleException):
            hp.decode(bad, n, 1, empty_like(schema, n))
    finally:
        host_unregister(out)
        hp.close()


VARLEN_HOST = ["mixed40_nulls", "nested_nulls", "strings_lists", "flat_mix", "deep_nested", "maps", "list_struct",
               "string_elems"]


@pytest.mark.parametrize("chunk", [1 << 20, 1024])
@pytest.mark.parametrize("frame", [0, 1])
@pytest.mark.parametrize("n", [0, 1, 777, 5000])
@pytest.mark.parametrize("name", VARLEN_HOST)
def test_host_varlen_parity(name, n, frame, chunk):
    """fory_rowfmt_host_encode_var / decode_var: host columns -> the oracle's rows and row
    offsets (one chunk, or 1024-row chunks: slices of every nested column at their
    parents' offsets); host rows -> the input columns (device buffers kept in the ctx)."""
    schema, make = catalog()[name]
    cols = make(n, n + 3)
    expect, eoffs = oracle.encode(schema, cols, n, frame)
    hp = HostPipeline(NativePlan(schema), chunk_rows=chunk)
    rows, offs = hp.encode_var(cols, n, frame)  # starts from a 1-byte buffer: capacity error, grow, retry
    assert rows.nbytes == expect.nbytes
    bad = np.nonzero(rows != expect)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"
    assert np.array_equal(offs, eoffs)
    dec = hp.decode_var(expect, eoffs, n, frame)
    assert columns_equal(schema, cols, dec) == []
    # the context's buffers are reused (and grown) across calls
    rows2, _ = hp.encode_var(cols, n, frame, np.zeros(expect.nbytes + 8, np.uint8))
    assert np.array_equal(rows2, expect)
    hp.close()


def test_host_varlen_collection_frames():
    for schema, cols in collection_cases(900, 21):
        n = cols[0].length
        expect, eoffs = oracle.encode(schema, cols, n, 2)
        hp = HostPipeline(NativePlan(schema), chunk_rows=256)
        rows, offs = hp.encode_var(cols, n, 2)
        assert np.array_equal(rows, expect) and np.array_equal(offs, eoffs)
        assert columns_equal(schema, cols, hp.decode_var(expect, eoffs, n, 2)) == []
        assert columns_equal(schema, cols, hp.decode_var_into(expect, eoffs, n, 2)) == []


def test_host_varlen_errors():
    schema, make = catalog()["mixed40"]
    n = 300
    cols = make(n, 1)
    expect, eoffs = oracle.encode(schema, cols, n, 1)
    hp = HostPipeline(NativePlan(schema))
    bad = expect.copy()
    bad[int(eoffs[17]) + 5] ^= 1  # a frame's schema hash
    with pytest.raises(ClassNotCompatibleException):
        hp.decode_var(bad, eoffs, n, 1)
    with pytest.raises(IndexOutOfBoundsException):  # host_encode on a varlen ctx is refused; capacity:
        import ctypes
        from fury_amd import _lib
        from fury_amd.format.native import _check
        total = ctypes.c_int64(0)
        small = np.zeros(100, np.uint8)
        _check(_lib.load().fory_rowfmt_host_encode_var(hp.handle, hp._host_array(cols), n, 1, small.ctypes.data,
                                                        small.nbytes, None, ctypes.byref(total)))
    assert total.value == expect.nbytes


def test_host_varlen_staged_decode_is_dropped_by_an_encode():
    """A context serves one call at a time: an encode between decode_var_sizes and
    decode_var reuses the staged device buffers, so decode_var must refuse (not
    decode the encode's bytes or read freed memory)."""
    from fury_amd.format import IllegalArgumentException
    schema, make = catalog()["mixed40_nulls"]
    n = 2000
    cols = make(n, 9)
    expect, eoffs = oracle.encode(schema, cols, n, 1)
    hp = HostPipeline(NativePlan(schema))
    counts, nbytes = hp.decode_var_sizes(expect, eoffs, n, 1)
    big = make(4 * n, 10)  # grows the context's buffers
    hp.encode_var(big, 4 * n, 1)
    with pytest.raises(IllegalArgumentException):
        hp.decode_var_finish(counts, nbytes)
    # a fresh sizes call makes it decodable again
    counts, nbytes = hp.decode_var_sizes(expect, eoffs, n, 1)
    assert columns_equal(schema, cols, hp.decode_var_finish(counts, nbytes)) == []
    hp.close()


@pytest.mark.parametrize("name", ["mixed40_nulls", "nested_nulls", "maps"])
def test_host_varlen_decode_of_a_sub_range(name):
    """Rows k.. of a stream whose first row starts at a non-16-byte-aligned offset: the
    device sees the host buffer's phase, offsets rebased to the staged run."""
    schema, make = catalog()[name]
    n = 1500
    cols = make(n, 4)
    for frame in (0, 1):
        expect, eoffs = oracle.encode(schema, cols, n, frame)
        k = next(j for j in range(1, n) if eoffs[j] % 16 != 0)
        hp = HostPipeline(NativePlan(schema))
        dec = hp.decode_var(expect, eoffs[k:], n - k, frame)
        ref = oracle.decode(schema, expect[int(eoffs[k]):], eoffs[k:] - eoffs[k], n - k, frame)
        assert columns_equal(schema, ref, dec) == []
        hp.close()


@pytest.mark.parametrize("frame", [0, 1])
@pytest.mark.parametrize("name", ["holder", "lists", "maps_nested", "bean_a", "deep", "chain"])
def test_host_varlen_nested_collections(name, frame):
    """The tree engine's shapes (list<list<...>>, List<Bean with strings>, Map<K, Bean>,
    BeanA, list^9) through the host path: bytes and offsets == the oracle, decode
    sizes every nesting level (one decode_sizes pass per level) and round-trips; the
    stream-only decode indexes the frames on the device."""
    from helpers import nested_columns
    n = 60 if name == "chain" else 900
    schema, cols = nested_columns(name, n, 31 + frame)
    expect, eoffs = oracle.encode(schema, cols, n, frame)
    hp = HostPipeline(NativePlan(schema), chunk_rows=256 if name != "chain" else 64)
    rows, offs = hp.encode_var(cols, n, frame)
    assert np.array_equal(rows, expect) and np.array_equal(offs, eoffs)
    assert columns_equal(schema, cols, hp.decode_var(expect, eoffs, n, frame)) == []
    if frame == 1:
        dec, consumed = hp.decode_stream(np.concatenate([expect, np.zeros(40, np.uint8)]), n)
        assert consumed == expect.nbytes
        assert columns_equal(schema, cols, dec) == []
    hp.close()


@pytest.mark.parametrize("name", ["mixed40_nulls", "nested_nulls", "maps", "list_struct", "holder", "maps_nested"])
def test_host_varlen_pipeline_registered(name):
    """Registered (pinned) host columns and output: the chunk pipeline's copies are
    asynchronous (H2D of chunk k+1 || encode of chunk k || D2H of chunk k-1), ordered
    by events only; bytes and offsets == the oracle over many chunks, twice on one
    context (slots reused)."""
    from helpers import nested_columns
    n = 6000
    if name in ("holder", "maps_nested"):
        schema, cols = nested_columns(name, n, 77)
    else:
        schema, make = catalog()[name]
        cols = make(n, 77)
    expect, eoffs = oracle.encode(schema, cols, n, 1)
    hp = HostPipeline(NativePlan(schema), chunk_rows=512)

    def paged(a):  # a copy on whole pages of its own (registrations must not share a page)
        raw = np.zeros(((a.nbytes + 4095) // 4096 + 1) * 4096, np.uint8)
        k = (-raw.ctypes.data) % 4096
        b = raw[k:k + (a.nbytes + 4095) // 4096 * 4096]
        b[:a.nbytes] = a.view(np.uint8).reshape(-1)
        return b, b[:a.nbytes].view(a.dtype)

    regs = []
    for c in cols:
        for attr in ("values", "offsets", "validity"):
            a = getattr(c, attr)
            if a is not None and a.nbytes > 0:
                whole, view = paged(a)
                regs.append(whole)
                setattr(c, attr, view)
    whole_out, out = paged(np.zeros(expect.nbytes + 64, np.uint8))
    arrays = regs + [whole_out]
    for a in arrays:
        host_register(a)
    try:
        for _ in range(2):
            out[:] = 0
            rows, offs = hp.encode_var(cols, n, 1, out)
            assert np.array_equal(offs, eoffs)
            bad = np.nonzero(out[:expect.nbytes] != expect)[0]
            assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"
        dec = hp.decode_var_into(out[:expect.nbytes], eoffs, n, 1)  # (sized by a first call)
        counts = [c.length for c in dec]
        nb = [c.values.nbytes if c.values is not None and c.offsets is not None else 0 for c in dec]
        outs = hp.alloc_columns(np.array(counts), np.array(nb))
        for c in outs:
            for attr in ("values", "offsets", "validity"):
                a = getattr(c, attr)
                if a is not None and a.nbytes > 0:
                    whole, view = paged(a)
                    arrays.append(whole)
                    host_register(whole)
                    setattr(c, attr, view)
        for _ in range(2):
            for c in outs:
                for a in (c.values, c.offsets, c.validity):
                    if a is not None:
                        a.view(np.uint8)[:] = 0x5A
            assert columns_equal(schema, cols, hp.decode_var_into(out[:expect.nbytes], eoffs, n, 1, outs)) == []
    finally:
        for a in arrays:
            host_unregister(a)
        hp.close()


def same_arrays(x, y):
    """Byte identity of two decodes (offsets, validity bits of the batch, values)."""
    errs = []
    for i, (a, b) in enumerate(zip(x, y)):
        k = a.length
        if k != b.length:
            errs.append(f"{i}: length {k} != {b.length}")
            continue
        if a.offsets is not None and not np.array_equal(a.offsets[:k + 1], b.offsets[:k + 1]):
            errs.append(f"{i}: offsets differ at {np.nonzero(a.offsets[:k + 1] != b.offsets[:k + 1])[0][:5]}")
        if a.validity is not None:
            ua = np.unpackbits(a.validity, bitorder="little")[:k]
            ub = np.unpackbits(b.validity, bitorder="little")[:k]
            if not np.array_equal(ua, ub):
                errs.append(f"{i}: validity differs at {np.nonzero(ua != ub)[0][:5]}")
        if a.values is not None:
            m = int(a.offsets[k]) if a.offsets is not None else k  # string bytes / elements
            va, vb = a.values[:m].view(np.uint8), b.values[:m].view(np.uint8)
            if not np.array_equal(va, vb):
                errs.append(f"{i}: values differ")
    return errs


@pytest.mark.parametrize("chunk", [1024, 1 << 20])
@pytest.mark.parametrize("frame", [0, 1, 3])
@pytest.mark.parametrize("name", VARLEN_HOST)
def test_host_varlen_decode_into(name, frame, chunk):
    """fory_rowfmt_host_decode_var_into: one pipelined call into caller-sized columns.
    Empty columns first (FORY_ERR_CAPACITY with the batch's sizes), then sized ones;
    then oversized buffers reused across calls. Chunked: each chunk's offsets moved to
    its place in the batch, list-item validity bits shifted across byte boundaries."""
    n = 5000
    schema, make = catalog()[name]
    cols = make(n, n + 5)
    expect, eoffs = oracle.encode(schema, cols, n, frame)
    hp = HostPipeline(NativePlan(schema), chunk_rows=chunk)
    dec = hp.decode_var_into(expect, eoffs, n, frame)
    assert columns_equal(schema, cols, dec) == []
    assert same_arrays(dec, hp.decode_var(expect, eoffs, n, frame)) == []  # == the whole-batch decode
    counts = np.array([c.length for c in dec], np.int64)
    nbytes = np.array([c.values.nbytes if c.values is not None and c.offsets is not None else 0 for c in dec], np.int64)
    big = hp.alloc_columns(counts + counts // 3 + 5, nbytes + 100)
    for c in big:  # garbage in the reused buffers: every byte of the batch's range is rewritten
        for a in (c.values, c.offsets, c.validity):
            if a is not None:
                a.view(np.uint8)[:] = 0xA5
    for _ in range(2):
        dec2 = hp.decode_var_into(expect, eoffs, n, frame, big)
        assert columns_equal(schema, cols, dec2) == []
    hp.close()


@pytest.mark.parametrize("name", ["holder", "lists", "maps_nested", "bean_a", "deep"])
def test_host_varlen_decode_into_nested(name):
    """The tree engine's shapes through the one-call decode, 256-row chunks: every
    nesting level sized per chunk, offsets of every level rebased."""
    from helpers import nested_columns
    n = 1100
    schema, cols = nested_columns(name, n, 41)
    expect, eoffs = oracle.encode(schema, cols, n, 1)
    hp = HostPipeline(NativePlan(schema), chunk_rows=256)
    dec = hp.decode_var_into(expect, eoffs, n, 1)
    assert columns_equal(schema, cols, dec) == []
    assert same_arrays(dec, hp.decode_var(expect, eoffs, n, 1)) == []
    hp.close()


def test_host_varlen_decode_into_errors_and_empty():
    schema, make = catalog()["mixed40_nulls"]
    n = 3000
    cols = make(n, 2)
    expect, eoffs = oracle.encode(schema, cols, n, 1)
    hp = HostPipeline(NativePlan(schema), chunk_rows=1024)
    bad = expect.copy()
    bad[int(eoffs[2500]) + 5] ^= 1  # a frame's schema hash, in the third chunk
    with pytest.raises(ClassNotCompatibleException):
        hp.decode_var_into(bad, eoffs, n, 1)
    empty = hp.decode_var_into(expect, eoffs[:1], 0, 1)
    assert all(c.length == 0 for c in empty)
    assert columns_equal(schema, cols, hp.decode_var_into(expect, eoffs, n, 1)) == []  # usable after an error
    hp.close()
