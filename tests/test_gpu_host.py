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


@pytest.mark.parametrize("frame", [0, 1])
def test_host_fresh_context_while_the_null_stream_is_busy(frame):
    """A context created and used at once while the device's null stream is still busy
    (here a spin kernel launched on it). Until round 6 the context zeroed its
    arena with a null-stream hipMemset, which its non-blocking streams do not wait for:
    the first call's H2D copies could land first and be zeroed, so chunk 0 encoded zero
    columns (the first-chunk failures of rounds 5 and 6, profiles/r06/intermittent/README.md
    §6). Now the arena is zeroed on the context's own stream and waited for. (A guard, not a
    reproduction: the old build passed this test too, profiles/r06/memset_race/q1-q4; the
    race itself is shown by scripts/microbench/memset_race.hip.)"""
    schema, make = catalog()["struct104"]
    n = 5000
    cols = make(n, 11)
    expect, _ = oracle.encode(schema, cols, n, frame)
    plan = NativePlan(schema)
    assert torch.cuda.current_stream().cuda_stream == 0  # torch's default stream is the null stream
    for _ in range(3):
        # ~1 s of spinning on the null stream: it must outlast the context's creation and the
        # first call's pinned staging allocations (a 20 ms spin did not, q1 in
        # profiles/r06/memset_race/). Not through torch.cuda.ExternalStream(0): a spin launched
        # under it leaves hipStreamQuery(null stream) ready (close6/null_stream_probe.json)
        torch.cuda._sleep(2_000_000_000)
        hp = HostPipeline(plan, chunk_rows=1024)
        out = np.zeros(expect.nbytes, np.uint8)
        hp.encode(cols, n, frame, out)
        bad = np.nonzero(out != expect)[0]
        assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}, rows {np.unique(bad // (expect.nbytes // n))[:4]}"
        hp.close()
    torch.cuda.synchronize()


def test_host_pipeline_registered_buffers_and_errors():
    schema, make = catalog()["struct104"]
    n = 3000
    cols = make(n, 3)
    plan = NativePlan(schema)
    hp = HostPipeline(plan, chunk_rows=512)
    out_pages, _ = page_buffer(n * plan.stride(1))  # a registration on pages of its own
    out = out_pages[:n * plan.stride(1)]
    host_register(out_pages)
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
        host_unregister(out_pages)
        hp.close()


def unregister_all(arrays):
    """Unregisters every array, each on its own: one failure must not leave the rest
    registered when numpy frees and re-issues their pages (round-2 cleanup stopped at
    the first failure). The library checks that each range no longer reads as
    registered (fory_rowfmt_host_unregister: FORY_ERR_DEVICE otherwise); here every
    array's first and last byte are pageable again."""
    errors = []
    for a in arrays:
        try:
            host_unregister(a)
        except Exception as e:  # noqa: BLE001 - reported after the loop
            errors.append(e)
    if errors:
        raise errors[0]
    for a in arrays:
        assert copy_path(a) == 0 and copy_path(a[-1:]) == 0


@pytest.fixture(autouse=True)
def _no_registration_left():
    """Every test leaves no registration behind (a registration that outlives its numpy
    buffer is how a later pageable copy could be DMA'd through a stale mapping)."""
    yield
    assert registered_ranges() == 0


def registered_ranges():
    import ctypes
    return _internal("fory_rowfmt_internal_host_registered_ranges", ctypes.c_int, [])()


def page_buffer(nbytes, pages_before=0):
    """A uint8 view on whole pages of its own (a registration never shares a page with
    other data), plus the owning array."""
    npages = (nbytes + 4095) // 4096
    raw = np.zeros((npages + pages_before + 2) * 4096, np.uint8)
    k = (-raw.ctypes.data) % 4096 + pages_before * 4096
    return raw[k:k + npages * 4096], raw


def _internal(name, restype, argtypes):
    import ctypes
    from fury_amd import _lib
    f = getattr(_lib.load(), name)
    f.restype, f.argtypes = restype, argtypes
    return f


def copy_path(a, nbytes=None):
    import ctypes
    f = _internal("fory_rowfmt_internal_host_copy_path", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64])
    return f(a.ctypes.data, a.nbytes if nbytes is None else nbytes)


def first_byte_pinned(a):
    import ctypes
    f = _internal("fory_rowfmt_internal_host_first_byte_pinned", ctypes.c_int, [ctypes.c_void_p])
    return f(a.ctypes.data)


def staged_pieces(hp):
    import ctypes
    f = _internal("fory_rowfmt_internal_host_staged_pieces", ctypes.c_int64, [ctypes.c_void_p])
    return f(hp.handle)


def test_host_copy_classification_is_by_whole_range():
    """The round-2 host-path fault mechanism, deterministically: a copy was judged
    pinned by its FIRST byte, so a range that begins inside a registration and runs
    past it (or a range whose pages were registered before and have been unregistered
    and re-used) could be handed to an async DMA as pinned. Now a copy is a direct DMA
    only when the whole range is one pinned mapping; everything else is staged."""
    buf, raw = page_buffer(64 << 10)
    assert copy_path(buf) == 0  # pageable
    head = buf[:32 << 10]  # register the first half only
    host_register(head)
    try:
        assert copy_path(head) == 1
        assert copy_path(head[4096:]) == 1  # inside the registration
        assert copy_path(buf) == 0  # starts inside, runs past the end: staged, never a direct DMA
        # round 2's rule judged the same range by its first byte: "pinned" -> an async DMA
        # over host pages the device has no mapping for (the fault mechanism)
        assert first_byte_pinned(buf) == 1
        assert copy_path(buf[(32 << 10) - 8:]) == 0  # the last 8 registered bytes + pageable ones
        assert copy_path(buf[32 << 10:]) == 0  # wholly past it
    finally:
        host_unregister(head)
    assert copy_path(head) == 0  # unregistered pages are pageable again
    # registered -> unregistered -> freed -> the same pages re-used by a fresh batch
    host_register(buf)
    host_unregister(buf)
    addr = buf.ctypes.data
    del buf, head, raw
    again, raw2 = page_buffer(64 << 10)
    assert copy_path(again) == 0, (hex(addr), hex(again.ctypes.data))


@pytest.mark.parametrize("name", ["struct104", "mixed40_nulls", "maps"])
def test_host_copies_straddling_a_registration(name):
    """Columns and output whose first pages are registered and whose rest is not (and
    pages registered, unregistered and re-used): every copy straddling a registration
    is staged (the context counts its staged pieces), the bytes equal the oracle's,
    and fully registered buffers are never staged."""
    n = 4000
    schema, make = catalog()[name]
    cols = make(n, 91)
    expect, eoffs = oracle.encode(schema, cols, n, 1)
    hp = HostPipeline(NativePlan(schema), chunk_rows=1024)
    regs, keep = [], []
    for c in cols:  # every host array on pages of its own, its first half registered
        for attr in ("values", "offsets", "validity"):
            a = getattr(c, attr)
            if a is None or a.nbytes < 8192:
                continue
            pb, raw = page_buffer(a.nbytes)
            pb[:a.nbytes] = a.view(np.uint8).reshape(-1)
            keep.append(raw)
            setattr(c, attr, pb[:a.nbytes].view(a.dtype))
            head = pb[:(a.nbytes // 2) // 4096 * 4096]
            if head.nbytes:
                host_register(head)
                regs.append(head)
    out, raw_out = page_buffer(expect.nbytes + 64)
    out_head = out[:(expect.nbytes // 2) // 4096 * 4096]
    host_register(out_head)
    regs.append(out_head)
    try:
        before = staged_pieces(hp)
        if NativePlan(schema).fixed_width:
            hp.encode(cols, n, 1, out[:expect.nbytes])
            got = out[:expect.nbytes]
        else:
            got, offs = hp.encode_var(cols, n, 1, out)
            assert np.array_equal(offs, eoffs)
        assert staged_pieces(hp) > before  # the straddling copies went through the staging
        bad = np.nonzero(got != expect)[0]
        assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"
    finally:
        unregister_all(regs)
    # the same pages, now pageable again: decode through them
    rows_pb, raw_rows = page_buffer(expect.nbytes)
    rows_pb[:expect.nbytes] = expect
    host_register(rows_pb)
    host_unregister(rows_pb)
    rows = rows_pb[:expect.nbytes]
    if NativePlan(schema).fixed_width:
        dec = empty_like(schema, n)
        hp.decode(rows, n, 1, dec)
    else:
        dec = hp.decode_var_into(rows, eoffs, n, 1)
        assert same_arrays(dec, hp.decode_var(rows, eoffs, n, 1)) == []
    assert columns_equal(schema, cols, dec) == []
    hp.close()


def test_host_registered_buffers_are_never_staged():
    """Whole-range registered columns and output: every copy is a direct async DMA."""
    schema, make = catalog()["struct104"]
    n = 3000
    cols = make(n, 5)
    expect, _ = oracle.encode(schema, cols, n, 1)
    regs = []
    for c in cols:
        pb, raw = page_buffer(c.values.nbytes)
        pb[:c.values.nbytes] = c.values.view(np.uint8)
        c.values = pb[:c.values.nbytes].view(c.values.dtype)
        regs.append(pb)
    out, raw_out = page_buffer(expect.nbytes)
    regs.append(out)
    for a in regs:
        host_register(a)
    hp = HostPipeline(NativePlan(schema), chunk_rows=1024)
    try:
        hp.encode(cols, n, 1, out[:expect.nbytes])
        assert np.array_equal(out[:expect.nbytes], expect)
        assert staged_pieces(hp) == 0
    finally:
        unregister_all(regs)
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


@pytest.mark.parametrize("name,n,chunk", [("mixed40_nulls", 40009, 1 << 20), ("struct104", 20011, 8192),
                                          ("nested_nulls", 60013, 16384)])
def test_host_pageable_pieces_over_a_mib(name, n, chunk, monkeypatch):
    """Pageable caller memory with staged pieces of 1..4 MiB whose sizes the host copy
    threads do not divide evenly: every byte crosses (round 5 lost the last n mod parts
    bytes of such pieces -- tests/test_host_copy_pool.py). The context runs with
    FORY_ROWFMT_HOST_VERIFY: every chunk's host-to-device pieces are read back and
    compared with the caller's bytes, so a wrong piece fails the call naming the piece
    and the source its device bytes match (round 5's one wrong output here was column-
    shaped: chunk 0's f0 slice whole and part of f1, profiles/r05/intermittent/)."""
    schema, make = catalog()[name]
    cols = make(n, 11)
    expect, eoffs = oracle.encode(schema, cols, n, 1)
    monkeypatch.setenv("FORY_ROWFMT_HOST_VERIFY", "1")
    hp = HostPipeline(NativePlan(schema), chunk_rows=chunk)
    if name == "struct104":
        out = np.zeros(expect.nbytes, np.uint8)
        hp.encode(cols, n, 1, out)
        dec = empty_like(schema, n)
        hp.decode(expect, n, 1, dec)
    else:
        out, offs = hp.encode_var(cols, n, 1, np.zeros(expect.nbytes, np.uint8))
        assert np.array_equal(offs, eoffs)
        dec = hp.decode_var(expect, eoffs, n, 1)
    bad = np.nonzero(out != expect)[0]
    if len(bad):  # (a diagnosis for the report: which frames, and what they hold instead)
        offs_e = eoffs if eoffs is not None else np.arange(n + 1, dtype=np.int64) * (expect.nbytes // n)
        frames = np.unique(np.searchsorted(offs_e, bad, side="right") - 1)
        f0 = int(frames[0])
        got = out[offs_e[f0]:offs_e[f0 + 1]]
        same = [int(r) for r in range(n) if offs_e[r + 1] - offs_e[r] == len(got)
                and np.array_equal(expect[offs_e[r]:offs_e[r + 1]], got)][:4]
        detail = (f"frames {frames[:6].tolist()}..{frames[-3:].tolist()} ({len(frames)}), chunks "
                  f"{sorted(set((frames // chunk).tolist()))[:8]}, zero bytes among them {int((out[bad] == 0).sum())}, "
                  f"got {out[bad[:8]].tolist()} want {expect[bad[:8]].tolist()}, frame {f0} as written equals "
                  f"expected frames {same}, staged pieces {staged_pieces(hp)}")
        assert False, f"{len(bad)} bytes differ, first at {bad[:8]}: {detail}"
    assert columns_equal(schema, cols, dec) == []
    hp.close()


def call_regs(hp):
    """(registrations the context made over its life, bytes, microseconds; call-scoped
    registrations alive in the process)."""
    import ctypes
    f = _internal("fory_rowfmt_internal_host_call_regs", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p])
    out = np.zeros(3, np.int64)
    alive = f(hp.handle if hp is not None else None, out.ctypes.data)
    return int(out[0]), int(out[1]), int(out[2]), alive


@pytest.mark.parametrize("frame", [0, 1])
def test_host_pageable_columns_registered_for_the_call(frame, monkeypatch):
    """Pageable columns and output of >= 4 MiB page interiors: each
    caller buffer's interior is registered for the call on its first copy and unregistered
    before the call returns; the copies inside it are direct DMAs, the unaligned heads and
    tails staged. Bytes equal the oracle's both ways (verify mode on), nothing stays
    registered, and a buffer the caller registered itself is used as is."""
    monkeypatch.setenv("FORY_ROWFMT_HOST_VERIFY", "1")
    schema, make = catalog()["struct104_boxed"]
    n = 600_011  # int64 columns: 4.8 MB; chunks of 128Ki records: slices inside the interiors
    cols = make(n, 29)
    expect, _ = oracle.encode(schema, cols, n, frame)
    hp = HostPipeline(NativePlan(schema), chunk_rows=1 << 17)
    out = np.zeros(expect.nbytes + 100, np.uint8)[3:3 + expect.nbytes]  # unaligned head and tail
    hp.encode(cols, n, frame, out)
    calls, nbytes, _, alive = call_regs(hp)
    assert alive == 0 and registered_ranges() == 0
    assert calls >= 53 and nbytes >= 52 * (8 * n - 8192)  # 52 int64/double columns + the output
    bad = np.nonzero(out != expect)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"
    dec = empty_like(schema, n)
    hp.decode(out, n, frame, dec)
    assert columns_equal(schema, cols, dec) == []
    assert call_regs(hp)[0] > calls and call_regs(hp)[3] == 0
    # the caller's own registration of the output: taken whole, not registered again
    pb, raw = page_buffer(expect.nbytes)
    host_register(pb)
    try:
        before = call_regs(hp)[0]
        hp.encode(cols, n, frame, pb[:expect.nbytes])
        assert np.array_equal(pb[:expect.nbytes], expect)
        assert call_regs(hp)[0] - before <= 104  # the columns only
    finally:
        host_unregister(pb)
    hp.close()


@pytest.mark.parametrize("name", ["mixed40_nulls", "nested_nulls"])
def test_host_varlen_pageable_registered_for_the_call(name, monkeypatch):
    """Varlen plans: pageable columns, rows and decode outputs registered per call the
    same way (encode_var + decode_var_into), bytes equal the oracle's, none left behind."""
    monkeypatch.setenv("FORY_ROWFMT_HOST_VERIFY", "1")
    schema, make = catalog()[name]
    n = 300_007
    cols = make(n, 3)
    expect, eoffs = oracle.encode(schema, cols, n, 1)
    hp = HostPipeline(NativePlan(schema), chunk_rows=1 << 16)
    out, offs = hp.encode_var(cols, n, 1, np.zeros(expect.nbytes, np.uint8))
    assert np.array_equal(offs, eoffs) and np.array_equal(out, expect)
    assert call_regs(hp)[0] > 0 and call_regs(hp)[3] == 0
    dec = hp.decode_var_into(expect, eoffs, n, 1)
    assert columns_equal(schema, cols, dec) == []
    assert call_regs(hp)[3] == 0 and registered_ranges() == 0
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
@pytest.mark.parametrize("name", ["holder", "lists", "maps_nested", "bean_a", "deep", "chain", "decimals"])
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
        unregister_all(arrays)
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


@pytest.mark.parametrize("name", ["holder", "lists", "maps_nested", "bean_a", "deep", "decimals"])
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


def test_host_register_refuses_overlaps_and_foreign_bases():
    """fory_rowfmt_host_register refuses bytes already registered (sharing a page is fine);
    unregister takes only a registered range's start; after it, both ends of the range read
    as unregistered while a neighbour on the same page stays registered."""
    from fury_amd.format import IllegalArgumentException
    buf, raw = page_buffer(5 * 4096)
    a, b = buf[:4096 + 100], buf[4096 + 200:3 * 4096]  # b shares a's second page
    host_register(a)
    try:
        with pytest.raises(IllegalArgumentException):
            host_register(buf[4096:4096 + 150])  # overlaps a's last bytes
        host_register(b)
        assert registered_ranges() == 2
        assert copy_path(b) == 1
        with pytest.raises(IllegalArgumentException):
            host_unregister(a[8:])  # not a registered start
    finally:
        host_unregister(a)
    assert copy_path(a) == 0 and copy_path(buf[4096 + 99:4096 + 100]) == 0
    assert copy_path(b) == 1  # the neighbour on the shared page is still registered
    host_unregister(b)


def paged_copy(a):
    """A copy of array a on whole pages of its own (+ the owning buffer)."""
    pb, raw = page_buffer(max(a.nbytes, 1))
    pb[:a.nbytes] = a.view(np.uint8).reshape(-1)
    return pb, pb[:a.nbytes].view(a.dtype).reshape(a.shape)


@pytest.mark.parametrize("frame", [0, 1, 3])
@pytest.mark.parametrize("n", [1, 64, 5003])
@pytest.mark.parametrize("name", ["struct104", "struct104_boxed", "all_types"])
def test_host_fixed_registered(name, n, frame):
    """Fixed-width plans with every column (values and validity) and the output registered
    on pages of their own: every column slice and row piece is one DMA (nothing staged),
    the oracle's bytes; decode the same way back; a hash mismatch is still
    ClassNotCompatibleException."""
    schema, make = catalog()[name]
    cols = make(n, n + 19)
    expect, _ = oracle.encode(schema, cols, n, frame)
    plan = NativePlan(schema)
    hp = HostPipeline(plan, chunk_rows=1024)
    regs = []
    try:
        for c in cols:
            for attr in ("values", "validity"):
                a = getattr(c, attr)
                if a is not None:
                    whole, view = paged_copy(a)
                    host_register(whole)
                    regs.append(whole)
                    setattr(c, attr, view)
        out_whole, _ = paged_copy(np.zeros(expect.nbytes, np.uint8))
        host_register(out_whole)
        regs.append(out_whole)
        out = out_whole[:expect.nbytes]
        hp.encode(cols, n, frame, out)
        assert staged_pieces(hp) == 0
        bad = np.nonzero(out != expect)[0]
        assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"
        dec = empty_like(schema, n)
        for c in dec:
            for attr in ("values", "validity"):
                a = getattr(c, attr)
                if a is not None:
                    whole, view = paged_copy(a)
                    host_register(whole)
                    regs.append(whole)
                    setattr(c, attr, view)
        hp.decode(out, n, frame, dec)
        assert staged_pieces(hp) == 0
        assert columns_equal(schema, cols, dec) == []
        if frame in (1, 3):
            out[(4 if frame == 1 else 0) + (n // 2) * plan.stride(frame)] ^= 1  # a frame's schema hash
            with pytest.raises(ClassNotCompatibleException):
                hp.decode(out, n, frame, dec)
    finally:
        unregister_all(regs)
        hp.close()


def test_host_fixed_registered_windows_and_a_pageable_column():
    """Registered output windows that split a validity byte, then one column left pageable
    (its slices staged, the others one DMA each): the same bytes either way."""
    schema, make = catalog()["struct104_boxed"]
    n = 3001
    cols = make(n, 7)
    expect, _ = oracle.encode(schema, cols, n, 1)
    plan = NativePlan(schema)
    stride = plan.stride(1)
    hp = HostPipeline(plan, chunk_rows=1024)
    regs = []
    try:
        for c in cols:
            for attr in ("values", "validity"):
                whole, view = paged_copy(getattr(c, attr))
                host_register(whole)
                regs.append(whole)
                setattr(c, attr, view)
        w1, _ = paged_copy(np.zeros(1003 * stride, np.uint8))  # window 2 starts at row 1003
        w2, _ = paged_copy(np.zeros((n - 1003) * stride, np.uint8))
        for w in (w1, w2):
            host_register(w)
            regs.append(w)
        rows, nbytes = hp.encode_windows(cols, n, 1, [w1[:1003 * stride], w2[:(n - 1003) * stride]])
        assert list(rows) == [1003, n - 1003] and staged_pieces(hp) == 0
        assert np.array_equal(np.concatenate([w1[:nbytes[0]], w2[:nbytes[1]]]), expect)
        host_unregister(regs.pop(0))  # one column pageable again
        out_whole, _ = paged_copy(np.zeros(expect.nbytes, np.uint8))
        host_register(out_whole)
        regs.append(out_whole)
        hp.encode(cols, n, 1, out_whole[:expect.nbytes])
        assert staged_pieces(hp) > 0
        assert np.array_equal(out_whole[:expect.nbytes], expect)
    finally:
        unregister_all(regs)
        hp.close()
