"""CPU: the C-ABI library loads, exports every symbol include/fory_rowfmt.h
declares, and its host-side planner (no GPU needed) matches the reference:
schema hash (python/pyfory/format/infer.py golden values), fixed size
(BinaryRowWriter.java:46-52), bitmap width (BitUtils.java:175-177), and the
reference's error behaviour for bad schemas."""
import ctypes
import os
import re

import pytest

from fury_amd import _lib
from fury_amd import workloads as W
from fury_amd.format import errors
from fury_amd.format.native import NativePlan
from fury_amd.format.types import ArrowType, DataType, DataTypes, Field, Schema, flatten

from helpers import all_types_schema, string_list_schema, wide_schema

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                      "fory_rowfmt.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fory_rowfmt_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 11
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_lib.PROTOTYPES), "ctypes prototypes out of sync with the header"
    assert lib.fory_rowfmt_abi_version() == 1


def test_plan_matches_reference(golden):
    cases = {"struct104": W.struct_schema(), "mixed40": W.mixed_schema(), "nested": W.nested_schema(),
             "struct_boxed": W.struct_schema(boxed=True)}
    for name, s in cases.items():
        p = NativePlan(s)
        assert p.schema_hash == golden["schema_hash"][name], name
    p = NativePlan(W.struct_schema())
    assert (p.num_fields, p.bitmap_bytes, p.fixed_size, p.fixed_width, p.row_size) == (104, 16, 848, True, 848)
    p = NativePlan(W.mixed_schema())
    assert (p.num_fields, p.bitmap_bytes, p.fixed_size, p.fixed_width, p.row_size) == (40, 8, 328, False, -1)
    p = NativePlan(W.nested_schema())
    assert (p.num_fields, p.num_columns, p.fixed_size, p.fixed_width) == (3, 7, 32, False)


def test_edge_plans(golden):
    s = Schema([Field(f"c{i:03d}", DataType(ArrowType.INT64), False) for i in range(300)])
    p = NativePlan(s)
    assert p.schema_hash == golden["schema_hash"]["wide_300"]  # exercises the overflow (>> 2) path
    assert p.bitmap_bytes == 40 and p.fixed_size == 40 + 2400
    assert NativePlan(Schema([])).schema_hash == golden["schema_hash"]["empty"]
    assert NativePlan(Schema([])).fixed_size == 0
    for s in (all_types_schema(), wide_schema(), string_list_schema()):
        NativePlan(s)


def test_plan_errors():
    lib = _lib.load()
    bad_nested = Schema([Field("x", DataType(ArrowType.INT32), False, [Field("y", DataType(ArrowType.INT32))])])
    with pytest.raises(errors.EncoderException):
        NativePlan(bad_nested)
    with pytest.raises(errors.EncoderException):  # a map needs [key, value] children
        NativePlan(Schema([Field("m", DataType(ArrowType.MAP), True)]))
    # every nesting has a device path (op programs, or the tree engine for
    # Map<K, Bean>, list<list<...>>, List<Bean with var fields>)
    NativePlan(Schema([DataTypes.map_field("m", Field("key", DataType(ArrowType.STRING), False),
                                           Field("value", DataType(ArrowType.INT32), True))]))
    NativePlan(Schema([DataTypes.map_field("m", Field("key", DataType(ArrowType.STRING), False),
                                           DataTypes.struct_field("value", True, [
                                               Field("a", DataType(ArrowType.INT32))]))]))
    with pytest.raises(errors.EncoderException):  # Map's keys must be non-nullable (DataTypes.java:419)
        NativePlan(Schema([Field("m", DataType(ArrowType.MAP), True, [Field("key", DataType(ArrowType.INT32), True),
                                                                       Field("value", DataType(ArrowType.INT32))])]))
    with pytest.raises(errors.EncoderException):  # ... also behind a nesting the tree engine takes
        NativePlan(Schema([DataTypes.array_field("l", DataTypes.array_field("item", Field("item", DataType(ArrowType.INT32)))),
                           Field("m", DataType(ArrowType.MAP), True, [Field("key", DataType(ArrowType.INT32), True),
                                                                       Field("value", DataType(ArrowType.INT32))])]))
    NativePlan(Schema([DataTypes.array_field("l", Field("item", DataType(ArrowType.STRING)))]))
    NativePlan(Schema([DataTypes.array_field("l", DataTypes.array_field(
        "item", Field("item", DataType(ArrowType.INT32))))]))
    NativePlan(Schema([DataTypes.array_field("l", DataTypes.struct_field(
        "item", True, [Field("s", DataType(ArrowType.STRING))]))]))
    # truncated descriptor: a struct promising 2 children with only 1 present
    desc, n = flatten(Schema([DataTypes.struct_field("s", True, [Field("a", DataType(ArrowType.INT32))])]))
    desc[0].num_children = 2
    h = ctypes.c_void_p()
    assert lib.fory_rowfmt_plan_create(desc, n, ctypes.byref(h)) == _lib.FORY_ERR_ENCODER
    assert "truncated" in _lib.last_error()
    desc[0].num_children = 1
    desc[0].reserved = 5
    assert lib.fory_rowfmt_plan_create(desc, n, ctypes.byref(h)) == _lib.FORY_ERR_INVALID_ARGUMENT


def test_argument_validation_without_gpu():
    """Calls that fail validation return before touching the device."""
    lib = _lib.load()
    p = NativePlan(W.struct_schema())
    cols = (_lib.Column * 104)()
    # workspace too small
    rc = lib.fory_rowfmt_encode(p.handle, cols, 10, 0, None, ctypes.c_void_p(16), 1 << 20, None,
                                None, 0, None)
    assert rc == _lib.FORY_ERR_INVALID_ARGUMENT and "workspace" in _lib.last_error()
    # bad frame mode
    rc = lib.fory_rowfmt_encode(p.handle, cols, 10, 7, None, None, 0, None, None, 0, None)
    assert rc == _lib.FORY_ERR_INVALID_ARGUMENT
    # zero rows: nothing to do
    rc = lib.fory_rowfmt_encode(p.handle, cols, 0, 1, None, None, 0, None, None, 0, None)
    assert rc == _lib.FORY_OK
    assert lib.fory_rowfmt_workspace_bytes(p.handle, 1 << 26) > 104 * 40


def test_host_path_validation_without_gpu():
    """The host path rejects bad arguments before touching the device."""
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.fory_rowfmt_host_ctx_create(None, 0, 1024, ctypes.byref(h)) == _lib.FORY_ERR_INVALID_ARGUMENT
    cols = (_lib.Column * 1)()
    assert lib.fory_rowfmt_host_encode(None, cols, 1, 0, None, 0) == _lib.FORY_ERR_INVALID_ARGUMENT
    assert lib.fory_rowfmt_host_decode(None, None, 0, 1, 0, cols) == _lib.FORY_ERR_INVALID_ARGUMENT
    assert lib.fory_rowfmt_host_register(None, 16) == _lib.FORY_ERR_INVALID_ARGUMENT
    total = ctypes.c_int64(0)
    assert lib.fory_rowfmt_host_encode_var(None, cols, 1, 0, None, 0, None, ctypes.byref(total)) == \
        _lib.FORY_ERR_INVALID_ARGUMENT
    assert lib.fory_rowfmt_host_decode_var_sizes(None, None, None, 1, 0, None, None) == _lib.FORY_ERR_INVALID_ARGUMENT
    assert lib.fory_rowfmt_host_decode_var(None, cols) == _lib.FORY_ERR_INVALID_ARGUMENT
    used = ctypes.c_int64(0)
    assert lib.fory_rowfmt_host_decode_stream_sizes(None, None, 0, 1, None, None, ctypes.byref(used)) == \
        _lib.FORY_ERR_INVALID_ARGUMENT


def test_frame_index_validation_without_gpu():
    """fory_rowfmt_index_frames: RAW rows are not self-delimiting, collection frames carry
    no schema hash; a fixed-width stream too short for N frames is corrupt — all
    decided before any device work."""
    lib = _lib.load()
    p = NativePlan(W.struct_schema())
    assert lib.fory_rowfmt_index_frames(p.handle, None, 0, 1, 0, None, None, None, 0, None) == \
        _lib.FORY_ERR_INVALID_ARGUMENT
    assert lib.fory_rowfmt_index_frames(p.handle, None, 0, 1, 2, None, None, None, 0, None) == \
        _lib.FORY_ERR_UNSUPPORTED
    assert lib.fory_rowfmt_index_frames(p.handle, None, 860 * 3 - 1, 3, 1, ctypes.c_void_p(64), None, None, 0,
                                        None) == _lib.FORY_ERR_CORRUPT
    m = NativePlan(W.mixed_schema())
    assert lib.fory_rowfmt_index_frames(m.handle, ctypes.c_void_p(18), 10000, 3, 1, ctypes.c_void_p(64), None,
                                        None, 0, None) == _lib.FORY_ERR_INVALID_ARGUMENT  # misaligned rows
    need = lib.fory_rowfmt_index_workspace_bytes(m.handle, 1 << 24, 8 << 30)
    assert 0 < need < (1 << 24) * 8  # a few bytes per record


def test_split_windows_greedy():
    """fory_rowfmt_split_windows (host-only): whole rows per <= max-byte window, greedy,
    the way a JNI caller fills int-sized MemoryBuffers (MemoryBuffer.java:87)."""
    import numpy as np
    from fury_amd.format.native import split_windows
    from fury_amd.format.errors import IndexOutOfBoundsException
    rng = np.random.default_rng(1)
    sizes = rng.integers(20, 900, size=5000)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    for cap in (900, 1000, 4096, 100000, int(offs[-1]), 1 << 40):
        first = split_windows(offs, 5000, cap)
        assert first[0] == 0 and first[-1] == 5000
        for a, b in zip(first[:-1], first[1:]):
            assert b > a and offs[b] - offs[a] <= cap
            if b < 5000:  # greedy: the next row would not fit
                assert offs[b + 1] - offs[a] > cap
    # fixed stride
    first = split_windows(None, 10, 2000, stride=860)
    assert list(first) == [0, 2, 4, 6, 8, 10]
    with pytest.raises(IndexOutOfBoundsException):  # a row larger than a window
        split_windows(offs, 5000, 500)
    assert list(split_windows(offs, 0, 100)) == [0]
