"""CPU: encode / decode v5's per-plan record rotation (fixed.hip: v5_rotation over a model
of the MI355X LDS access groups, v5_store_cycles). At Struct104's raw stride (848 B = 212
dwords) the in-order writes of a 4-byte field put a 16-lane ds_write_b64 group on 4 of 32
banks; the chosen rotation must model fewer cycles than in order, never more, and be a
valid shift (0..4, or 31 = in order). Byte identity of every rotation is the GPU suite's
(tests/test_gpu_parity.py, fixed-width schemas x frames)."""
import ctypes

import pytest


def fns():
    from fury_amd import _lib
    lib = _lib.load()
    rot = getattr(lib, "fory_rowfmt_internal_v5_rotation")
    rot.restype, rot.argtypes = ctypes.c_int, [ctypes.c_int] * 5
    cyc = getattr(lib, "fory_rowfmt_internal_v5_cycles")
    cyc.restype, cyc.argtypes = ctypes.c_int, [ctypes.c_int] * 6
    return rot, cyc


@pytest.mark.parametrize("read", [0, 1])
@pytest.mark.parametrize("w", [4, 8])
@pytest.mark.parametrize("fixed,bitmap,hdr", [(848, 16, 0), (848, 16, 12), (848, 16, 8), (72, 8, 0), (264, 8, 12),
                                              (8 + 8 * 300, 40, 0), (16, 8, 0)])
def test_rotation_never_models_worse(fixed, bitmap, hdr, w, read):
    rot, cyc = fns()
    stride = fixed + hdr
    r = rot(stride, hdr, hdr + bitmap, w, read)
    assert r == 31 or 0 <= r <= 4
    assert cyc(stride, hdr, hdr + bitmap, w, r, read) <= cyc(stride, hdr, hdr + bitmap, w, 31, read)


def test_struct104_raw_rotates_its_4_byte_fields():
    rot, cyc = fns()
    r = rot(848, 0, 16, 4, 0)
    assert r != 31
    assert cyc(848, 0, 16, 4, r, 0) * 2 <= cyc(848, 0, 16, 4, 31, 0)  # (modelled: 128 -> 32 group-cycles)
