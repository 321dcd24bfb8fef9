"""CPU: the staged copies' host memcpy (host.cpp CopyPool) moves every byte of a piece.

Round 5's first split rounded each part down when the piece size divided evenly into
64-byte multiples per part but not into the parts themselves, so the last (n mod parts)
bytes of a >= 1 MiB staged piece were never copied: pageable varlen encodes at 8Mi rows
lost a byte or four at the end of two chunks. The pool runs on host threads only (no GPU
call), so every split is checked here."""
import ctypes

import numpy as np
import pytest


def pool_copy():
    from fury_amd import _lib
    f = getattr(_lib.load(), "fory_rowfmt_internal_pool_copy")
    f.restype, f.argtypes = None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    return f


@pytest.mark.parametrize("n", [0, 1, 63, 1 << 20, (1 << 20) + 5, 8 * 64 * 2048 + 5, (1 << 20) * 3 + 7,
                               (4 << 20) - 3, 4 << 20, 8 * 64 * 8192 + 7, 4194303])
@pytest.mark.parametrize("dst_off,src_off", [(0, 0), (3, 0), (0, 5), (7, 9)])
def test_pool_copy_moves_every_byte(n, dst_off, src_off):
    """(non-temporal 16-byte stores from any source alignment into any destination alignment)"""
    f = pool_copy()
    rng = np.random.default_rng(n)
    src = rng.integers(0, 256, n + 64, dtype=np.uint8)
    dst = np.zeros(n + 64, np.uint8)
    f(dst.ctypes.data + dst_off, src.ctypes.data + src_off, n)
    assert np.array_equal(dst[dst_off:dst_off + n], src[src_off:src_off + n])
    assert not dst[:dst_off].any() and not dst[dst_off + n:].any()  # nothing outside the piece
