"""GPU: <= 2 GiB MemoryBuffer windows. A MemoryBuffer is int-sized
(java/fory-core/.../memory/MemoryBuffer.java:87), so a JVM caller takes a big batch
as several buffers, each holding whole frames: the oracle's single stream, cut
greedily at frame boundaries, must equal each window byte for byte — here for a
Struct104 frame stream larger than 2 GiB (two windows of 2^31 - 1 bytes) and for
varlen plans across many small windows, through the device path
(fory_rowfmt_split_windows over the encoder's row offsets) and the host path
(fory_rowfmt_host_encode_windows)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import oracle  # noqa: E402
from fury_amd import workloads as W  # noqa: E402
from fury_amd.format import IndexOutOfBoundsException  # noqa: E402
from fury_amd.format.columns import to_device  # noqa: E402
from fury_amd.format.encoder import RowEncoder  # noqa: E402
from fury_amd.format.native import DeviceColumn, HostPipeline, NativePlan, split_windows  # noqa: E402

from helpers import catalog  # noqa: E402

pytestmark = pytest.mark.gpu

MAX_INT = (1 << 31) - 1


def oracle_windows(stream, offs, n, cap):
    """The oracle's stream cut greedily at frame boundaries into <= cap windows."""
    out, a = [], 0
    while a < n:
        b = a
        while b < n and offs[b + 1] - offs[a] <= cap:
            b += 1
        assert b > a
        out.append(stream[offs[a]:offs[b]])
        a = b
    return out


def test_struct104_stream_beyond_2gib_in_memorybuffer_windows():
    n = 2_600_000  # 2.6M frames x 860 B = 2.24 GB > 2^31 - 1
    schema = W.struct_schema()
    host = W.struct_host_columns(n, seed_base=41)
    expect, offs = oracle.encode(schema, host, n, 1)
    assert expect.nbytes > MAX_INT
    want = oracle_windows(expect, offs, n, MAX_INT)
    assert len(want) == 2
    # device path: encode once, split at frame boundaries
    enc = RowEncoder(schema)
    vals = W.gen_struct_device(n, seed_base=41)
    rows = enc.encode([DeviceColumn(v, None, None, n) for v in vals], n, 1)
    first = split_windows(None, n, MAX_INT, stride=860)
    assert len(first) == 3
    for w in range(2):
        a, b = int(first[w]), int(first[w + 1])
        got = rows.buffer[a * 860:b * 860].cpu().numpy()
        assert np.array_equal(got, want[w]), w
    del rows
    torch.cuda.empty_cache()
    # host path: straight into two int-sized host buffers
    hp = HostPipeline(NativePlan(schema), chunk_rows=1 << 19)
    wins = [np.zeros(MAX_INT, np.uint8), np.zeros(MAX_INT, np.uint8)]
    nrows, nbytes = hp.encode_windows(host, n, 1, wins)
    assert int(nrows.sum()) == n
    for w in range(2):
        assert np.array_equal(wins[w][:nbytes[w]], want[w]), w
    hp.close()


@pytest.mark.parametrize("name", ["mixed40_nulls", "nested_nulls", "maps", "struct104_boxed"])
@pytest.mark.parametrize("frame", [0, 1, 3])
def test_windows_many_small(name, frame):
    schema, make = catalog()[name]
    n = 4000
    cols = make(n, 8)
    expect, offs = oracle.encode(schema, cols, n, frame)
    cap = 70_000
    want = oracle_windows(expect, offs, n, cap)
    hp = HostPipeline(NativePlan(schema), chunk_rows=1000)
    wins = [np.zeros(cap, np.uint8) for _ in range(len(want))]
    nrows, nbytes = hp.encode_windows(cols, n, frame, wins)
    assert int(nrows.sum()) == n
    for w, exp in enumerate(want):
        assert nbytes[w] == exp.nbytes and np.array_equal(wins[w][:nbytes[w]], exp), w
    # too few windows: IndexOutOfBoundsException
    with pytest.raises(IndexOutOfBoundsException):
        hp.encode_windows(cols, n, frame, wins[:-1])
    # device path: the encoder's own offsets split the same way
    enc = RowEncoder(schema)
    rows = enc.encode(to_device(cols), n, frame)
    d_offs = offs if rows.offsets is None else rows.offsets.cpu().numpy()
    first = split_windows(d_offs, n, cap)
    assert len(first) - 1 == len(want)
    buf = rows.buffer.cpu().numpy()
    for w, exp in enumerate(want):
        assert np.array_equal(buf[d_offs[first[w]]:d_offs[first[w + 1]]], exp)
    hp.close()
