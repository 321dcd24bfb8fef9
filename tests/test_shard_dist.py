"""CPU, world_size 2 (gloo): record sharding reproduces the single-process
encode byte for byte — each rank encodes its contiguous shard (oracle on CPU,
standing in for the per-GPU kernel), one all_gather of the shard byte totals
places the shards, and the concatenation equals the whole-batch frame stream
(= N x Encoder.encode(MemoryBuffer, T), Encoders.java:213-225)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from fury_amd.shard import shard_byte_offsets, shard_range  # noqa: E402


def test_shard_range_partitions():
    for n in (0, 1, 7, 64, 1000, 12345):
        for world in (1, 2, 3, 8):
            ranges = [shard_range(n, world, r) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            for (a, b), (c, _) in zip(ranges, ranges[1:]):
                assert b == c
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1
    assert shard_byte_offsets([5, 0, 7]) == [0, 5, 5]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, n, frame, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from helpers import catalog
    from oracle import oracle
    from fury_amd.shard import gather_shard_offset
    schema, make = catalog()[name]
    cols = make(n, 3)  # every rank builds the same batch; it encodes only its shard
    b, e = shard_range(n, world, rank)
    sub = _slice_columns(schema, cols, b, e)
    buf, _ = oracle.encode(schema, sub, e - b, frame)
    start, total = gather_shard_offset(len(buf))
    np.save(os.path.join(out_dir, f"shard{rank}.npy"), buf)
    np.save(os.path.join(out_dir, f"meta{rank}.npy"), np.array([start, total], dtype=np.int64))
    dist.barrier()
    dist.destroy_process_group()


def _slice_columns(schema, cols, b, e):
    """Rows [b, e) of pre-order host columns (top-level + struct children + list items)."""
    from fury_amd.format.columns import HostColumn, pack_validity, unpack_validity
    from fury_amd.format.types import ArrowType
    out = []
    pos = [0]

    def visit(f, lo, hi):
        c = cols[pos[0]]
        pos[0] += 1
        n = hi - lo
        v = None
        if f.nullable and c.validity is not None:
            v = pack_validity(unpack_validity(c.validity, c.length)[lo:hi])
        t = f.type.id
        if t in (ArrowType.STRING, ArrowType.BINARY):
            o = c.offsets[lo:hi + 1].astype(np.int64)
            out.append(HostColumn(c.values[o[0]:o[-1]].copy() if o[-1] > o[0] else np.zeros(8, np.uint8),
                                  (o - o[0]).astype(np.int32), v, n))
        elif t == ArrowType.LIST:
            o = c.offsets[lo:hi + 1].astype(np.int64)
            out.append(HostColumn(None, (o - o[0]).astype(np.int32), v, n))
            visit(f.children[0], int(o[0]), int(o[-1]))
        elif t == ArrowType.STRUCT:
            out.append(HostColumn(None, None, v, n))
            for ch in f.children:
                visit(ch, lo, hi)
        else:
            out.append(HostColumn(c.values[lo:hi].copy(), None, v, n))

    for f in schema.fields:
        visit(f, b, e)
    return out


@pytest.mark.parametrize("name,frame", [("struct104", 1), ("mixed40_nulls", 1), ("nested_nulls", 0)])
def test_two_rank_shards_concatenate_to_the_whole_batch(tmp_path, name, frame):
    from helpers import catalog
    from oracle import oracle
    n = 301
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), name, n, frame, str(tmp_path)), nprocs=world, join=True)
    schema, make = catalog()[name]
    whole, _ = oracle.encode(schema, make(n, 3), n, frame)
    parts = [np.load(tmp_path / f"shard{r}.npy") for r in range(world)]
    metas = [np.load(tmp_path / f"meta{r}.npy") for r in range(world)]
    assert all(int(m[1]) == len(whole) for m in metas)
    for r in range(world):
        s = int(metas[r][0])
        assert np.array_equal(whole[s:s + len(parts[r])], parts[r])
    assert np.array_equal(np.concatenate(parts), whole)
