"""GPU, two fresh rank processes (both on cuda:0 of a 1-GPU box, gloo for the one
int64 exchange): record sharding through the HIP path reproduces the whole-batch
stream. Each rank encodes its contiguous shard with the device kernels (C-ABI),
gather_shard_offset places it, and the concatenation equals the oracle's
whole-batch output (= N x Encoder.encode(MemoryBuffer, T), Encoders.java:213-225,
or N x BinaryRow.toBytes). Each rank also decodes its own shard on the device
back to its input columns. This is bench.py's multi-GPU partitioning
with the per-GPU kernel in place of the oracle used by tests/test_shard_dist.py."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, name, n, frame, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, HERE)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from helpers import catalog, columns_equal
    from test_shard_dist import _slice_columns
    from fury_amd.format.columns import to_device, to_host
    from fury_amd.format.encoder import RowEncoder
    from fury_amd.shard import gather_shard_offset, shard_range
    schema, make = catalog()[name]
    cols = make(n, 3)  # every rank builds the same batch; it encodes only its shard
    b, e = shard_range(n, world, rank)
    sub = _slice_columns(schema, cols, b, e)
    enc = RowEncoder(schema, device="cuda:0")
    rows = enc.encode(to_device(sub, "cuda:0"), e - b, frame)
    buf = rows.buffer.cpu().numpy()
    start, total = gather_shard_offset(len(buf))
    dec = to_host(enc.decode(rows))
    bad = columns_equal(schema, sub, dec)
    np.save(os.path.join(out_dir, f"shard{rank}.npy"), buf)
    np.save(os.path.join(out_dir, f"meta{rank}.npy"), np.array([start, total, len(bad)], dtype=np.int64))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,frame", [("struct104", 1), ("struct104", 0), ("mixed40_nulls", 1),
                                        ("nested_nulls", 0), ("nested_nulls", 1)])
def test_two_rank_device_shards_concatenate_to_the_whole_batch(tmp_path, name, frame):
    import sys
    sys.path.insert(0, HERE)
    from helpers import catalog
    from oracle import oracle
    n = 4097 + 301  # shards of 2199 records: partial last tile on each rank
    world = 2
    port = _free_port()
    mp.start_processes(_rank, args=(world, port, name, n, frame, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    schema, make = catalog()[name]
    whole, _ = oracle.encode(schema, make(n, 3), n, frame)
    parts = [np.load(tmp_path / f"shard{r}.npy") for r in range(world)]
    metas = [np.load(tmp_path / f"meta{r}.npy") for r in range(world)]
    assert all(int(m[1]) == len(whole) for m in metas)
    assert all(int(m[2]) == 0 for m in metas), "a rank's device decode differs from its input shard"
    for r in range(world):
        s = int(metas[r][0])
        assert np.array_equal(whole[s:s + len(parts[r])], parts[r])
    assert np.array_equal(np.concatenate(parts), whole)
