"""Record sharding across GPUs (one process per GPU, no collective on the data path).

Rows are independent (the row format has no cross-record state), so a batch of
N records is split into contiguous ranges, one per rank; every rank encodes /
decodes its own range from / into its own HBM. For a single global output
stream (e.g. one RPC buffer), the only exchange is G <= 8 shard byte totals:
rank r's rows start at the exclusive prefix of the totals of ranks < r. That
is one small all_gather of an int64 per rank, done once per batch, off the
kernel path (fixed-width schemas need none: offsets are row * stride).
"""
from __future__ import annotations

from typing import List, Tuple


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [begin, end) record range of `rank` (sizes differ by at most 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n_total, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def shard_byte_offsets(shard_totals: List[int]) -> List[int]:
    """Exclusive prefix of per-rank encoded byte totals = each shard's start in the global stream."""
    out, acc = [], 0
    for t in shard_totals:
        out.append(acc)
        acc += int(t)
    return out


def gather_shard_offset(local_total: int, group=None) -> Tuple[int, int]:
    """(start of this rank's bytes in the global stream, global total) via one all_gather."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([int(local_total)], dtype=torch.int64, device=dev)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    totals = [int(p.item()) for p in parts]
    starts = shard_byte_offsets(totals)
    return starts[dist.get_rank(group)], sum(totals)
