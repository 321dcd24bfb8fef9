"""Throughput of the tree engine (fury_amd/csrc/generic.hip) on the nested test shapes:
device-resident encode (sizes + scan + encode) and decode (level-by-level sizes +
values), bytes = row bytes + column bytes per direction. Diagnostic, not the bench.
Usage: python scripts/bench_nested_shapes.py [rows] [shape,shape...] [--encode-only]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from helpers import nested_columns  # noqa: E402
from fury_amd.format.columns import HostColumn, pack_validity, to_device, unpack_validity  # noqa: E402
from fury_amd.format.types import ArrowType, preorder  # noqa: E402


def tile_columns(schema, cols, reps):
    """The batch repeated reps times (Arrow columns: offsets shifted per copy)."""
    out = []
    for f, c in zip(preorder(schema), cols):
        k = c.length
        t = HostColumn(length=k * reps)
        if c.offsets is not None:
            o = c.offsets.astype(np.int64)
            t.offsets = np.concatenate([o[:k] + r * o[k] for r in range(reps)] + [o[k:k + 1] * reps]).astype(np.int32)
        if c.values is not None:
            if f.type.id in (ArrowType.STRING, ArrowType.BINARY):
                t.values = np.tile(c.values[:int(c.offsets[k])], reps)
            else:
                t.values = np.tile(c.values[:k], reps)
        if c.validity is not None:
            t.validity = pack_validity(np.tile(unpack_validity(c.validity, k), reps))
        out.append(t)
    return out
from fury_amd.format.encoder import RowEncoder  # noqa: E402

n0 = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
out = {}
shapes = sys.argv[2].split(",") if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else ["holder", "lists", "maps_nested", "bean_a"]
encode_only = "--encode-only" in sys.argv
for name in shapes:
    base = 16384  # generated once (the Python row generator is slow), then tiled
    print("generating", name, n0, flush=True)
    schema, cols = nested_columns(name, base, 5)
    n = n0 // base * base
    cols = tile_columns(schema, cols, n // base)
    col_bytes = sum(a.nbytes for c in cols for a in (c.values, c.offsets, c.validity) if a is not None)
    enc = RowEncoder(schema)
    dcols = to_device(cols)
    rows = enc.encode(dcols, n, 1)
    enc.decode(rows)
    torch.cuda.synchronize()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    te, td = [], []
    for _ in range(5):
        e0.record()
        rows = enc.encode(dcols, n, 1)
        e1.record()
        if not encode_only:
            enc.decode(rows)
        e2.record()
        torch.cuda.synchronize()
        te.append(e0.elapsed_time(e1))
        td.append(e1.elapsed_time(e2))
    rb = rows.buffer.numel()
    t_e, t_d = min(te), min(td)
    out[name] = {"rows": n, "row_bytes": rb, "column_bytes": col_bytes,
                 "encode_ms": round(t_e, 3), "decode_ms": round(t_d, 3),
                 "encode_GBps": round((rb + col_bytes) / t_e / 1e6, 1), "decode_GBps": round((rb + col_bytes) / t_d / 1e6, 1)}
    print(name, out[name], flush=True)
print(json.dumps(out))
