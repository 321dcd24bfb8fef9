"""Probe: do the varlen sizing passes hide behind the tile kernels when they run on a
second stream, chunk by chunk? Times, for the Mixed / Nested bench batches:
  whole       encoded_size, encode, decode_sizes, decode over the whole batch (bench.py)
  chunked     the same per chunk of rows, one stream (chunking overhead alone)
  overlapped  sizes of chunk c+1 on a second stream while chunk c encodes / decodes
Chunks are independent batches here (chunk-local row / Arrow offsets): a timing probe,
not a product path. Usage: python scripts/overlap_probe.py [mixed40|nested] [chunks] [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from bench import make_batch  # noqa: E402
from fury_amd.format import native  # noqa: E402
from fury_amd.format.encoder import RowEncoder  # noqa: E402
from fury_amd.format.native import DeviceColumn  # noqa: E402
from fury_amd.format.types import ArrowType, preorder  # noqa: E402

config = sys.argv[1] if len(sys.argv) > 1 else "mixed40"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
n = {"mixed40": 16 << 20, "nested": 8 << 20}[config]
dev = torch.device("cuda", 0)
schema, cols, _ = make_batch(config, n, 0, dev)
enc = RowEncoder(schema, device=dev)
plan = enc.plan
nodes = list(preorder(schema))
# rows-indexed columns: top-level fields and struct children of row-indexed structs
rowcol = []
for f in schema.fields:
    def walk(g, rowidx):
        rowcol.append(rowidx)
        inner = g.type.id in (ArrowType.LIST, ArrowType.MAP)
        for c in g.children:
            walk(c, rowidx and not inner)
    walk(f, True)


def chunk(cs, r0, r1):
    out = []
    for c, ri in zip(cs, rowcol):
        if not ri:
            out.append(c)
            continue
        d = DeviceColumn(length=r1 - r0)
        if c.values is not None:
            d.values = c.values if c.offsets is not None else c.values[r0:r1]
        if c.offsets is not None:
            d.offsets = c.offsets[r0:r1 + 1]
        if c.validity is not None:
            d.validity = c.validity[r0 // 8:]
        out.append(d)
    return out


bounds = [n * k // K // 64 * 64 for k in range(K)] + [n]
chunks = [chunk(cols, bounds[k], bounds[k + 1]) for k in range(K)]
s0 = torch.cuda.current_stream(dev)
s1 = torch.cuda.Stream(dev)
status = torch.zeros(1, dtype=torch.int32, device=dev)


def setup(cs, m):
    arr = native.column_array(cs)
    ws = torch.empty(max(256, plan.workspace_bytes(m)), dtype=torch.uint8, device=dev)
    offs = torch.empty(m + 1, dtype=torch.int64, device=dev)
    native.encoded_size(plan, arr, m, 0, offs, ws, s0.cuda_stream)
    total = int(offs[m].item())
    out = torch.empty(max(16, total), dtype=torch.uint8, device=dev)
    native.encode(plan, arr, m, 0, offs, out, status, ws, s0.cuda_stream)
    dcols = enc.decode(out[:total], m, 0, offs)
    return {"arr": arr, "ws": ws, "ws2": torch.empty_like(ws), "offs": offs, "out": out, "m": m,
            "darr": native.column_array(dcols), "dcols": dcols}


whole = setup(cols, n)
parts = [setup(c, bounds[k + 1] - bounds[k]) for k, c in enumerate(chunks)]
torch.cuda.synchronize()


def run_whole():
    w = whole
    st = s0.cuda_stream
    native.encoded_size(plan, w["arr"], n, 0, w["offs"], w["ws"], st)
    native.encode(plan, w["arr"], n, 0, w["offs"], w["out"], status, w["ws"], st)
    native.decode_sizes(plan, w["out"], w["offs"], n, 0, w["darr"], status, w["ws"], st)
    native.decode(plan, w["out"], w["offs"], n, 0, w["darr"], status, w["ws"], st)


def run_chunked(overlap):
    s1.wait_stream(s0)
    st0, st1 = s0.cuda_stream, (s1.cuda_stream if overlap else s0.cuda_stream)
    ev_s = [torch.cuda.Event() for _ in parts]
    ev_e = [torch.cuda.Event() for _ in parts]
    start = torch.cuda.Event()
    start.record(s0)
    s1.wait_event(start)
    # encode: sizes of every chunk on st1 (in order), encode of chunk c on st0 after its sizes
    for k, p in enumerate(parts):
        native.encoded_size(plan, p["arr"], p["m"], 0, p["offs"], p["ws2"], st1)
        ev_s[k].record(s1 if overlap else s0)
    for k, p in enumerate(parts):
        s0.wait_event(ev_s[k])
        native.encode(plan, p["arr"], p["m"], 0, p["offs"], p["out"], status, p["ws"], st0)
        ev_e[k].record(s0)
    # decode (a separate call: after the whole encode): totals of chunk c on st1, values on st0 after them
    ev_d = [torch.cuda.Event() for _ in parts]
    if overlap:
        s1.wait_event(ev_e[-1])
    for k, p in enumerate(parts):
        native.decode_sizes(plan, p["out"], p["offs"], p["m"], 0, p["darr"], status, p["ws2"], st1)
        ev_d[k].record(s1 if overlap else s0)
    for k, p in enumerate(parts):
        s0.wait_event(ev_d[k])
        native.decode(plan, p["out"], p["offs"], p["m"], 0, p["darr"], status, p["ws2"], st0)  # tile totals of decode_sizes
    end = torch.cuda.Event()
    end.record(s1)
    s0.wait_event(end)


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return round(min(ts), 3), round(sum(ts) / len(ts), 3)


res = {"config": config, "rows": n, "chunks": K,
       "whole_ms": timeit(run_whole),
       "chunked_ms": timeit(lambda: run_chunked(False)),
       "overlapped_ms": timeit(lambda: run_chunked(True))}
print(json.dumps(res), flush=True)
