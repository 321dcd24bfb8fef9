"""Encode-call and decode-call times (HIP events, 10 reps) of a varlen config, no checks:
for the FORY_ROWFMT_DBGSKIP timing splits. Usage: python kernel_times.py mixed40|nested"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
from fury_amd.format import native  # noqa: E402
from fury_amd.format.encoder import RowEncoder  # noqa: E402

cfg = sys.argv[1]
n = bench.DEFAULT_TOTAL[cfg]
dev = torch.device("cuda", 0)
schema, cols, col_bytes = bench.make_batch(cfg, n, 0, dev)
enc = RowEncoder(schema, device=dev)
plan = enc.plan
ws = enc.workspace(n)
arr = native.column_array(cols)
status = torch.zeros(1, dtype=torch.int32, device=dev)
offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
native.encoded_size(plan, arr, n, 0, offs, ws)
total = int(offs[n].item())
out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
native.encode(plan, arr, n, 0, offs, out, status, ws)
os.environ.pop("FORY_ROWFMT_DBGSKIP", None)
dcols = RowEncoder(schema, device=dev).decode(out[:total], n, 0, offs)  # shapes (a plan without the knob)
darr = native.column_array(dcols)
native.decode_sizes(plan, out, offs, n, 0, darr, status, ws)
res = {}
for name, fn in (("encode", lambda: native.encode(plan, arr, n, 0, offs, out, status, ws)),
                 ("decode", lambda: native.decode(plan, out, offs, n, 0, darr, status, ws))):
    for _ in range(3):
        fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(10):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    res[name + "_ms"] = round(ev[0].elapsed_time(ev[1]) / 10, 4)
res["algo_bytes"] = col_bytes + total
print(json.dumps(res))
