"""Struct104 encode/decode time vs buffer placement, in ONE process: the row buffer at
several byte shifts from its allocation, and fresh column allocations. Separates
placement effects from kernel changes when process-to-process times differ.
Usage: python scripts/ab_placement.py [rows] [rounds]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fury_amd import workloads as W  # noqa: E402
from fury_amd.format import native  # noqa: E402
from fury_amd.format.encoder import RowEncoder  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64 * 1024 * 1024
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
enc = RowEncoder(W.struct_schema())
plan = enc.plan
ws = enc.workspace(n)
status = torch.zeros(1, dtype=torch.int32, device="cuda")
shifts = [0, 256, 4096, 1 << 16, 1 << 21, 3 << 20]
base = torch.empty(n * 848 + max(shifts), dtype=torch.uint8, device="cuda")
dcols = enc.alloc_fixed_outputs(n)
darr = native.column_array(dcols)
res = {}


def timed(fn, reps=5):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    ts = []
    for _ in range(reps):
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    return round(sorted(ts)[reps // 2], 3)


for gen in range(rounds):  # fresh column allocations each round
    vals = W.gen_struct_device(n)
    cols = [native.DeviceColumn(v, None, None, n) for v in vals]
    arr = native.column_array(cols)
    for sh in shifts:
        out = base[sh:sh + n * 848]
        te = timed(lambda: native.encode(plan, arr, n, 0, None, out, status, ws))
        td = timed(lambda: native.decode(plan, out, None, n, 0, darr, status, ws))
        r = res.setdefault(f"shift={sh}", {"enc_ms": [], "dec_ms": []})
        r["enc_ms"].append(te)
        r["dec_ms"].append(td)
    native.read_status(status)
    del vals, cols, arr
    torch.cuda.empty_cache()
print(json.dumps(res))
