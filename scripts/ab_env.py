"""In-process A/B of one environment knob on Struct104 encode/decode (interleaved rounds,
median of 5 per round). Usage: python scripts/ab_env.py VAR v1,v2,... [rows] [rounds] [frame]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fury_amd import workloads as W  # noqa: E402
from fury_amd.format import native  # noqa: E402
from fury_amd.format.encoder import RowEncoder  # noqa: E402

var = sys.argv[1]
values = sys.argv[2].split(",")
n = int(sys.argv[3]) if len(sys.argv) > 3 else 64 * 1024 * 1024
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
frame = int(sys.argv[5]) if len(sys.argv) > 5 else 0
vals = W.gen_struct_device(n)
cols = [native.DeviceColumn(v, None, None, n) for v in vals]
enc = RowEncoder(W.struct_schema())
plan = enc.plan
ws = enc.workspace(n)
arr = native.column_array(cols)
status = torch.zeros(1, dtype=torch.int32, device="cuda")
out = torch.empty(n * plan.stride(frame), dtype=torch.uint8, device="cuda")
dcols = enc.alloc_fixed_outputs(n)
darr = native.column_array(dcols)
res = {}
ref = None
for rnd in range(rounds):
    for v in values:
        os.environ[var] = v
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        native.encode(plan, arr, n, frame, None, out, status, ws)
        native.decode(plan, out, None, n, frame, darr, status, ws)
        te, td = [], []
        for _ in range(5):
            ev[0].record()
            native.encode(plan, arr, n, frame, None, out, status, ws)
            ev[1].record()
            native.decode(plan, out, None, n, frame, darr, status, ws)
            ev[2].record()
            torch.cuda.synchronize()
            te.append(ev[0].elapsed_time(ev[1]))
            td.append(ev[1].elapsed_time(ev[2]))
        ok = all(torch.equal(a.values.view(torch.uint8), b.values.view(torch.uint8)) for a, b in zip(dcols, cols))
        native.read_status(status)
        r = res.setdefault(f"{var}={v}", {"enc_ms": [], "dec_ms": [], "ok": True})
        r["enc_ms"].append(round(sorted(te)[2], 3))
        r["dec_ms"].append(round(sorted(td)[2], 3))
        r["ok"] &= ok
algo = n * (624 + plan.stride(frame))
for r in res.values():
    r["enc_TBs"] = round(algo / (min(r["enc_ms"]) * 1e-3) / 1e12, 3)
    r["dec_TBs"] = round(algo / (min(r["dec_ms"]) * 1e-3) / 1e12, 3)
print(json.dumps(res))
