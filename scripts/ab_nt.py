"""A/B of cache-policy variants (FORY_ROWFMT_NT bits: 1 nt column loads, 2 nt row stores
for encode v5; 4 nt LDS-DMA row loads, 8 nt column stores for decode) on Struct104, in ONE
process with interleaved rounds. Usage: python scripts/ab_nt.py [rows] [rounds] [modes]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fury_amd import workloads as W  # noqa: E402
from fury_amd.format import native  # noqa: E402
from fury_amd.format.encoder import RowEncoder  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64 * 1024 * 1024
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
modes = [int(m) for m in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 1, 2, 3, 4, 8, 12, 15]
iters = 5
vals = W.gen_struct_device(n)
cols = [native.DeviceColumn(v, None, None, n) for v in vals]
enc = RowEncoder(W.struct_schema())
plan = enc.plan
ws = enc.workspace(n)
arr = native.column_array(cols)
status = torch.zeros(1, dtype=torch.int32, device="cuda")
res = {}
frame = 0
out = torch.empty(n * plan.stride(frame), dtype=torch.uint8, device="cuda")
dcols = enc.alloc_fixed_outputs(n)
darr = native.column_array(dcols)
os.environ.pop("FORY_ROWFMT_PIPE", None)
ref = None
for rnd in range(rounds):
    for m in modes:
        os.environ["FORY_ROWFMT_NT"] = str(m)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        native.encode(plan, arr, n, frame, None, out, status, ws)
        native.decode(plan, out, None, n, frame, darr, status, ws)
        te, td = [], []
        for _ in range(iters):
            ev[0].record()
            native.encode(plan, arr, n, frame, None, out, status, ws)
            ev[1].record()
            native.decode(plan, out, None, n, frame, darr, status, ws)
            ev[2].record()
            torch.cuda.synchronize()
            te.append(ev[0].elapsed_time(ev[1]))
            td.append(ev[1].elapsed_time(ev[2]))
        ok = all(torch.equal(a.values.view(torch.uint8), b.values.view(torch.uint8)) for a, b in zip(dcols, cols))
        h = int(out[:: 4093].to(torch.int64).sum().item())
        if ref is None:
            ref = h
        ok = ok and h == ref
        native.read_status(status)
        r = res.setdefault(f"nt{m}", {"enc_ms": [], "dec_ms": [], "ok": True})
        r["enc_ms"].append(round(sorted(te)[len(te) // 2], 3))
        r["dec_ms"].append(round(sorted(td)[len(td) // 2], 3))
        r["ok"] &= ok
algo = n * (624 + plan.stride(frame))
for r in res.values():
    r["enc_TBs"] = round(algo / (min(r["enc_ms"]) * 1e-3) / 1e12, 3)
    r["dec_TBs"] = round(algo / (min(r["dec_ms"]) * 1e-3) / 1e12, 3)
print(json.dumps(res, indent=1))
