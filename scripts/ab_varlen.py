"""A/B of the varlen/nested engines in ONE process: FORY_ROWFMT_VARTILE=0 (per-record
global interpreter) vs the LDS tile engine at several LDS budgets (FORY_ROWFMT_VARCAP).
Checks every variant's rows byte-for-byte against the first variant's and the decoded
columns against the inputs. Usage: python scripts/ab_varlen.py [config] [rows] [rounds] [variants JSON]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from fury_amd.format import native  # noqa: E402
from fury_amd.format.encoder import RowEncoder  # noqa: E402

config = sys.argv[1] if len(sys.argv) > 1 else "mixed40"
n = int(sys.argv[2]) if len(sys.argv) > 2 else bench.DEFAULT_ROWS[config]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
iters = 4
dev = torch.device("cuda", 0)
schema, cols, col_bytes = bench.make_batch(config, n, 0, dev)
enc = RowEncoder(schema, device=dev)
plan = enc.plan
ws = enc.workspace(n)
arr = native.column_array(cols)
status = torch.zeros(1, dtype=torch.int32, device=dev)
variants = {"global": {"FORY_ROWFMT_VARTILE": "0"}, "tile": {"FORY_ROWFMT_VARFLAT": "0"}, "flat": {},
            "cap12k": {"FORY_ROWFMT_VARCAP": "12288"}, "cap24k": {"FORY_ROWFMT_VARCAP": "24576"},
            "flat_cap48k": {"FORY_ROWFMT_VARCAP": "49152"}}
if len(sys.argv) > 4:  # variants as JSON: {"name": {"ENV": "value", ...}, ...}
    variants = json.loads(sys.argv[4])
res = {}


def set_env(envs):
    for k in ("FORY_ROWFMT_VARTILE", "FORY_ROWFMT_VARCAP", "FORY_ROWFMT_VARFLAT",
              "FORY_ROWFMT_VARSTG", "FORY_ROWFMT_SPILLCAP"):
        os.environ.pop(k, None)
    os.environ.update(envs)


def col_bytes_equal(a, b):
    for x, y in ((a.values, b.values), (a.offsets, b.offsets)):
        if (x is None) != (y is None):
            return False
        if x is not None:
            m = min(x.numel() * x.element_size(), y.numel() * y.element_size())
            if not torch.equal(x.reshape(-1).view(torch.uint8)[:m], y.reshape(-1).view(torch.uint8)[:m]):
                return False
    return True


for frame in (0, 1):
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    native.encoded_size(plan, arr, n, frame, offs, ws)
    total = int(offs[n].item())
    out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    ref_rows = None
    for rnd in range(rounds):
        for name, envs in variants.items():
            set_env(envs)
            out.zero_()
            native.encode(plan, arr, n, frame, offs, out, status, ws)
            dcols = enc.decode(out[:total], n, frame, offs)
            darr = native.column_array(dcols)
            native.read_status(status)
            rows_ok = True
            if ref_rows is None:
                ref_rows = out.clone()
            else:
                rows_ok = bool(torch.equal(out, ref_rows))
            dec_ok = all(col_bytes_equal(a, b) for a, b in zip(dcols, cols)) if config.startswith("mixed40") else None
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            te, td = [], []
            for _ in range(iters):
                ev[0].record()
                native.encoded_size(plan, arr, n, frame, offs, ws)
                native.encode(plan, arr, n, frame, offs, out, status, ws)
                ev[1].record()
                native.decode_sizes(plan, out, offs, n, frame, darr, status, ws)
                native.decode(plan, out, offs, n, frame, darr, status, ws)
                ev[2].record()
                torch.cuda.synchronize()
                te.append(ev[0].elapsed_time(ev[1]))
                td.append(ev[1].elapsed_time(ev[2]))
            native.read_status(status)
            key = f"{config}_frame{frame}_{name}"
            r = res.setdefault(key, {"enc_ms": [], "dec_ms": [], "rows_ok": True, "dec_ok": dec_ok})
            r["enc_ms"].append(round(min(te), 3))
            r["dec_ms"].append(round(min(td), 3))
            r["rows_ok"] = r["rows_ok"] and rows_ok
            algo = col_bytes + total
            r["enc_GBs_algo"] = round(algo / (min(r["enc_ms"]) * 1e-3) / 1e9, 1)
            r["dec_GBs_algo"] = round(algo / (min(r["dec_ms"]) * 1e-3) / 1e9, 1)
            r["GiBs_metric"] = round(2 * total / ((min(r["enc_ms"]) + min(r["dec_ms"])) * 1e-3) / 2**30, 1)
            del dcols, darr
set_env({})
print(json.dumps(res, indent=1))
