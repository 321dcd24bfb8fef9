"""Phase timeline of the flat varlen encode kernel and of the decode values pass
(debug, FORY_ROWFMT_VARPROF=1):
per-tile durations of each phase (s_memrealtime, 100 MHz), tile lifetime and the
average number of tiles resident. Usage: python scripts/var_timeline.py [config] [rows]"""
import ctypes
import json
import os
import sys

os.environ["FORY_ROWFMT_VARPROF"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from fury_amd import _lib  # noqa: E402
from fury_amd.format import native  # noqa: E402
from fury_amd.format.encoder import RowEncoder  # noqa: E402

config = sys.argv[1] if len(sys.argv) > 1 else "mixed40"
n = int(sys.argv[2]) if len(sys.argv) > 2 else bench.DEFAULT_TOTAL[config]
dev = torch.device("cuda", 0)
schema, cols, col_bytes = bench.make_batch(config, n, 0, dev)
enc = RowEncoder(schema, device=dev)
plan = enc.plan
ws = enc.workspace(n)
arr = native.column_array(cols)
status = torch.zeros(1, dtype=torch.int32, device=dev)
res = {}
lib = _lib.load()
lib.fory_rowfmt_debug_timeline.restype = ctypes.c_int64
lib.fory_rowfmt_debug_timeline.argtypes = [ctypes.c_void_p, ctypes.c_int64]
names = ["bounds+stage0", "wave0 layout", "fixed", "barrier1", "var place", "barrier2", "flush"]
if os.environ.get("FORY_ROWFMT_VARENC", "0") != "1":  # encode v7's stamps
    names = ["RT1 (bounds, offsets, fixed)", "sizes+spans issued+fixed slots", "barrier A",
             "positions+slots (NEST: walk, barrier B)", "span wait", "copies+barrier C", "store (to completion)"]
for frame in (0, 1):
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    native.encoded_size(plan, arr, n, frame, offs, ws)
    total = int(offs[n].item())
    out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    for _ in range(3):
        native.encode(plan, arr, n, frame, offs, out, status, ws)
    torch.cuda.synchronize()
    tiles = (n + 63) // 64
    buf = np.zeros(tiles * 8, dtype=np.uint64)
    got = lib.fory_rowfmt_debug_timeline(buf.ctypes.data, buf.size)
    t = buf[:got].reshape(-1, 8).astype(np.int64)
    t = t[t[:, 7] > 0]
    d = np.diff(t, axis=1) * 10 / 1000.0  # us
    life = (t[:, 7] - t[:, 0]) * 10 / 1000.0
    span = (t[:, 7].max() - t[:, 0].min()) * 10 / 1000.0
    r = {"tiles_stamped": int(len(t)), "kernel_span_us": round(float(span), 1),
         "tile_life_us_median": round(float(np.median(life)), 2), "tile_life_us_p90": round(float(np.percentile(life, 90)), 2),
         "avg_resident_tiles": round(float(life.sum() / span), 1)}
    for k, nm in enumerate(names):
        r[nm] = {"median_us": round(float(np.median(d[:, k])), 2), "p90_us": round(float(np.percentile(d[:, k], 90)), 2),
                 "mean_us": round(float(d[:, k].mean()), 2)}
    res[f"{config}_frame{frame}"] = r

def summarize(t, names):
    t = t[t[:, 7] > 0]
    d = np.diff(t, axis=1) * 10 / 1000.0  # us
    life = (t[:, 7] - t[:, 0]) * 10 / 1000.0
    span = (t[:, 7].max() - t[:, 0].min()) * 10 / 1000.0
    r = {"tiles_stamped": int(len(t)), "kernel_span_us": round(float(span), 1),
         "tile_life_us_median": round(float(np.median(life)), 2),
         "avg_resident_tiles": round(float(life.sum() / span), 1)}
    for k, nm in enumerate(names):
        if nm:
            r[nm] = {"median_us": round(float(np.median(d[:, k])), 2), "mean_us": round(float(d[:, k].mean()), 2)}
    return r


dnames = ["stage rows", "frame/struct bases", "fixed fields", "var fields", "barrier", None, None]
for frame in (0, 1):
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    native.encoded_size(plan, arr, n, frame, offs, ws)
    total = int(offs[n].item())
    out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    native.encode(plan, arr, n, frame, offs, out, status, ws)
    for _ in range(3):
        enc.decode(out[:total], n, frame, offs)
    torch.cuda.synchronize()
    tiles = (n + 63) // 64
    buf = np.zeros(tiles * 8, dtype=np.uint64)
    got = lib.fory_rowfmt_debug_timeline(buf.ctypes.data, buf.size)
    res[f"{config}_decode_frame{frame}"] = summarize(buf[:got].reshape(-1, 8).astype(np.int64), dnames)
print(json.dumps(res, indent=1))
