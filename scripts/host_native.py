"""Host-inclusive rate through the C-ABI host path (fory_rowfmt_host_encode/decode:
C++ three-stream chunk pipeline, H2D || kernel || D2H). Struct104 columns in
registered (pinned) host memory -> rows in host memory -> columns back. Recorded in
DESIGN.md, never bench `value`. Usage: python scripts/host_native.py [rows] [chunk_rows]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fury_amd import workloads as W  # noqa: E402
from fury_amd.format.columns import HostColumn  # noqa: E402
from fury_amd.format.native import HostPipeline, NativePlan, host_register, host_unregister  # noqa: E402

# HOST_MEM=pageable: plain (unregistered) numpy buffers: the library registers each
# buffer's page interior for the call (round 6) and stages the unaligned ends through the
# context's pinned blocks; default: the caller registers the buffers
PAGEABLE = os.environ.get("HOST_MEM", "registered") == "pageable"
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8 * 1024 * 1024
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
res = {"host_memory": "pageable (call-scoped registration + staged ends)" if PAGEABLE else "registered", "metric": "row-format encode+decode GiB/s, host-inclusive (C-ABI host path: pinned H2D + kernel + D2H)",
       "rows": n, "chunk_rows": chunk}
plan = NativePlan(W.struct_schema())
vals = W.gen_struct_device(n)
host = [HostColumn(v.cpu().numpy(), None, None, n) for v in vals]
del vals
torch.cuda.synchronize()
back = [HostColumn(np.empty_like(c.values), None, None, n) for c in host]
for frame in (0, 1):
    stride = plan.stride(frame)
    rows = np.empty(n * stride, np.uint8)
    bufs = [c.values for c in host] + [c.values for c in back] + [rows]
    for b in bufs:
        if not PAGEABLE:
            host_register(b)
    hp = HostPipeline(plan, chunk_rows=chunk)
    hp.encode(host, n, frame, rows)  # warm-up
    hp.decode(rows, n, frame, back)
    te, td = [], []
    for _ in range(3):
        t0 = time.perf_counter()
        hp.encode(host, n, frame, rows)
        te.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        hp.decode(rows, n, frame, back)
        td.append(time.perf_counter() - t0)
    ok = all(np.array_equal(a.values.view(np.uint8), b.values.view(np.uint8)) for a, b in zip(host, back))
    import ctypes
    from fury_amd import _lib
    f = _lib.load().fory_rowfmt_internal_host_call_regs
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]
    st = np.zeros(3, np.int64)
    f(hp.handle, st.ctypes.data)  # call-scoped registrations over the 8 calls (pageable buffers)
    regs = {"count": int(st[0]), "GiB": round(int(st[1]) / 2**30, 2), "ms": round(int(st[2]) / 1000, 1), "calls": 8}
    hp.close()
    for b in bufs:
        if not PAGEABLE:
            host_unregister(b)
    t_enc, t_dec = min(te), min(td)
    col_bytes = sum(c.values.nbytes for c in host)
    row_bytes = n * stride
    res["raw" if frame == 0 else "frame"] = {
        "round_trip_ok": ok, "encode_s": round(t_enc, 4), "decode_s": round(t_dec, 4),
        "value_GiBs": round(2 * row_bytes / (t_enc + t_dec) / 2**30, 2), "call_scoped_registrations": regs,
        "encode_pcie_GBs": {"h2d": round(col_bytes / t_enc / 1e9, 1), "d2h": round(row_bytes / t_enc / 1e9, 1)},
        "decode_pcie_GBs": {"h2d": round(row_bytes / t_dec / 1e9, 1), "d2h": round(col_bytes / t_dec / 1e9, 1)},
    }
print(json.dumps(res))
