"""Host-inclusive rate of the varlen configs through the C-ABI host path
(fory_rowfmt_host_encode_var: chunk pipeline; host_decode_var_sizes + host_decode_var:
whole batch, H2D + kernels + D2H in series; host_decode_var_into: chunk pipeline). Host columns and rows in registered (pinned)
memory. Recorded in DESIGN.md, never bench `value`.
Usage: python scripts/host_native_var.py [rows]"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from fury_amd import _lib  # noqa: E402
from fury_amd import workloads as W  # noqa: E402
from fury_amd.format.columns import HostColumn, NP_DTYPE, validity_bytes  # noqa: E402
from fury_amd.format.native import HostPipeline, NativePlan, _check, host_register, host_unregister  # noqa: E402
from fury_amd.format.types import ArrowType, preorder  # noqa: E402

# HOST_MEM=pageable: plain (unregistered) numpy buffers, so every copy goes through the
# context's pinned staging blocks; default: the buffers are registered
PAGEABLE = os.environ.get("HOST_MEM", "registered") == "pageable"
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4 * 1024 * 1024
lib = _lib.load()
res = {"host_memory": "pageable (staged)" if PAGEABLE else "registered", "metric": "row-format encode+decode GiB/s, host-inclusive (C-ABI varlen host path, whole batch)", "rows": n}
for config in ("mixed40", "nested"):
    schema = W.mixed_schema() if config == "mixed40" else W.nested_schema()
    host = W.mixed_host_columns(n, seed=23) if config == "mixed40" else W.nested_host_columns(n, seed=29)
    plan = NativePlan(schema)
    hp = HostPipeline(plan)
    rows, offs = hp.encode_var(host, n, 1)  # sizes the output once
    fields = preorder(schema)
    counts = np.zeros(len(fields), np.int64)
    nbytes = np.zeros(len(fields), np.int64)
    _check(lib.fory_rowfmt_host_decode_var_sizes(hp.handle, rows.ctypes.data, offs.ctypes.data, n, 1,
                                                 counts.ctypes.data, nbytes.ctypes.data))
    back = []
    for i, f in enumerate(fields):
        k, t = int(counts[i]), f.type.id
        c = HostColumn(length=k)
        if t in (ArrowType.STRING, ArrowType.BINARY):
            c.values = np.empty(max(1, int(nbytes[i])), np.uint8)
        elif t in NP_DTYPE:
            c.values = np.empty(max(1, k), NP_DTYPE[t])
        if t in (ArrowType.STRING, ArrowType.BINARY, ArrowType.LIST, ArrowType.MAP):
            c.offsets = np.empty(k + 1, np.int32)
        if f.nullable:
            c.validity = np.empty(validity_bytes(k), np.uint8)
        back.append(c)
    arrays = [a for c in host + back for a in (c.values, c.offsets, c.validity) if a is not None and a.nbytes]
    out = np.empty(rows.nbytes, np.uint8)
    ro = np.empty(n + 1, np.int64)
    arrays += [out, ro]
    for a in arrays:
        if not PAGEABLE:
            host_register(a)
    hin, hback = hp._host_array(host), hp._host_array(back)
    total = ctypes.c_int64(0)
    te, td, ti = [], [], []
    hc, hb = np.zeros(len(fields), np.int64), np.zeros(len(fields), np.int64)
    for c, k in zip(back, counts):
        c.length = int(k)
    for _ in range(4):
        t0 = time.perf_counter()
        _check(lib.fory_rowfmt_host_encode_var(hp.handle, hin, n, 1, out.ctypes.data, out.nbytes, ro.ctypes.data,
                                               ctypes.byref(total)))
        te.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        _check(lib.fory_rowfmt_host_decode_var_sizes(hp.handle, out.ctypes.data, ro.ctypes.data, n, 1,
                                                     counts.ctypes.data, nbytes.ctypes.data))
        _check(lib.fory_rowfmt_host_decode_var(hp.handle, hback))
        td.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        _check(lib.fory_rowfmt_host_decode_var_into(hp.handle, out.ctypes.data, ro.ctypes.data, n, 1, hback,
                                                    hc.ctypes.data, hb.ctypes.data))
        ti.append(time.perf_counter() - t0)
    ok = bool(np.array_equal(out, rows))
    for a in arrays:
        if not PAGEABLE:
            host_unregister(a)
    hp.close()
    t_enc, t_dec, t_into = min(te[1:]), min(td[1:]), min(ti[1:])
    col_bytes = sum(a.nbytes for c in host for a in (c.values, c.offsets, c.validity) if a is not None)
    res[config] = {"frames_equal_first_call": ok, "encode_s": round(t_enc, 4), "decode_s": round(t_dec, 4),
                   "value_GiBs": round(2 * rows.nbytes / (t_enc + t_dec) / 2**30, 2),
                   "row_bytes": int(rows.nbytes), "column_bytes": int(col_bytes),
                   "pcie_GBs_encode": round((col_bytes + rows.nbytes) / t_enc / 1e9, 1),
                   "pcie_GBs_decode": round((col_bytes + rows.nbytes) / t_dec / 1e9, 1),
                   "decode_into_s": round(t_into, 4),
                   "value_GiBs_decode_into": round(2 * rows.nbytes / (t_enc + t_into) / 2**30, 2),
                   "pcie_GBs_decode_into": round((col_bytes + rows.nbytes) / t_into / 1e9, 1),
                   "sizes_match": bool(np.array_equal(hc, counts) and np.array_equal(hb, nbytes))}
print(json.dumps(res))
