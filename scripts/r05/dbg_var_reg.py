"""Varlen host path with registered buffers: after each call (encode_var, decode_var_sizes +
decode_var, decode_var_into), are the encoded frames still the first call's? Reports the
first differing byte and its row. Usage: python scripts/r05/dbg_var_reg.py [rows] [config]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from fury_amd import _lib  # noqa: E402
from fury_amd import workloads as W  # noqa: E402
from fury_amd.format.columns import HostColumn, NP_DTYPE, validity_bytes  # noqa: E402
from fury_amd.format.native import HostPipeline, NativePlan, _check, host_register, host_unregister  # noqa: E402
from fury_amd.format.types import ArrowType, preorder  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8 * 1024 * 1024
config = sys.argv[2] if len(sys.argv) > 2 else "mixed40"
lib = _lib.load()
schema = W.mixed_schema() if config == "mixed40" else W.nested_schema()
host = W.mixed_host_columns(n, seed=23) if config == "mixed40" else W.nested_host_columns(n, seed=29)
plan = NativePlan(schema)
hp = HostPipeline(plan)
rows, offs = hp.encode_var(host, n, 1)
rows2, offs2 = hp.encode_var(host, n, 1)
print("pageable repeat equal:", np.array_equal(rows, rows2), np.array_equal(offs, offs2), flush=True)
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
out = np.zeros(rows.nbytes, np.uint8)
ro = np.zeros(n + 1, np.int64)
register_in = os.environ.get("REG_IN", "1") == "1"
register_back = os.environ.get("REG_BACK", "1") == "1"
regs = []
for c in host:
    for a in (c.values, c.offsets, c.validity):
        if a is not None and a.nbytes and register_in:
            regs.append(a)
for c in back:
    for a in (c.values, c.offsets, c.validity):
        if a is not None and a.nbytes and register_back:
            regs.append(a)
if os.environ.get("REG_OUT", "1") == "1":
    regs += [out, ro]
for a in regs:
    host_register(a)
hin, hback = hp._host_array(host), hp._host_array(back)
total = ctypes.c_int64(0)
hc, hb = np.zeros(len(fields), np.int64), np.zeros(len(fields), np.int64)
for c, k in zip(back, counts):
    c.length = int(k)


def report(tag):
    d = np.nonzero(out != rows)[0]
    if len(d) == 0:
        print(tag, "equal", flush=True)
        return
    r = np.searchsorted(offs, d[:8], side="right") - 1
    print(tag, "DIFF", len(d), "bytes; first", d[:8].tolist(), "rows", r.tolist(),
          "row offsets equal", np.array_equal(ro, offs), "offs of first row", int(offs[r[0]]), int(offs[r[0] + 1]),
          "got", out[d[0]:d[0] + 16].tolist(), "want", rows[d[0]:d[0] + 16].tolist(), flush=True)
    bad_rows = np.unique(np.searchsorted(offs, d, side="right") - 1)
    print(tag, "bad rows", len(bad_rows), "first/last", bad_rows[:4].tolist(), bad_rows[-4:].tolist(),
          "chunk of first", int(bad_rows[0]) // (1 << 20), flush=True)


for it in range(3):
    out[:] = 0
    _check(lib.fory_rowfmt_host_encode_var(hp.handle, hin, n, 1, out.ctypes.data, out.nbytes, ro.ctypes.data,
                                           ctypes.byref(total)))
    report(f"it{it} encode")
    _check(lib.fory_rowfmt_host_decode_var_sizes(hp.handle, out.ctypes.data, ro.ctypes.data, n, 1,
                                                 counts.ctypes.data, nbytes.ctypes.data))
    _check(lib.fory_rowfmt_host_decode_var(hp.handle, hback))
    report(f"it{it} decode_var")
    _check(lib.fory_rowfmt_host_decode_var_into(hp.handle, out.ctypes.data, ro.ctypes.data, n, 1, hback,
                                                hc.ctypes.data, hb.ctypes.data))
    report(f"it{it} decode_into")
for a in regs:
    host_unregister(a)
hp.close()
