"""Host-inclusive rate of the row-format path (recorded in DESIGN.md, never bench `value`).

The reference path starts and ends in host memory (JVM off-heap MemoryBuffers
on their way to / from an RPC socket). Here: Struct104 columns in pinned host
memory -> H2D -> encode -> D2H rows (pinned), then rows -> H2D -> decode -> D2H
columns, chunk-pipelined over three HIP streams (copy-in / kernel / copy-out)
with double-buffered device chunks, so PCIe traffic in both directions
overlaps the kernels. Reports the same metric as bench.py (row bytes written
+ read / time) plus the PCIe GB/s it implies.
Usage: python scripts/host_inclusive.py [rows] [chunk_rows]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fury_amd import workloads as W  # noqa: E402
from fury_amd.format import native  # noqa: E402
from fury_amd.format.encoder import RowEncoder  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8 * 1024 * 1024
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 1024 * 1024
assert n % chunk == 0
dev = torch.device("cuda", 0)
schema = W.struct_schema()
enc = RowEncoder(schema, device=dev)
plan = enc.plan
stride = plan.stride(0)

# pinned host inputs (device-generated java.util.Random values, copied once)
vals = W.gen_struct_device(n, device=dev)
host_cols = [torch.empty(v.shape, dtype=v.dtype, pin_memory=True) for v in vals]
for h, v in zip(host_cols, vals):
    h.copy_(v)
del vals
host_rows = torch.empty(n * stride, dtype=torch.uint8, pin_memory=True)
host_out = [torch.empty(h.shape, dtype=h.dtype, pin_memory=True) for h in host_cols]
torch.cuda.synchronize()

s_in, s_k, s_out = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
dcols = [[torch.empty(chunk, dtype=h.dtype, device=dev) for h in host_cols] for _ in range(2)]
drows = [torch.empty(chunk * stride, dtype=torch.uint8, device=dev) for _ in range(2)]
ws = [torch.empty(max(256, plan.workspace_bytes(chunk)), dtype=torch.uint8, device=dev) for _ in range(2)]
status = torch.zeros(1, dtype=torch.int32, device=dev)
arrs = [native.column_array([native.DeviceColumn(c, None, None, chunk) for c in dcols[b]]) for b in range(2)]
nchunks = n // chunk


def encode_pass():
    ev_in = [torch.cuda.Event() for _ in range(nchunks)]
    ev_k = [torch.cuda.Event() for _ in range(nchunks)]
    ev_out = [torch.cuda.Event() for _ in range(nchunks)]
    for k in range(nchunks):
        b = k & 1
        a, e = k * chunk, (k + 1) * chunk
        with torch.cuda.stream(s_in):
            if k >= 2:
                s_in.wait_event(ev_k[k - 2])  # device chunk buffer b free again
            for dc, hc in zip(dcols[b], host_cols):
                dc.copy_(hc[a:e], non_blocking=True)
            ev_in[k].record(s_in)
        with torch.cuda.stream(s_k):
            s_k.wait_event(ev_in[k])
            if k >= 2:
                s_k.wait_event(ev_out[k - 2])  # row buffer b drained
            native.encode(plan, arrs[b], chunk, 0, None, drows[b], status, ws[b], s_k.cuda_stream)
            ev_k[k].record(s_k)
        with torch.cuda.stream(s_out):
            s_out.wait_event(ev_k[k])
            host_rows[a * stride:e * stride].copy_(drows[b], non_blocking=True)
            ev_out[k].record(s_out)
    torch.cuda.synchronize()


def decode_pass():
    ev_in = [torch.cuda.Event() for _ in range(nchunks)]
    ev_k = [torch.cuda.Event() for _ in range(nchunks)]
    ev_out = [torch.cuda.Event() for _ in range(nchunks)]
    dec_arr = [native.column_array([native.DeviceColumn(c, None, None, chunk) for c in dcols[b]]) for b in range(2)]
    for k in range(nchunks):
        b = k & 1
        a, e = k * chunk, (k + 1) * chunk
        with torch.cuda.stream(s_in):
            if k >= 2:
                s_in.wait_event(ev_k[k - 2])
            drows[b].copy_(host_rows[a * stride:e * stride], non_blocking=True)
            ev_in[k].record(s_in)
        with torch.cuda.stream(s_k):
            s_k.wait_event(ev_in[k])
            if k >= 2:
                s_k.wait_event(ev_out[k - 2])
            native.decode(plan, drows[b], None, chunk, 0, dec_arr[b], status, ws[b], s_k.cuda_stream)
            ev_k[k].record(s_k)
        with torch.cuda.stream(s_out):
            s_out.wait_event(ev_k[k])
            for hc, dc in zip(host_out, dcols[b]):
                hc[a:e].copy_(dc, non_blocking=True)
            ev_out[k].record(s_out)
    torch.cuda.synchronize()


encode_pass()
decode_pass()
res = {}
t0 = time.perf_counter()
encode_pass()
t_enc = time.perf_counter() - t0
t0 = time.perf_counter()
decode_pass()
t_dec = time.perf_counter() - t0
native.read_status(status)
ok = all(torch.equal(a.view(torch.uint8), b.view(torch.uint8)) for a, b in zip(host_out, host_cols))
row_bytes = n * stride
col_bytes = sum(h.numel() * h.element_size() for h in host_cols)
res = {
    "metric": "row-format encode+decode GiB/s, host-inclusive (pinned H2D + kernel + D2H, chunk-pipelined)",
    "rows": n, "chunk_rows": chunk, "round_trip_ok": ok,
    "encode_s": round(t_enc, 4), "decode_s": round(t_dec, 4),
    "value_GiBs": round(2 * row_bytes / (t_enc + t_dec) / 2**30, 2),
    "encode_pcie_GBs": {"h2d": round(col_bytes / t_enc / 1e9, 1), "d2h": round(row_bytes / t_enc / 1e9, 1)},
    "decode_pcie_GBs": {"h2d": round(row_bytes / t_dec / 1e9, 1), "d2h": round(col_bytes / t_dec / 1e9, 1)},
}
print(json.dumps(res))
