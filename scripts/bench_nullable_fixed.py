"""Nullable fixed-width timing: Struct104 with boxed fields (every field nullable,
`struct_schema(boxed=True)`, 10 % nulls per field), device-resident, encode and decode
kernel calls timed with HIP events on torch's current stream (the stream the C-ABI
calls are given). Prints one JSON line; A/B of two builds via FORY_ROWFMT_LIB.
Usage: python scripts/bench_nullable_fixed.py [rows] [frame] [null_rate]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fury_amd import workloads as W  # noqa: E402
from fury_amd.format import native  # noqa: E402
from fury_amd.format.encoder import RowEncoder  # noqa: E402
from fury_amd.format.types import ArrowType  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16 * 1024 * 1024
frame = int(sys.argv[2]) if len(sys.argv) > 2 else 0
null_rate = float(sys.argv[3]) if len(sys.argv) > 3 else 0.1
dev = torch.device("cuda", 0)
schema = W.struct_schema(boxed=True)
g = torch.Generator(device=dev)
g.manual_seed(5)
DT = {ArrowType.INT32: torch.int32, ArrowType.INT64: torch.int64, ArrowType.FLOAT: torch.float32,
      ArrowType.DOUBLE: torch.float64}
cols = []
nb = ((n + 7) // 8 + 3) // 4 * 4
for f in schema.fields:
    dt = DT[f.type.id]
    v = torch.randint(-2**31, 2**31 - 1, (n * (2 if dt.itemsize == 8 else 1),), generator=g, device=dev,
                      dtype=torch.int32).view(dt)
    bits = (torch.rand(n, generator=g, device=dev) >= null_rate).to(torch.uint8)
    pad = torch.zeros(nb * 8 - n, dtype=torch.uint8, device=dev)
    b8 = torch.cat([bits, pad]).view(-1, 8)
    val = (b8 << torch.arange(8, device=dev, dtype=torch.uint8)).sum(1, dtype=torch.int32).to(torch.uint8)
    cols.append(native.DeviceColumn(v, None, val.contiguous(), n))
enc = RowEncoder(schema, device=dev)
p = enc.plan
ws = enc.workspace(n)
arr = native.column_array(cols)
status = torch.zeros(1, dtype=torch.int32, device=dev)
stride = p.stride(frame)
out = torch.empty(n * stride, dtype=torch.uint8, device=dev)
outs = enc.alloc_fixed_outputs(n)
oarr = native.column_array(outs)
row_bytes = n * stride
col_bytes = sum(c.values.numel() * c.values.element_size() + c.validity.numel() for c in cols)


def timed(fn, reps=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


e_ms = timed(lambda: native.encode(p, arr, n, frame, None, out, status, ws))
d_ms = timed(lambda: native.decode(p, out, None, n, frame, oarr, status, ws))
native.read_status(status)
# round trip: validity exact, values equal where valid
bad = 0
for a, b in zip(outs, cols):
    bad += int((a.validity[:(n + 7) // 8] != b.validity[:(n + 7) // 8]).sum().item())
    vb = torch.repeat_interleave(b.validity[:(n + 7) // 8], 8)[:n]
    bitpos = torch.arange(n, device=dev) % 8
    valid = ((vb >> bitpos.to(torch.uint8)) & 1).bool()
    it = torch.int32 if a.values.element_size() == 4 else torch.int64  # raw bits (NaN patterns)
    av, bv = a.values[:n].view(it), b.values[:n].view(it)
    bad += int((av[valid] != bv[valid]).sum().item()) + int((av[~valid] != 0).sum().item())
gb = (row_bytes + col_bytes) / 1e9
print(json.dumps({"workload": f"struct104 boxed (all 104 fields nullable, {null_rate:.0%} nulls), {n} records, frame {frame}",
                  "lib": os.environ.get("FORY_ROWFMT_LIB", "in-tree"), "encode_ms": round(e_ms, 3),
                  "decode_ms": round(d_ms, 3), "encode_frac": round(gb / e_ms * 1e3 / 8000, 3),
                  "decode_frac": round(gb / d_ms * 1e3 / 8000, 3), "bytes_per_launch_GB": round(gb, 3),
                  "round_trip_mismatches": bad}))
if bad:
    sys.exit(1)
