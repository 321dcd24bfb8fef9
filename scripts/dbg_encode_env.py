"""Diagnostic: Struct104 encode time alone vs interleaved with decode (bench layout)."""
import os, sys, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import bench
from fury_amd.format import native
from fury_amd.format.encoder import RowEncoder

n = 64 << 20
dev = torch.device("cuda", 0)
schema, cols, col_bytes = bench.make_batch("struct104", n, 0, dev)
enc = RowEncoder(schema, device=dev)
p = enc.plan
ws = enc.workspace(n)
stride = p.stride(0)
out = torch.empty(n * stride, dtype=torch.uint8, device=dev)
dcols = enc.alloc_fixed_outputs(n)
a_in, a_out = native.column_array(cols), native.column_array(dcols)
status = torch.zeros(1, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream().cuda_stream

def t(fn, reps=6):
    for _ in range(2): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = []
    for _ in range(reps):
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ms.append(e0.elapsed_time(e1))
    return round(sum(ms) / len(ms), 3)

encode = lambda: native.encode(p, a_in, n, 0, None, out, status, ws, s)
decode = lambda: native.decode(p, out, None, n, 0, a_out, status, ws, s)
res = {"encode_alone": t(encode), "decode_alone": t(decode)}
def pair():
    encode(); decode()
res["encode+decode_pair"] = t(pair)
# encode right after a decode
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ms = []
for _ in range(6):
    decode(); e0.record(); encode(); e1.record(); torch.cuda.synchronize(); ms.append(e0.elapsed_time(e1))
res["encode_after_decode"] = round(sum(ms) / len(ms), 3)
# columns copied into fresh separate allocations
cols2 = [native.DeviceColumn(c.values.clone(), None, None, n) for c in cols]
torch.cuda.synchronize()
a_in2 = native.column_array(cols2)
res["encode_alone_cloned_cols"] = t(lambda: native.encode(p, a_in2, n, 0, None, out, status, ws, s))
addrs = sorted(c.values.data_ptr() for c in cols)
res["col_addr_gaps_MiB"] = sorted(set(((b - a) >> 20) for a, b in zip(addrs, addrs[1:])))[:12]
print(json.dumps(res))
