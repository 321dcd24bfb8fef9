"""Debug: host-pipeline encode after the fixed parity tests (reproduces a mismatch)."""
import os, sys, subprocess
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
from helpers import catalog
from oracle import oracle
from fury_amd.format.native import HostPipeline, NativePlan
from fury_amd.format.columns import to_device
from fury_amd.format.encoder import RowEncoder

schema, make = catalog()["struct104"]
def host_once(tag):
    n = 5000
    cols = make(n, n + 7)
    expect, _ = oracle.encode(schema, cols, n, 0)
    plan = NativePlan(schema)
    hp = HostPipeline(plan, chunk_rows=1000)
    out = np.zeros(expect.nbytes, np.uint8)
    hp.encode(cols, n, 0, out)
    hp.close()
    bad = np.nonzero(out != expect)[0]
    rows = np.unique(bad // 848)
    print(tag, "bad bytes", len(bad), "rows", len(rows), rows[:10], rows[-5:] if len(rows) else None, flush=True)
    if len(rows):
        r = rows[0]
        got = out[r*848:(r+1)*848].view(np.uint32)[4:20]
        exp = expect[r*848:(r+1)*848].view(np.uint32)[4:20]
        print(" got", got, "\n exp", exp, flush=True)
        # is the bad row equal to some other expected row?
        e = expect.reshape(n, 848)
        o = out.reshape(n, 848)
        m = np.nonzero((e == o[r]).all(1))[0]
        print(" row", r, "equals expected rows", m[:5], flush=True)
host_once("fresh")
enc = RowEncoder(schema)
for n in (0, 1, 7, 63, 64, 65, 1000, 4097):
    c = make(n, n)
    for fr in (0, 1, 3):
        rows = enc.encode(to_device(c), n, fr)
        enc.decode(rows)
host_once("after parity-like")
