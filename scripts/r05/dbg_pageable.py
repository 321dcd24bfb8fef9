"""Repeats the pageable fixed-width host encode of test_host_pageable_pieces_over_a_mib
(Struct104, 20011 records, 8192-record chunks, STREAM frames) and reports every
mismatch against the oracle: bytes, frames, chunk, and what the wrong bytes hold."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import numpy as np  # noqa: E402

from oracle import oracle  # noqa: E402
from fury_amd.format.native import HostPipeline, NativePlan  # noqa: E402
from helpers import catalog  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
n = 20011
schema, make = catalog()["struct104"]
cols = make(n, 11)
expect, _ = oracle.encode(schema, cols, n, 1)
stride = expect.nbytes // n
fails = 0
for rep in range(reps):
    hp = HostPipeline(NativePlan(schema), chunk_rows=chunk)
    out = np.zeros(expect.nbytes, np.uint8)
    hp.encode(cols, n, 1, out)
    bad = np.nonzero(out != expect)[0]
    if len(bad):
        fails += 1
        rows = np.unique(bad // stride)
        zero = int((out[bad] == 0).sum())
        print(f"rep {rep}: {len(bad)} bytes differ in {len(rows)} frames {rows[:4].tolist()}..{rows[-3:].tolist()} "
              f"chunks {sorted(set((rows // chunk).tolist()))}, zeros among them {zero}, "
              f"frame {rows[0]} offsets {(bad[bad // stride == rows[0]] - rows[0] * stride)[:12].tolist()} "
              f"got {out[bad[:6]].tolist()} want {expect[bad[:6]].tolist()}", flush=True)
        # is the wrong frame a copy of another frame of the expected stream?
        r0 = rows[0]
        got = out[r0 * stride:(r0 + 1) * stride]
        same = [int(r) for r in range(n) if np.array_equal(expect[r * stride:(r + 1) * stride], got)]
        print(f"  frame {r0} equals expected frames {same[:4]}", flush=True)
    hp.close()
print(f"{fails} of {reps} encodes differ", flush=True)
