"""Replays the sequence of test_host_pageable_pieces_over_a_mib (tests/test_gpu_host.py)
in one process many times -- Mixed-with-nulls, then Struct104, then Nested-with-nulls,
each on a fresh host context with pageable caller memory -- and reports every encode
whose bytes differ from the oracle (the round's one intermittent failure was the
Struct104 case right after the Mixed case: profiles/r05/intermittent/README.md)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from oracle import oracle  # noqa: E402
from fury_amd.format.native import HostPipeline, NativePlan  # noqa: E402
from helpers import catalog  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
cases = [("mixed40_nulls", 40009, 1 << 20), ("struct104", 20011, 8192), ("nested_nulls", 60013, 16384)]
prep = []
for name, n, chunk in cases:
    schema, make = catalog()[name]
    cols = make(n, 11)
    expect, eoffs = oracle.encode(schema, cols, n, 1)
    prep.append((name, n, chunk, schema, cols, expect, eoffs))

fails = 0
t0 = time.time()
for rep in range(reps):
    for name, n, chunk, schema, cols, expect, eoffs in prep:
        hp = HostPipeline(NativePlan(schema), chunk_rows=chunk)
        if name == "struct104":
            out = np.zeros(expect.nbytes, np.uint8)
            hp.encode(cols, n, 1, out)
        else:
            out, offs = hp.encode_var(cols, n, 1, np.zeros(expect.nbytes, np.uint8))
            if not np.array_equal(offs, eoffs):
                print(f"rep {rep} {name}: offsets differ", flush=True)
                fails += 1
        bad = np.nonzero(out != expect)[0]
        if len(bad):
            fails += 1
            offs_e = eoffs if eoffs is not None else np.arange(n + 1, dtype=np.int64) * (expect.nbytes // n)
            frames = np.unique(np.searchsorted(offs_e, bad, side="right") - 1)
            f0 = int(frames[0])
            got = out[offs_e[f0]:offs_e[f0 + 1]]
            same = [int(r) for r in range(n) if offs_e[r + 1] - offs_e[r] == len(got)
                    and np.array_equal(expect[offs_e[r]:offs_e[r + 1]], got)][:4]
            print(f"rep {rep} {name}: {len(bad)} bytes differ in {len(frames)} frames "
                  f"{frames[:6].tolist()}..{frames[-3:].tolist()}, chunks {sorted(set((frames // chunk).tolist()))[:8]}, "
                  f"zeros {int((out[bad] == 0).sum())}, frame {f0} equals expected frames {same}", flush=True)
        hp.close()
    if rep % 10 == 9:
        print(f"{rep + 1} reps, {fails} failures, {time.time() - t0:.0f} s", flush=True)
print(f"{fails} failing encodes in {reps} x {len(cases)}", flush=True)
