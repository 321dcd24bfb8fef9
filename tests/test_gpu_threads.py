"""GPU: launch state is thread-safe (include/fory_rowfmt.h: plans may be shared
across threads and streams). A fresh process starts several host threads that
make their FIRST launches of every kernel family at the same time — fixed-width,
cooperative varlen, generic tile interpreter, frame index — on their own streams,
one of them sharing a plan with another; every result must equal the oracle's.
(ctypes releases the GIL around each C-ABI call, so the threads overlap inside
the library: LDS attributes, CU counts and occupancy answers are cached per
device behind one mutex, fury_amd/csrc/launch_state.cpp.)"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))

SCRIPT = r'''
import os, sys, threading
sys.path.insert(0, os.path.dirname(HERE)); sys.path.insert(0, HERE)
import numpy as np, torch
from helpers import catalog, columns_equal
from oracle import oracle
from fury_amd.format.columns import to_device, to_host
from fury_amd.format.encoder import RowEncoder
torch.cuda.init()
names = ["struct104", "mixed40_nulls", "nested_nulls", "maps", "all_types", "mixed40_nulls", "string_elems", "wide300"]
shared = RowEncoder(catalog()["mixed40_nulls"][0]).plan  # one plan used by two threads (own workspaces)
errors = []
start = threading.Barrier(len(names))
def work(k, name):
    try:
        schema, make = catalog()[name]
        n = 3000 + 17 * k
        cols = make(n, k)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            enc = RowEncoder(schema)
            if name == "mixed40_nulls":
                enc.plan = shared
            dcols = to_device(cols)
            start.wait()
            for frame in (1, 0):
                rows = enc.encode(dcols, n, frame)
                expect, offs = oracle.encode(schema, cols, n, frame)
                got = rows.buffer.cpu().numpy()
                if not np.array_equal(got, expect):
                    errors.append(f"{name} frame {frame}: encode differs"); return
                dec = to_host(enc.decode(rows.buffer, n, frame, None if frame else rows.offsets))
                bad = columns_equal(schema, cols, dec)
                if bad:
                    errors.append(f"{name} frame {frame}: decode differs: {bad[:2]}"); return
    except Exception as e:  # noqa
        errors.append(f"{name}: {type(e).__name__}: {e}")
ts = [threading.Thread(target=work, args=(k, nm)) for k, nm in enumerate(names)]
[t.start() for t in ts]
[t.join() for t in ts]
print("ERRORS" if errors else "OK", errors)
sys.exit(1 if errors else 0)
'''


def test_concurrent_first_launches_from_host_threads():
    code = "HERE = " + repr(HERE) + "\n" + SCRIPT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "OK" in r.stdout
