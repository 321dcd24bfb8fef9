"""GPU: the C-ABI driven from plain C (tests/c/capi_roundtrip.c, built by `make`), the
way a JNI / cgo shim calls it — HIP runtime C API for device memory, no Python or
torch in the process: varlen encode == oracle bytes (raw + frame stream), decode ==
input columns, and the host path (fory_rowfmt_host_*) on a fixed-width schema."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

BIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "capi_roundtrip")


def test_capi_from_c():
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} not built: run `make` (or __graft_entry__.build())")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "capi_roundtrip: all ok" in r.stdout
