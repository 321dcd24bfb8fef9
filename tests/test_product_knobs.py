"""CPU: the product library reads no knob that changes the bytes it writes or skips work.

Round 4 had a timing knob (FORY_ROWFMT_DBGSKIP) that made the default encode skip its image
store and still return OK, and a rejected kernel (encode v8) compiled into the shipped
library. Every environment knob is read in one place (launch_state.cpp: knobs_from_env, at
plan creation); this test pins that list to the engine / budget selectors whose every choice
the GPU parity suite checks byte for byte, and checks the built library holds neither the
debug knob nor the rejected kernels."""
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "fury_amd", "csrc")
LIB = os.path.join(REPO, "fury_amd", "lib", "libfory_rowfmt.so")

# each selects an engine, a kernel form or an LDS budget (all byte-identical: tests/test_gpu_*),
# or turns on timeline stamps / diagnostics to stderr next to the normal output
ALLOWED = {
    "FORY_ROWFMT_VARTILE", "FORY_ROWFMT_VARFLAT", "FORY_ROWFMT_VARCAP", "FORY_ROWFMT_VARFIT",
    "FORY_ROWFMT_VARSTG", "FORY_ROWFMT_SPILLCAP", "FORY_ROWFMT_VARNW", "FORY_ROWFMT_SIZES_PROGRAM",
    "FORY_ROWFMT_IDXFRAMES", "FORY_ROWFMT_VARPROF", "FORY_ROWFMT_VARDIAG", "FORY_ROWFMT_VARENC",
    "FORY_ROWFMT_VARXCD", "FORY_ROWFMT_DECREGS", "FORY_ROWFMT_TREECOL",
    "FORY_ROWFMT_HOST_VERIFY",  # host path: reads back and checks its H2D pieces (same bytes, slower)
}


def sources():
    for name in sorted(os.listdir(CSRC)):
        if name.endswith((".hip", ".cpp", ".h")):
            with open(os.path.join(CSRC, name), encoding="utf-8") as f:
                yield name, f.read()


def test_knobs_are_read_once_and_are_selectors():
    seen = {}
    for name, src in sources():
        for m in re.finditer(r'getenv\("([A-Z_0-9]+)"\)|(?:num|set)\("([A-Z_0-9]+)"', src):
            seen.setdefault(m.group(1) or m.group(2), set()).add(name)
    fory = {k: v for k, v in seen.items() if k.startswith("FORY_ROWFMT")}
    assert set(fory) <= ALLOWED, set(fory) - ALLOWED
    assert all(v == {"launch_state.cpp"} for v in fory.values()), fory  # read in one place only


def test_no_debug_skip_or_rejected_kernels_in_the_sources():
    for name, src in sources():
        assert "DBGSKIP" not in src and "dbg_skip" not in src, name
        assert "flat8" not in src and "flat9_lean" not in src and "flat9n" not in src, name


def test_the_built_library_holds_no_debug_knob():
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    with open(LIB, "rb") as f:
        blob = f.read()
    assert b"FORY_ROWFMT_DBGSKIP" not in blob
    assert b"var_encode_flat8_kernel" not in blob and b"var_encode_flat9_lean_kernel" not in blob
    assert b"var_encode_flat9n_kernel" not in blob  # round 5: measured slower than the round-3 kernel
    assert b"var_encode_flat9_kernel" in blob  # (the default Mixed encode is there)
