import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


# FORY_TEST_HOST_LAST=1 runs the host-path files after every device test: the session order
# in which round 6 saw a fresh host context's first chunk come back zeroed (the null-stream
# arena memset, profiles/r06/intermittent/README.md §5-6). Off by default; the default order
# is the one the round's suites ran.
_HOST_PATH_LAST = ("test_gpu_host.py", "test_gpu_host_copies.py", "test_gpu_windows.py")


def pytest_collection_modifyitems(session, config, items):
    if os.environ.get("FORY_TEST_HOST_LAST") != "1":
        return

    def rank(item):
        name = os.path.basename(str(item.fspath))
        return _HOST_PATH_LAST.index(name) + 1 if name in _HOST_PATH_LAST else 0
    items[:] = sorted(items, key=rank)  # (stable: every other test keeps its place)


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(REPO, "tests", "golden", "schema_hashes.json")) as fh:
        return json.load(fh)


@pytest.fixture(autouse=True)
def _device_drained(request):
    """GPU tests end with the device drained: a kernel's asynchronous fault (an illegal
    address) is reported by the test whose kernels caused it, not by whatever synchronising
    call comes next (rounds 2 and 4 saw faults surface at a later test's torch H2D copy)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
        _check_debug_bounds()


_DBG_SITES = ["enc_mask", "enc_tile", "enc_store", "dec_valid", "dec_tile", "dec_store", "tail_null", "tail_store",
              "tail_valid", "tail_load", "slot_table"]


def _check_debug_bounds():
    """Debug-bounds library (`make debug`, FORY_ROWFMT_LIB=fury_amd/lib/debug/...): the
    fixed-width kernels counted no out-of-range access during the test (fixed.hip,
    FORY_DEBUG_BOUNDS). A product library has no counters (the call returns -1)."""
    import ctypes
    mod = sys.modules.get("fury_amd._lib")
    if mod is None or mod._lib is None:
        return
    f = getattr(mod._lib, "fory_rowfmt_internal_debug_bounds", None)
    if f is None:
        return
    f.restype, f.argtypes = ctypes.c_int, [ctypes.POINTER(ctypes.c_longlong), ctypes.c_int, ctypes.c_int]
    buf = (ctypes.c_longlong * 48)()
    n = f(buf, 16, 1)
    if n == -1:
        return
    assert n > 0, "debug-bounds counters unreadable"
    bad = {(_DBG_SITES[i] if i < len(_DBG_SITES) else str(i)): (buf[3 * i], buf[3 * i + 1], buf[3 * i + 2])
           for i in range(min(n, 16)) if buf[3 * i]}
    assert not bad, f"out-of-range accesses (site: count, first value, limit): {bad}"
