"""CPU: the host path's copy machinery (fury_amd/csrc/host.cpp) against a mock HIP runtime
whose DMAs run late (tests/c/host_copy_mock.cpp, built by `make`).

The machinery under test:
  - the staging ring (block reuse after the block's last DMA, owed D2H host copies);
  - the small-piece buffers (switching between a stream's two buffers);
  - call-scoped registration of caller buffers (pieces, direct DMAs inside them, staged ends);
  - the drain on every return path.

The mock runs an async copy only when something waits for it or when its seeded progress
model picks it, and reads and writes the copy's host bytes at that moment. So a block
reused too early shows up as wrong bytes. A DMA on unpinned memory, or through a range
unregistered or freed before it ran, shows up as a logged violation.

ADVICE r5 (medium) asked for "a CPU test of the staging ring's block-reuse order". The
mutation test shows the mock catches each bug it targets: one host.cpp line changed per
mutant, built against the same mock, and every mutant fails."""
import json
import os
import shutil
import subprocess
import tempfile
from concurrent.futures import ThreadPoolExecutor

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "tests", "c", "host_copy_mock")
HOST_CPP = os.path.join(REPO, "fury_amd", "csrc", "host.cpp")
MOCK_CPP = os.path.join(REPO, "tests", "c", "host_copy_mock.cpp")
DEFS = ["-D__HIP_PLATFORM_AMD__", "-DFORY_STAGE_BLOCK_MB=1", "-DFORY_STAGE_BLOCKS=4", "-DFORY_REG_MIN_KB=64",
        "-DFORY_REG_PIECE_KB=1024"]


def _have_toolchain():
    return shutil.which("g++") and os.path.isdir("/opt/rocm/include/hip")


pytestmark = pytest.mark.skipif(not _have_toolchain(), reason="needs g++ and the HIP headers")


def _build():
    subprocess.run(["make", "-s", "tests/c/host_copy_mock"], cwd=REPO, check=True, capture_output=True, timeout=600)


def _run(binary, seed, timeout=300):
    r = subprocess.run([binary, str(seed)], capture_output=True, text=True, timeout=timeout)
    lines = []
    for l in r.stdout.splitlines():
        try:
            lines.append(json.loads(l))
        except ValueError:  # (a mutant may die mid-line)
            pass
    return r.returncode, lines


@pytest.mark.parametrize("seed", [1, 2])
def test_host_copies_against_late_dmas(seed):
    _build()
    rc, lines = _run(BIN, seed)
    summary = lines[-1]
    bad = [l for l in lines if "failed" in l]
    assert rc == 0 and summary.get("summary") and summary["failures"] == 0 and summary["violations"] == 0, bad[:5]
    # every scenario ran, and the paths it is meant to reach were reached
    assert sum(1 for l in lines if l.get("ok") is True) == 9
    assert summary["staged_pieces"] > 10000 and summary["call_registrations"] > 100


MUTANTS = {
    # a staging block rewritten before the DMA that last used it has run
    "ring reuse without the wait": (
        '    int rc = hip_check(hipEventSynchronize(st.ev[j]), "hipEventSynchronize(staging)");',
        "    int rc = 0;"),
    # a small buffer reused before its DMAs have run
    "small buffer reuse without the wait": (
        '    int rc = hip_check(hipEventSynchronize(sm.ev[b]), "hipEventSynchronize(small staging)");',
        "    int rc = 0;"),
    # a call that returns early leaves its copies queued and unregisters under them
    "no drain when a call returns early": (
        "    for (hipStream_t s : {c->s_in, c->s_k, c->s_out})\n      if (s) (void)hipStreamSynchronize(s);\n"
        "    if (stage_drain(c->stage)) stage_abandon(c->stage);\n",
        ""),
    # a direct DMA that runs past the registered piece it starts in
    "direct DMA past its registration": (
        "    const uintptr_t x0 = std::max(cur, e.lo), x1 = std::min(z, e.hi);",
        "    const uintptr_t x0 = std::max(cur, e.lo), x1 = std::min(z, e.hi + 4096);"),
}


def test_mock_catches_each_mutant():
    src = open(HOST_CPP).read()
    for old, _ in MUTANTS.values():
        assert old in src, old  # the mutated line still exists in the product source
    tmp = tempfile.mkdtemp(prefix="host_mut_")
    try:
        def build_and_run(item):
            name, (old, new) = item
            key = str(abs(hash(name)))
            f = os.path.join(tmp, f"host_{key}.cpp")
            open(f, "w").write(src.replace(old, new, 1))
            exe = os.path.join(tmp, f"mock_{key}")
            subprocess.run(["g++", "-O1", "-std=c++17", "-w", *DEFS, "-I/opt/rocm/include",
                            "-I" + os.path.join(REPO, "fury_amd", "csrc"), f, MOCK_CPP, "-o", exe, "-lpthread"],
                           check=True, capture_output=True, timeout=600)
            return name, _run(exe, 1)

        with ThreadPoolExecutor(max_workers=4) as ex:
            results = dict(ex.map(build_and_run, MUTANTS.items()))
        for name, (rc, lines) in results.items():
            # caught: wrong bytes or a logged violation, or the process died of the bug
            caught = rc < 0 or any("failed" in l for l in lines)
            assert rc != 0 and caught, (name, rc, lines[-1:])
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
