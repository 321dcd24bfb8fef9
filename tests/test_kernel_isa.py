"""CPU: properties of the built gfx950 code that the varlen pipelines depend on (DESIGN
§5.10), read from the in-tree object (fury_amd/lib/varlen.o) with the ROCm LLVM tools:

- encode v9 and the decode totals pass contain no flat memory op: a flat load / store /
  atomic counts in both vmcnt and lgkmcnt and completes out of order, so the compiler
  turns every later wait into a full drain and v9's two-tile pipeline collapses;
- encode v9 for Mixed-like plans (4 waves, no fixed-column validity) fits 4 workgroups
  per CU: at most 128 VGPRs and no scratch.
Skipped when the object or the tools are absent (no build in this checkout)."""
import os
import re
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(REPO, "fury_amd", "lib", "varlen.o")
LLVM = "/opt/rocm/lib/llvm/bin"


def _code_object(tmp):
    fb, co = os.path.join(tmp, "fb"), os.path.join(tmp, "co")
    subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", OBJ, fb], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return co


@pytest.fixture(scope="module")
def isa():
    if not os.path.exists(OBJ) or not os.path.exists(f"{LLVM}/llvm-objdump"):
        pytest.skip("no built varlen.o / ROCm LLVM tools")
    with tempfile.TemporaryDirectory() as tmp:
        co = _code_object(tmp)
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True, text=True).stdout
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    flat, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = m.group(1)
            flat.setdefault(cur, 0)
        elif cur and re.search(r"\sflat_(load|store|atomic)", line):
            flat[cur] += 1
    res, name = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            name = m.group(1)
            res[name] = {}
        m = re.match(r"\s+\.(vgpr_count|private_segment_fixed_size):\s+(\d+)", line)
        if m and name:
            res[name][m.group(1)] = int(m.group(2))
    return flat, res


def test_v9_and_decode_totals_have_no_flat_ops(isa):
    flat, _ = isa
    v9 = {k: v for k, v in flat.items() if "var_encode_flat9" in k}
    tot = {k: v for k, v in flat.items() if re.search(r"var_decode_flat_kernelILi\d+ELb0E", k)}
    assert v9 and tot
    assert all(v == 0 for v in v9.values()), {k: v for k, v in v9.items() if v}
    assert all(v == 0 for v in tot.values()), {k: v for k, v in tot.items() if v}


def test_v9_mixed_instantiation_fits_four_workgroups(isa):
    _, res = isa
    # var_encode_flat9_kernel<HDR, NW=4, OWN=2, K=2, NUL=2> (var-field validity only)
    ks = [k for k in res if re.search(r"var_encode_flat9_kernelILi\d+ELi4ELi2ELi2ELi2E", k)]
    assert len(ks) == 3  # HDR 0 / 8 / 12
    for k in ks:
        assert res[k]["vgpr_count"] <= 128, (k, res[k])
        assert res[k].get("private_segment_fixed_size", 0) == 0, (k, res[k])
