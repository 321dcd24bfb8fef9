"""CPU: bench.py's multi-rank guards (BASELINE C4 runs one rank per GPU): a run asking
for more GPUs than are visible, or launched with WORLD_SIZE != --gpus, exits non-zero
before measuring anything; two ranks on one device are refused unless the run is an
explicit --oversubscribe rehearsal."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def run_bench(args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    env["HIP_VISIBLE_DEVICES"] = env.get("HIP_VISIBLE_DEVICES", "")
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=300)


def test_more_gpus_than_visible_is_refused():
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("this host has >= 2 GPUs")
    r = run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "refusing" in r.stderr or "GPU(s) visible" in r.stderr


def test_world_size_must_equal_gpus():
    r = run_bench(["--gpus", "1", "--steps", "1", "--warmup", "0"],
                  {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 1" in r.stderr


def test_device_list_must_be_distinct():
    a = {"ordinal": 0, "pci_bus_id": "0000:05:00.0"}
    b = {"ordinal": 1, "pci_bus_id": "0000:15:00.0"}
    assert bench.check_devices([a, b], False) is None
    assert bench.check_devices([a, dict(a)], False) is not None  # same GPU twice
    assert bench.check_devices([a, dict(a)], True) is None  # explicit rehearsal
    # no bus id known: the ordinals decide
    assert bench.check_devices([{"ordinal": 0}, {"ordinal": 0}], False) is not None
    assert bench.check_devices([{"ordinal": 0}, {"ordinal": 1}], False) is None
    assert bench.check_devices([a], False) is None


def test_pmc_traffic_needs_the_same_build(tmp_path):
    import json
    p = tmp_path / "pmc.json"
    json.dump({"struct104:64:0": {"encode": 123, "lib_sha16": "0000000000000000"}}, open(p, "w"))
    assert bench.pmc_traffic(str(p), "struct104", 64, 0, "encode") is None  # another build
    json.dump({"struct104:64:0": {"encode": 123, "lib_sha16": bench.lib_sha16()}}, open(p, "w"))
    assert bench.pmc_traffic(str(p), "struct104", 64, 0, "encode") == 123
    json.dump({"struct104:64:0": {"encode": 123}}, open(p, "w"))  # unstamped
    assert bench.pmc_traffic(str(p), "struct104", 64, 0, "encode") is None


def test_init_dist_goes_through_the_rank_launcher():
    # --init-dist starts torchrun ranks even for --gpus 1, so it is refused the same way
    # when the GPU is not there
    import torch
    if torch.cuda.device_count() >= 1:
        pytest.skip("this host has a GPU")
    r = run_bench(["--gpus", "1", "--init-dist", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "refusing" in r.stderr


def test_stdout_carries_nothing_but_the_line():
    # a rank that fails before measuring prints nothing on stdout (fd 1 points at stderr
    # for the run; only the JSON line goes to the saved stdout)
    r = run_bench(["--gpus", "1", "--steps", "1", "--warmup", "0"],
                  {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert r.stdout == ""
