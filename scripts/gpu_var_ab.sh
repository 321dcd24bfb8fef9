#!/bin/bash
# Varlen A/B of the in-tree build against LIBS (default: fury_amd/lib_ab/libfory_rowfmt_base.so):
# varlen parity subset first (VARTESTS, pytest -k), then scripts/ab_builds.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_nested.py -x -q --timeout 200 --timeout-method thread -k "${VARTESTS:-varlen_parity or large_round_trip or unaligned or collection or nested}" > gpurun_out/var_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/var_pytest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-2} CONFIGS="${CONFIGS:-nested mixed40}" bash scripts/ab_builds.sh
