#!/bin/bash
# Round-5 step V: (1) the pageable host sequence replayed 600 times on the closing library;
# (2) the persistent prefetching decode values pass (A/B build FORY_DEC_PF=1, in
# fury_amd/lib_ab/pf1): varlen parity files, then Mixed 16Mi / Nested 8Mi benches
# alternating with the closing library, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=$PWD/gpurun_out/${1:-r05v2}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/r05/stress_pageable.py 600 > $O/stress.log 2>&1 || exit $?
tail -1 $O/stress.log
PF=$PWD/fury_amd/lib_ab/pf1/libfory_rowfmt.so
FORY_ROWFMT_LIB=$PF timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_nested.py tests/test_gpu_frames.py tests/test_gpu_v9.py > $O/pytest_pf1.log 2>&1 || { tail -30 $O/pytest_pf1.log; exit 1; }
tail -2 $O/pytest_pf1.log
for r in 1 2; do
  for cfg in mixed40 nested; do
    for v in default pf1; do
      if [ $v = pf1 ]; then export FORY_ROWFMT_LIB=$PF; else unset FORY_ROWFMT_LIB; fi
      timeout -k 10 200 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $O/${cfg}_${v}_$r.json 2> $O/${cfg}_${v}_$r.err
      rc=$?; echo "$cfg $v $r: $(python3 -c "import json; d=json.load(open('$O/${cfg}_${v}_$r.json')); k=d['kernels_ms']; print(d['value'], k['encode_call_avg'], k['decode_call_avg'], k['decode_avg'])")"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
