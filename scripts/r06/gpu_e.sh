#!/bin/bash
# Round 6, call E: encode v10 (output-stationary) parity, the host path, Nested / Mixed
# benches with v10 against the round-3 tile kernel (VARENC=1) on one box.
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_os.py > $O/pytest_os.log 2>&1 || { tail -40 $O/pytest_os.log; exit 1; }
tail -1 $O/pytest_os.log
timeout -k 10 600 $T tests/test_gpu_host.py tests/test_gpu_windows.py > $O/pytest_host.log 2>&1 || { tail -30 $O/pytest_host.log; exit 1; }
tail -1 $O/pytest_host.log
B="python -u bench.py --no-cpu-baseline --extras 0 --steps 10 --warmup 3"
for r in 1 2; do
  timeout -k 10 300 $B --config nested > $O/nested_v10_$r.json 2>$O/nested_v10_$r.err || exit 1
  FORY_ROWFMT_VARENC=1 timeout -k 10 300 $B --config nested > $O/nested_r3_$r.json 2>$O/nested_r3_$r.err || exit 1
done
timeout -k 10 300 $B --config nested --frame > $O/nested_v10_frame.json 2>$O/nested_v10_frame.err || exit 1
FORY_ROWFMT_VARENC=10 timeout -k 10 300 $B --config mixed40 > $O/mixed_v10.json 2>$O/mixed_v10.err || exit 1
timeout -k 10 300 $B --config mixed40 > $O/mixed_v9.json 2>$O/mixed_v9.err || exit 1
HOST_MEM=pageable timeout -k 10 300 python -u scripts/host_native.py > $O/host_fixed_pageable.json || exit $?
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d.get('value'), d.get('kernels_ms') or {k:d[k].get('value_GiBs') for k in ('raw','frame') if k in d})")"; done
