#!/bin/bash
# Varlen iteration: GPU parity tests, then the varlen engine A/B (mixed40, nested).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc; fi
for cfg in ${CFGS:-mixed40 nested}; do
  timeout -k 10 400 python scripts/ab_varlen.py $cfg > gpurun_out/ab_$cfg.json 2> gpurun_out/ab_$cfg.err
  rc=$?; echo "ab $cfg exit $rc"; tail -3 gpurun_out/ab_$cfg.err
  python -c "import json,sys;d=json.load(open('gpurun_out/ab_$cfg.json'));[print(k,v) for k,v in d.items()]" || exit 1
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python scripts/var_timeline.py mixed40 > gpurun_out/timeline_mixed.json 2> gpurun_out/timeline.err
rc=$?; echo "timeline exit $rc"; python -c "
import json; d=json.load(open('gpurun_out/timeline_mixed.json'))
for k,v in d.items(): print(k, {a:(b['median_us'] if isinstance(b,dict) else b) for a,b in v.items()})"
exit $rc
