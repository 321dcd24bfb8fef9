#!/bin/bash
# rocprofv3 kernel stats + FETCH/WRITE for the varlen configs (default engines).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/prof_mixed BENCH_EXTRA="--config mixed40" ROWS=16777216 bash scripts/profile.sh > gpurun_out/prof_mixed.log 2>&1
rc=$?; echo "prof mixed exit $rc"; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/prof_nested BENCH_EXTRA="--config nested" ROWS=8388608 bash scripts/profile.sh > gpurun_out/prof_nested.log 2>&1
rc=$?; echo "prof nested exit $rc"; [ $rc -eq 0 ] || exit $rc
for d in prof_mixed prof_nested; do
  echo "== $d"; cat gpurun_out/$d/trace_bench.json | cut -c1-600; python3 -c "
import json; d=json.load(open('gpurun_out/$d/summary.json'))
for k,v in d['kernels'].items(): print(k, v['calls'], round(v['avg_ns']/1e3,1), 'us')
for k,v in d['pmc'].items(): print(k, {c: round(x/1e9,3) for c,x in v.items() if c.endswith('bytes') or c.endswith('x2')})
"
done
