#!/bin/bash
# Varlen configs: bench lines (raw + frame-stream) and a rocprofv3 kernel trace of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/var}
mkdir -p $OUT
for cfg in mixed40 nested; do
  for fr in "" "--frame"; do
    tag=$cfg${fr:+_frame}
    timeout -k 10 300 python bench.py --config $cfg $fr --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err
    rc=$?; echo "bench $tag exit $rc"; [ $rc -eq 0 ] || exit $rc
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$cfg -o trace --output-format csv -- python3 bench.py --config $cfg --frame --steps 5 --warmup 2 --no-cpu-baseline > $OUT/trace_$cfg.json 2> $OUT/trace_$cfg.err
  rc=$?; echo "trace $cfg exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/prof_summary.py $OUT/trace_$cfg > $OUT/summary_$cfg.json
done
for f in $OUT/bench_*.json; do echo "== $f"; python3 -c "
import json,sys; d=json.load(open('$f')); print(d['value'], d['kernels_ms'], d['roofline']['frac'], d['roofline'].get('call_frac'))"; done
for cfg in mixed40 nested; do python3 -c "
import json; d=json.load(open('$OUT/summary_$cfg.json'))
for k,v in d['kernels'].items(): print('$cfg', k, v['calls'], round(v['avg_ns']/1e3,1), 'us')"; done
