#!/bin/bash
# Encode v7 (strings through registers): varlen parity, then A/B against the round-3 encode
# (FORY_ROWFMT_VARENC=1) on the Mixed / Nested benches and phase timelines, one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04d
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py tests/test_gpu_nested.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for enc in 0 1 2; do
    for cfg in mixed40 nested; do
      # enc 2: encode v7 + the decode staging its rows through registers (FORY_ROWFMT_DECREGS=1)
      FORY_ROWFMT_DECREGS=$([ $enc -eq 2 ] && echo 1 || echo 0) FORY_ROWFMT_VARENC=$([ $enc -eq 1 ] && echo 1 || echo 0) FORY_ROWFMT_VARDIAG=1 timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > $O/ab_${cfg}_enc${enc}_$rep.json 2> $O/ab_${cfg}_enc${enc}_$rep.err
      rc=$?; [ $rc -eq 0 ] || exit $rc
      python -c "import json,sys; d=json.load(open('$O/ab_${cfg}_enc${enc}_$rep.json')); print('$cfg enc$enc rep$rep', d['value'], d['kernels_ms'])"
    done
  done
done
grep -h "encode" $O/ab_*_1.err | sort | uniq -c
for cfg in mixed40 nested; do
  FORY_ROWFMT_VARDIAG=1 timeout -k 10 200 python bench.py --config $cfg --frame --steps 10 --warmup 3 --no-cpu-baseline > $O/frame_${cfg}.json 2> $O/frame_${cfg}.err
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python -c "import json,sys; d=json.load(open('$O/frame_${cfg}.json')); print('$cfg frame', d['value'], d['kernels_ms'])"
  grep -h "decode" $O/frame_${cfg}.err | sort | uniq -c
done
for cfg in mixed40 nested; do
  timeout -k 10 200 python scripts/var_timeline.py $cfg > $O/timeline_${cfg}.json 2> $O/timeline_${cfg}.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 $O/timeline_${cfg}.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('$O/timeline_${cfg}.json'))
for k,v in d.items():
    if 'decode' in k: continue
    print(k, 'life', v.get('tile_life_us_median'), 'resident', v.get('avg_resident_tiles'), 'span', v.get('kernel_span_us'), {a:b['median_us'] for a,b in v.items() if isinstance(b,dict)})
"
done
