#!/bin/bash
# Round-5 step Y: the decode totals pass staging only each record's fixed part (string-only
# flat plans; A/B build in fury_amd/lib_ab/fr1): varlen parity files, then Mixed 16Mi raw and
# frame-stream benches alternating with the closing library, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=$PWD/gpurun_out/${1:-r05y}
mkdir -p $O
export PYTHONUNBUFFERED=1
FR=$PWD/fury_amd/lib_ab/fr1/libfory_rowfmt.so
FORY_ROWFMT_LIB=$FR timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_frames.py tests/test_gpu_v9.py tests/test_gpu_host.py > $O/pytest_fr1.log 2>&1 || { tail -30 $O/pytest_fr1.log; exit 1; }
tail -1 $O/pytest_fr1.log
for r in 1 2; do
  for fm in raw frame; do
    for v in default fr1; do
      if [ $v = fr1 ]; then export FORY_ROWFMT_LIB=$FR; else unset FORY_ROWFMT_LIB; fi
      fl=""; [ $fm = frame ] && fl="--frame"
      timeout -k 10 200 python bench.py --config mixed40 $fl --steps 5 --warmup 2 --no-cpu-baseline > $O/${fm}_${v}_$r.json 2> $O/${fm}_${v}_$r.err
      rc=$?; echo "$fm $v $r: $(python3 -c "import json; d=json.load(open('$O/${fm}_${v}_$r.json')); k=d['kernels_ms']; print(d['value'], k['encode_call_avg'], k['decode_call_avg'], k['decode_avg'], k.get('frame_index_avg'))")"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
