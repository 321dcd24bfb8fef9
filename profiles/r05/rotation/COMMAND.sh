#!/bin/bash
# Round-5 step N: encode v5 with rotated record order per chunk (LDS bank spread) vs
# in-order (norot = HEAD): fixed-width parity, then alternating Struct104 (not-null, 64Mi,
# raw and stream) and boxed Struct104 (nullable, 16Mi, raw and stream).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=$PWD/gpurun_out/${1:-r05n}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capi_c.py -m gpu -q -x -k "not varlen" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in intree norot; do
    if [ $v = intree ]; then unset FORY_ROWFMT_LIB; else export FORY_ROWFMT_LIB=fury_amd/lib_ab/libfory_rowfmt_$v.so; fi
    for fr in raw frame; do
      ff=""; [ $fr = frame ] && ff="--frame"
      timeout -k 10 300 python bench.py --config struct104 --extras 0 --no-cpu-baseline --steps 5 --warmup 2 $ff > $O/s104_${v}_${fr}_$r.json 2> $O/s104_${v}_${fr}_$r.err
      rc=$?; echo "s104 $v $fr $r: $(python3 -c "import json; d=json.load(open('$O/s104_${v}_${fr}_$r.json')); k=d['kernels_ms']; print(d['value'], k['encode_avg'], k['decode_avg'])")"; [ $rc -eq 0 ] || exit $rc
    done
    for fr in 0 1; do
      timeout -k 10 120 python scripts/bench_nullable_fixed.py 16777216 $fr 0.1 > $O/nul_${v}_${fr}_$r.json 2> $O/nul_${v}_${fr}_$r.err
      rc=$?; echo "nul $v $fr $r: $(python3 -c "import json; d=json.load(open('$O/nul_${v}_${fr}_$r.json')); print(d['encode_ms'], d['decode_ms'], d['round_trip_mismatches'])")"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
