#!/bin/bash
# Round-5 step Q: not-null encode v5 with 128-record tiles (one workgroup per CU, 5 chunk
# loads per wave; r128) vs 64 (two per CU; in-tree): parity of r128, then alternating
# Struct104 64Mi raw / stream rates.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=$PWD/gpurun_out/${1:-r05q}
mkdir -p $O
export PYTHONUNBUFFERED=1
FORY_ROWFMT_LIB=fury_amd/lib_ab/libfory_rowfmt_r128.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x \
  -k "not test_varlen_parity and not test_collection_frame_parity" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in intree r128; do
    if [ $v = intree ]; then unset FORY_ROWFMT_LIB; else export FORY_ROWFMT_LIB=fury_amd/lib_ab/libfory_rowfmt_$v.so; fi
    for fr in raw frame; do
      ff=""; [ $fr = frame ] && ff="--frame"
      timeout -k 10 300 python bench.py --config struct104 --extras 0 --no-cpu-baseline --steps 5 --warmup 2 $ff > $O/s104_${v}_${fr}_$r.json 2> $O/s104_${v}_${fr}_$r.err
      rc=$?; echo "s104 $v $fr $r: $(python3 -c "import json; d=json.load(open('$O/s104_${v}_${fr}_$r.json')); k=d['kernels_ms']; print(d['value'], k['encode_avg'], k['decode_avg'])")"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
