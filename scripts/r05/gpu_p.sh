#!/bin/bash
# Round-5 step P: tree-engine instance images at an odd-dword LDS pitch (intree) vs the
# pitch of their size (treehead), and encode / decode v5 record rotation as kept (encode
# always, decode for nullable plans; intree) vs none (norot): parity, then alternating rates.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=$PWD/gpurun_out/${1:-r05p}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_treecol.py tests/test_gpu_nested.py tests/test_gpu_capi_c.py \
  -m gpu -q -x -k "not test_varlen_parity and not test_collection_frame_parity" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in intree treehead; do
    if [ $v = intree ]; then unset FORY_ROWFMT_LIB; else export FORY_ROWFMT_LIB=fury_amd/lib_ab/libfory_rowfmt_$v.so; fi
    timeout -k 10 300 python scripts/bench_nested_shapes.py 2097152 holder,bean_a > $O/shapes_${v}_$r.log 2>&1
    rc=$?; echo "$v $r: $(grep '^{' $O/shapes_${v}_$r.log | python3 -c "import json,sys; d=json.load(sys.stdin); print({k:(v['encode_ms'],v['decode_ms']) for k,v in d.items()})")"; [ $rc -eq 0 ] || exit $rc
  done
done
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
