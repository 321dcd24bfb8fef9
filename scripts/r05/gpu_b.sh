#!/bin/bash
# Round-5 step B: parity of encode v9n (struct / list plans), nullable fixed v5 and the host
# zero copy; A/B of the nullable kernels (in-tree vs 1-WG variant vs round-4 build) and of
# Nested encode v9n vs the round-3 tile kernel; host-inclusive rates.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05b}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "v9n or boxed or all_types or struct104" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_parity.log 2>&1
rc=$?; tail -3 $O/pytest_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_capi_c.py tests/test_gpu_v9.py tests/test_gpu_nested.py \
  -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_host.log 2>&1
rc=$?; tail -3 $O/pytest_host.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in new nul1wg r04; do
    if [ $lib = new ]; then unset FORY_ROWFMT_LIB; else export FORY_ROWFMT_LIB=fury_amd/lib_ab/libfory_rowfmt_$lib.so; fi
    for fr in 0 1; do
      timeout -k 10 120 python scripts/bench_nullable_fixed.py 16777216 $fr 0.1 > $O/nul_${lib}_${fr}_$r.json 2>$O/nul_${lib}_${fr}_$r.err
      rc=$?; echo "$lib frame $fr: $(cat $O/nul_${lib}_${fr}_$r.json)"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
unset FORY_ROWFMT_LIB
for r in 1 2; do
  for e in 0 10; do
    FORY_ROWFMT_VARENC=$e timeout -k 10 200 python bench.py --config nested --steps 10 --warmup 3 --no-cpu-baseline > $O/nested_e${e}_$r.json 2>$O/nested_e${e}_$r.err
    rc=$?; [ $rc -eq 0 ] || exit $rc
    python3 -c "import json; d=json.load(open('$O/nested_e${e}_$r.json')); k=d['kernels_ms']; print('nested enc=$e', d['value'], k['encode_call_avg'], k['decode_call_avg'], k['encode_avg'], k['decode_avg'])"
  done
done
for mem in registered pageable; do
  HOST_MEM=$mem timeout -k 10 300 python scripts/host_native.py 8388608 1048576 > $O/host_fixed_$mem.json 2> $O/host_fixed_$mem.err
  rc=$?; echo "fixed $mem exit $rc"; cat $O/host_fixed_$mem.json; [ $rc -eq 0 ] || exit $rc
  HOST_MEM=$mem timeout -k 10 400 python scripts/host_native_var.py 8388608 > $O/host_var_$mem.json 2> $O/host_var_$mem.err
  rc=$?; echo "var $mem exit $rc"; cat $O/host_var_$mem.json; [ $rc -eq 0 ] || exit $rc
done
