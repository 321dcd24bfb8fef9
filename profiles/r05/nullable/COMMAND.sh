#!/bin/bash
# Nullable fixed-width v5 (mask tables, ballot validity) + host zero copy: parity tests,
# then an alternating A/B of the nullable encode/decode at 16Mi boxed Struct104 records
# (in-tree vs the 1-workgroup-per-CU variant vs the round-4 build), then host rates.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05nul}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host.py tests/test_gpu_capi_c.py -m gpu -q -x \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
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
for mem in registered pageable; do
  HOST_MEM=$mem timeout -k 10 300 python scripts/host_native.py 8388608 1048576 > $O/host_fixed_$mem.json 2> $O/host_fixed_$mem.err
  rc=$?; echo "fixed $mem exit $rc"; cat $O/host_fixed_$mem.json; [ $rc -eq 0 ] || exit $rc
  HOST_MEM=$mem timeout -k 10 400 python scripts/host_native_var.py 8388608 > $O/host_var_$mem.json 2> $O/host_var_$mem.err
  rc=$?; echo "var $mem exit $rc"; cat $O/host_var_$mem.json; [ $rc -eq 0 ] || exit $rc
done
