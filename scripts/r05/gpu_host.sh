#!/bin/bash
# Host path: GPU tests of test_gpu_host.py, then host-inclusive rates,
# registered (zero copy for fixed-width plans) and pageable (staged, parallel memcpy).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05host}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py -m gpu -q -x --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_host.log 2>&1
rc=$?; tail -3 $O/pytest_host.log; [ $rc -eq 0 ] || exit $rc
for mem in registered pageable; do
  HOST_MEM=$mem timeout -k 10 300 python scripts/host_native.py 8388608 1048576 > $O/host_fixed_$mem.json 2> $O/host_fixed_$mem.err
  rc=$?; echo "fixed $mem exit $rc"; cat $O/host_fixed_$mem.json; [ $rc -eq 0 ] || exit $rc
  HOST_MEM=$mem timeout -k 10 400 python scripts/host_native_var.py 8388608 > $O/host_var_$mem.json 2> $O/host_var_$mem.err
  rc=$?; echo "var $mem exit $rc"; cat $O/host_var_$mem.json; [ $rc -eq 0 ] || exit $rc
done
