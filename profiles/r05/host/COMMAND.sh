#!/bin/bash
# Round-5 step I: host path after removing the gather / direct forms (per-slice DMAs with
# registry-resolved mappings; 16 MiB staging pieces, up to 16 copy threads): host tests,
# registered and pageable rates, fixed and varlen.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05i}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_windows.py -m gpu -q -x \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for mem in registered pageable; do
  HOST_MEM=$mem timeout -k 10 300 python scripts/host_native.py 8388608 1048576 > $O/host_fixed_$mem.json 2> $O/host_fixed_$mem.err
  rc=$?; echo "fixed $mem exit $rc"; cat $O/host_fixed_$mem.json; [ $rc -eq 0 ] || exit $rc
  HOST_MEM=$mem timeout -k 10 400 python scripts/host_native_var.py 8388608 > $O/host_var_$mem.json 2> $O/host_var_$mem.err
  rc=$?; echo "var $mem exit $rc"; cat $O/host_var_$mem.json; [ $rc -eq 0 ] || exit $rc
done
# tree engine: the container decode with two item groups in flight per lane
timeout -k 10 600 python -u -m pytest tests/test_gpu_treecol.py tests/test_gpu_nested.py -m gpu -q -x \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_tree.log 2>&1
rc=$?; tail -3 $O/pytest_tree.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_nested_shapes.py 2097152 holder,bean_a > $O/shapes.log 2>&1
rc=$?; grep "^{" $O/shapes.log; exit $rc
