#!/bin/bash
# Round-5 step D: registered fixed-width host path (gather launches vs kernels on the host
# mappings vs per-slice copies), and the varlen registered round trip check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05d}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_host.py -m gpu -q -x -k "zero_copy or fixed" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for hp in 0 1 2; do
  FORY_ROWFMT_HOSTPATH=$hp timeout -k 10 300 python scripts/host_native.py 8388608 1048576 > $O/host_fixed_hp$hp.json 2> $O/host_fixed_hp$hp.err
  rc=$?; echo "fixed hostpath $hp exit $rc"; cat $O/host_fixed_hp$hp.json; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python scripts/r05/dbg_var_reg.py 8388608 mixed40 > $O/dbg_var.log 2>&1
rc=$?; cat $O/dbg_var.log; [ $rc -eq 0 ] || exit $rc
REG_BACK=0 timeout -k 10 300 python scripts/r05/dbg_var_reg.py 8388608 mixed40 > $O/dbg_var_noback.log 2>&1
rc=$?; cat $O/dbg_var_noback.log; exit $rc
