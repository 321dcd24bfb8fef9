#!/bin/bash
# Round-5 step S: pinned staging / scratch / table slots / status word as coherent host
# memory: host tests, pageable and registered rates (fixed and varlen).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05s}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_windows.py -m gpu -q -x \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for mem in pageable registered; do
  HOST_MEM=$mem timeout -k 10 300 python scripts/host_native.py 8388608 1048576 > $O/host_fixed_$mem.json 2> $O/host_fixed_$mem.err
  rc=$?; echo "fixed $mem: $(python3 -c "import json; d=json.load(open('$O/host_fixed_$mem.json')); print(d['raw']['value_GiBs'], d['frame']['value_GiBs'])")"; [ $rc -eq 0 ] || exit $rc
  HOST_MEM=$mem timeout -k 10 400 python scripts/host_native_var.py 8388608 > $O/host_var_$mem.json 2> $O/host_var_$mem.err
  rc=$?; echo "var $mem: $(python3 -c "import json; d=json.load(open('$O/host_var_$mem.json')); print([(c, d[c]['value_GiBs'], d[c]['value_GiBs_decode_into'], d[c]['frames_equal_first_call']) for c in ('mixed40','nested')])")"; [ $rc -eq 0 ] || exit $rc
done
