#!/bin/bash
# Round-5 step H: host path with registry-resolved mappings (no runtime pointer queries per
# copy): registered rates for the three fixed-width forms, a timeline of the per-slice form,
# and the tree-engine kernel stats after the container-encode change.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=$PWD/gpurun_out/${1:-r05h}
R=$PWD
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_host.py -m gpu -q -x \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for hp in 2 0 1; do
  FORY_ROWFMT_HOSTPATH=$hp timeout -k 10 300 python scripts/host_native.py 8388608 1048576 > $O/host_fixed_hp$hp.json 2> $O/host_fixed_hp$hp.err
  rc=$?; echo "fixed hostpath $hp exit $rc"; cat $O/host_fixed_hp$hp.json; [ $rc -eq 0 ] || exit $rc
done
HOST_MEM=pageable timeout -k 10 300 python scripts/host_native.py 8388608 1048576 > $O/host_fixed_pageable.json 2> $O/host_fixed_pageable.err
rc=$?; echo "fixed pageable exit $rc"; cat $O/host_fixed_pageable.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
FORY_ROWFMT_HOSTPATH=2 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d $O/trace_hp2 -o t -- python3 $R/scripts/host_native.py 4194304 1048576 > $O/trace_hp2.log 2>&1
rc=$?; echo "trace exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tree -o tree -- python3 $R/scripts/bench_nested_shapes.py 2097152 holder,bean_a > $O/tree.log 2>&1
rc=$?; grep "^{" $O/tree.log; exit $rc
