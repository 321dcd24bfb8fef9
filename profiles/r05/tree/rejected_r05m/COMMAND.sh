#!/bin/bash
# Round-5 step M: container encode items issued with the containers, list decode items with the header check (in-tree) vs HEAD:
# parity, then alternating Holder / BeanA rates at 2Mi records.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=$PWD/gpurun_out/${1:-r05l}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_treecol.py tests/test_gpu_nested.py -m gpu -q -x \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in intree head; do
    if [ $v = intree ]; then unset FORY_ROWFMT_LIB; else export FORY_ROWFMT_LIB=fury_amd/lib_ab/libfory_rowfmt_$v.so; fi
    timeout -k 10 300 python scripts/bench_nested_shapes.py 2097152 holder,bean_a > $O/shapes_${v}_$r.log 2>&1
    rc=$?; echo "$v $r: $(grep '^{' $O/shapes_${v}_$r.log | python3 -c "import json,sys; d=json.load(sys.stdin); print({k:(v['encode_ms'],v['decode_ms']) for k,v in d.items()})")"; [ $rc -eq 0 ] || exit $rc
  done
done
