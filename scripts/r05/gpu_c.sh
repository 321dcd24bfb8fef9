#!/bin/bash
# Round-5 step C: v9n parity (both chunk sizes), host tests, Nested A/B (round-3 kernel vs
# v9n 64-B / 128-B first chunks), host-inclusive rates, tree-engine kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05c}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host.py -m gpu -q -x -k "v9n or host" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for e in 0 10 11; do
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
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tree -o tree -- python3 scripts/bench_nested_shapes.py 2097152 holder,bean_a > $O/tree.log 2>&1
rc=$?; tail -4 $O/tree.log; exit $rc
