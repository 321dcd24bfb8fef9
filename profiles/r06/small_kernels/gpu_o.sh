#!/bin/bash
# Round 6, call O: the encode sizing kernel at four rows per thread (after call N removed its
# scratch array); parity of the plans it sizes,
# then the Mixed and Nested lines (raw and frames) with a
# kernel trace of the raw pair.
set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_nested.py tests/test_gpu_parity.py tests/test_gpu_v9.py -k "nested or mixed or struct_list or flat_mix or strings or lists or deep or maps or var" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in mixed40 nested; do
  for fr in "" "--frame"; do
    timeout -k 10 300 python -u bench.py --config $cfg $fr --no-cpu-baseline > $O/$cfg$fr.json 2> $O/$cfg$fr.err || exit $?
    python3 -c "import json;d=json.load(open('$O/$cfg$fr.json'));print('$cfg$fr', d['value'], d['kernels_ms'])"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r06o_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config nested --no-cpu-baseline --steps 5 > /tmp/r06o_prof.log 2>&1 || { tail -20 /tmp/r06o_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && find /tmp/r06o_prof -name "*kernel_stats.csv" -exec cp {} $O/nested_kernel_stats.csv \;
grep -E "sizes|encode_flat|decode_flat" $O/nested_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
