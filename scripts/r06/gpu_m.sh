#!/bin/bash
# Round 6, call M: global-qualified loads in the encode sizing kernel (var_sizes_flat_kernel)
# and split LDS / global loads in the tree decode's field pass (td_instance): the varlen and
# tree parity files, then Mixed / Nested bench lines and the tree engine's shapes at 2Mi.
set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_v9.py tests/test_gpu_nested.py tests/test_gpu_treecol.py tests/test_gpu_frames.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in mixed40 nested; do
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline > $O/$cfg.json 2> $O/$cfg.err || exit $?
  python3 -c "import json;d=json.load(open('$O/$cfg.json'));print('$cfg', d['value'], d['kernels_ms'])"
done
timeout -k 10 400 python -u scripts/bench_nested_shapes.py 2097152 bean_a,holder > $O/shapes.log 2>&1 || { tail -20 $O/shapes.log; exit 1; }
grep -E "^(holder|bean_a) " $O/shapes.log
