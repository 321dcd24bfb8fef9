#!/bin/bash
# Fixed-width A/B of the in-tree build against fury_amd/lib_ab/libfory_rowfmt_base.so:
# fixed-width parity subset first, then Struct104 (bench.py) and nullable Struct104
# (scripts/bench_nullable_fixed.py), alternating builds, ROUNDS times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host.py -x -q --timeout 200 --timeout-method thread -k "encode_decode_parity or nullable_fixed or fixed_decode_into or struct_large or host" > gpurun_out/nul_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/nul_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in $(seq ${ROUNDS:-2}); do
for lib in new base; do
  if [ $lib = base ]; then export FORY_ROWFMT_LIB=${BASELIB:-fury_amd/lib_ab/libfory_rowfmt_base.so}; else unset FORY_ROWFMT_LIB; fi
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_s104_$lib.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab_s104_$lib.json')); k=d['kernels_ms']; print('struct104 $lib', d['value'], k['encode_avg'], k['decode_avg'])"
  for fr in 0 1; do
    timeout -k 10 120 python scripts/bench_nullable_fixed.py 16777216 $fr || exit 1
  done
done
done
