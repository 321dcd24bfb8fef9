# Experiment script of a rejected variant (6 waves/SIMD nested encode); its
# FORY_AB_LEAN6 knob left the library with it. Kept as the record of how it was measured.
set -o pipefail
mkdir -p gpurun_out
FORY_AB_LEAN6=1 FORY_ROWFMT_VARDIAG=1 timeout 100 python bench.py --config nested --steps 2 --warmup 1 --no-cpu-baseline 2>&1 >/dev/null | grep "encode" | sort | uniq
for r in 1 2; do
for v in base lean6; do
  if [ $v = lean6 ]; then export FORY_AB_LEAN6=1; else unset FORY_AB_LEAN6; fi
  timeout -k 10 200 python bench.py --config nested --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); k=d['kernels_ms']; print('nested $v', d['value'], k['encode_call_avg'], k['decode_call_avg'])"
done
done
