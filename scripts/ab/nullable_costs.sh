set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --total-rows 16777216 > gpurun_out/ab_s104_16m.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/ab_s104_16m.json')); k=d['kernels_ms']; print('struct104 notnull 16M', d['value'], k['encode_avg'], k['decode_avg'])"
for nr in 0.0 0.1 0.5; do timeout -k 10 120 python scripts/bench_nullable_fixed.py 16777216 0 $nr || exit 1; done
for x in 16 64; do echo "NULXCD=$x"; FORY_AB_NULXCD=$x timeout -k 10 120 python scripts/bench_nullable_fixed.py 16777216 0 0.1 || exit 1; done
