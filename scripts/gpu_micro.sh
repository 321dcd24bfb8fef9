#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 ./scripts/microbench/colread > gpurun_out/colread.jsonl 2> gpurun_out/colread.err
rc=$?; echo "colread exit $rc"; cat gpurun_out/colread.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ab_fixed.py 67108864 2 > gpurun_out/ab.json 2> gpurun_out/ab.err
rc=$?; echo "ab exit $rc"; python -c "import json;d=json.load(open('gpurun_out/ab.json'));[print(k,v.get('enc_ms'),v.get('dec_ms'),v.get('enc_GBs',v.get('enc_GBs_algo')),v.get('dec_GBs')) for k,v in d.items()]"
exit $rc
