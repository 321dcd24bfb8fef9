#!/bin/bash
# Round 6, call S: the memset race microbench with the old library's exact order (hipMemset,
# then three new non-blocking streams, the copy on the first), then the first half of the
# closing profiles on the fixed library (Struct104, Mixed, Mixed frames; no bench line).
# Usage: gpu_s.sh TAG (output under gpurun_out/TAG).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-close5}
mkdir -p $O
timeout -k 10 120 scripts/microbench/bin/memset_race 5 100000000 > $O/memset_race.jsonl 2>&1 || { cat $O/memset_race.jsonl; exit 1; }
cat $O/memset_race.jsonl
SPECS="struct104:67108864: mixed40:16777216: mixed40:16777216:--frame" SKIP_BENCH=1 bash scripts/r06/gpu_close.sh ${1:-close5}
