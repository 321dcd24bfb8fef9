#!/bin/bash
# Round 6, call R: the memset race microbench with its two extra protocols (does a
# hipHostMalloc or hipMalloc between the null-stream hipMemset and the copy wait for the
# null stream?), then the whole GPU suite and smoke on the fixed library.
# Usage: gpu_r.sh TAG (output under gpurun_out/TAG).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r06r}
mkdir -p $O
timeout -k 10 120 scripts/microbench/bin/memset_race 5 100000000 > $O/memset_race.jsonl 2>&1 || { cat $O/memset_race.jsonl; exit 1; }
cat $O/memset_race.jsonl
bash scripts/r06/gpu_final3.sh ${1:-r06r}
