#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 ./scripts/microbench/copybw > gpurun_out/copybw.jsonl 2> gpurun_out/copybw.err
rc=$?; echo "copybw exit $rc"; cat gpurun_out/copybw.jsonl; exit $rc
