#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 ./scripts/microbench/colread > gpurun_out/colread2.jsonl 2> gpurun_out/colread2.err
rc=$?; echo "colread exit $rc"; grep -E "dec_traffic|enc_traffic|copy" gpurun_out/colread2.jsonl; exit $rc
