#!/bin/bash
# Round 3: overlap probe (sizing passes on a second stream, chunk by chunk) for Mixed / Nested.
set -o pipefail
mkdir -p gpurun_out
for spec in "mixed40 8" "mixed40 16" "nested 8" "nested 16"; do
  timeout -k 10 240 python -u scripts/overlap_probe.py $spec 5 >> gpurun_out/r03e_overlap.jsonl 2>> gpurun_out/r03e_overlap.err
  rc=$?; echo "probe $spec exit $rc"; [ $rc -eq 0 ] || exit $rc
done
cat gpurun_out/r03e_overlap.jsonl
