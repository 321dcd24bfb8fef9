#!/bin/bash
# Round 6, call B: the staging-ring probe (scripts/microbench/ring_probe.hip): fresh
# streams / events / blocks per context, Struct104 8192-record chunk pieces.
set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
P=scripts/microbench/bin/ring_probe
timeout -k 10 200 $P 400 0 1 > $O/ring_nc_fresh.jsonl || exit $?
timeout -k 10 200 $P 400 1 1 > $O/ring_coh_fresh.jsonl || exit $?
timeout -k 10 200 $P 400 0 0 > $O/ring_nc_reuse.jsonl || exit $?
HSA_ENABLE_SDMA=0 timeout -k 10 200 $P 400 0 1 > $O/ring_nc_fresh_nosdma.jsonl || exit $?
tail -qn1 $O/*.jsonl
