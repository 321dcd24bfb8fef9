#!/bin/bash
# Round 6: the Struct104 encode's box state, one probe per box: enc_ab
# (product encode v5 vs plain stores vs dispatch order, decode v5; 64Mi records) timed, then
# the same binary under one PMC pass of write-side and wave-wait counters. Output under
# gpurun_out/box/<host>-<time>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
H=$(hostname | tr -cd 'A-Za-z0-9_-' | cut -c1-40)
O=gpurun_out/box/$H-$(date +%H%M%S)
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 scripts/microbench/bin/enc_ab 67108864 1 > $O/enc_ab.jsonl 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
want=""
for c in TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_64B_sum SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR; do
  b=${c%_sum}
  grep -qw "$b" $O/counters.txt && want="$want $c"
done
echo "counters:$want" > $O/pmc_counters.txt
if [ -n "$want" ]; then
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $want -d /tmp/box_pmc -o pmc --output-format csv -- \
    scripts/microbench/bin/enc_ab 67108864 1 > $O/pmc_run.log 2>&1 || { echo "pmc pass exit $?"; exit 1; }
  find /tmp/box_pmc -name "*counter_collection.csv" -exec cp {} $O/counter_collection.csv \;
fi
echo "box probe: $O"
