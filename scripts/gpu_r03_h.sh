#!/bin/bash
# Round 3: counters of the columnar tree engine (holder + bean_a, 524288 records):
# SQ wave-time buckets, then FETCH_SIZE, then WRITE_SIZE, one pass each.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES"
i=0
for grp in "$SQ" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp -d $R/gpurun_out/r03h_pmc$i -o pmc --output-format csv -- python3 $R/scripts/bench_nested_shapes.py 524288 holder,bean_a > $R/gpurun_out/r03h_pmc$i.log 2>&1
  rc=$?; echo "pmc pass $i exit $rc"; [ $rc -eq 0 ] || exit $rc
done
python3 $R/scripts/pmc_kernels.py $R/gpurun_out/r03h_pmc1 $R/gpurun_out/r03h_pmc2 $R/gpurun_out/r03h_pmc3 > $R/gpurun_out/r03h_summary.json
echo "summary exit $?"
