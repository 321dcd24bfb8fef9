#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace + stats of bench.py, then one
# PMC counter group per pass (never combined with sys/runtime traces).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
mkdir -p $OUT
ROWS=${ROWS:-67108864}
BENCH="bench.py --steps 5 --warmup 2 --no-cpu-baseline --total-rows $ROWS --weak-rows 0 ${BENCH_EXTRA}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 $BENCH > $OUT/trace_bench.json 2> $OUT/trace.err
rc=$?; echo "trace exit $rc"; [ $rc -eq 0 ] || exit $rc
for grp in FETCH_SIZE WRITE_SIZE ${EXTRA_PMC}; do
  name=$(echo "$grp" | tr ',' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $(echo $grp | tr ',' ' ') -d $OUT/pmc_$name -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --total-rows $ROWS --weak-rows 0 ${BENCH_EXTRA} > $OUT/pmc_$name.json 2> $OUT/pmc_$name.err
  rc=$?; echo "pmc $grp exit $rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/prof_summary.py $OUT > $OUT/summary.json; echo "summary exit $?"; cat $OUT/summary.json
