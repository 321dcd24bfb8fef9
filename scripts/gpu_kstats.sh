#!/bin/bash
# rocprofv3 kernel-trace stats of bench.py for one config: per-kernel avg times.
# Usage: CONFIG=nested ROWS=8388608 bash scripts/gpu_kstats.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CONFIG=${CONFIG:-struct104}
OUT=gpurun_out/kstats_$CONFIG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o trace --output-format csv -- python3 bench.py --config $CONFIG --steps 5 --warmup 2 --no-cpu-baseline ${ROWS:+--rows $ROWS} ${BENCH_EXTRA} > $OUT/bench.json 2> $OUT/trace.err
rc=$?; echo "trace $CONFIG exit $rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    print(f'{float(r["AverageNs"])/1e3:10.1f} us x{int(r["Calls"]):4d}  {r["Name"][:150]}')
PY
