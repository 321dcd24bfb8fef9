#!/bin/bash
# Round-4 closing run, part C: the struct104 profile without the extra configs (their
# kernels would mix into its summary), stamped into pmc_latest.json, then the default bench
# line again, and the host-inclusive rates (registered and pageable buffers).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04close
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cp profiles/pmc_latest.json $O/pmc_latest.json
OUT=$O/prof_struct104 BENCH_EXTRA="--config struct104 --extras 0" ROWS=67108864 bash scripts/profile.sh > $O/prof_struct104.log 2>&1
rc=$?; echo "prof struct104 exit $rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_to_traffic.py $O/prof_struct104/summary.json struct104:67108864:0 $O/pmc_latest.json profiles/r04/prof_struct104 || exit 1
cp $O/pmc_latest.json profiles/pmc_latest.json
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench exit $rc"; cut -c1-300 $O/bench.json; [ $rc -eq 0 ] || exit $rc
bash scripts/r04/gpu_host.sh
