#!/bin/bash
# Round 6 closing run on the final build: rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE
# passes of the bench for Struct104 (64Mi rows) and the extra configs (Mixed 16Mi, Nested
# 8Mi; raw and frame-stream), stamped into pmc_latest.json (lib_sha16, trace_ms), then the
# default bench line (which reads that file). Usage: gpu_close.sh TAG (output under
# gpurun_out/TAG; the profiles' trace source names profiles/r06/TAG/prof_*).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-close}
O=gpurun_out/$TAG
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash scripts/r06/gpu_box.sh || exit $?
cp profiles/pmc_latest.json $O/pmc_latest.json
# SPECS (optional): a subset of the configs, to split the closing run over two calls (the
# second starts from the profiles/pmc_latest.json the first left); SKIP_BENCH=1: no bench line
SPECS=${SPECS:-"struct104:67108864: mixed40:16777216: mixed40:16777216:--frame nested:8388608: nested:8388608:--frame"}
for spec in $SPECS; do
  cfg=${spec%%:*}; rest=${spec#*:}; rows=${rest%%:*}; fr=${rest#*:}
  tag=$cfg${fr:+_frame}; fbit=${fr:+1}; fbit=${fbit:-0}
  ex=""; [ "$cfg" = struct104 ] && ex="--extras 0"
  OUT=$O/prof_$tag BENCH_EXTRA="--config $cfg $fr $ex" ROWS=$rows bash scripts/profile.sh > $O/prof_$tag.log 2>&1
  rc=$?; echo "prof $tag exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/pmc_to_traffic.py $O/prof_$tag/summary.json $cfg:$rows:$fbit $O/pmc_latest.json profiles/r06/$TAG/prof_$tag || exit 1
done
cp $O/pmc_latest.json profiles/pmc_latest.json
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench exit $rc"; cut -c1-400 $O/bench.json; [ $rc -eq 0 ] || exit $rc
exit 0
