#!/bin/bash
# Round 6, call I: decode totals gathered by the frame index (fory_rowfmt_decode_sizes_stream):
# frame + parity tests, then Mixed / Nested frame-stream bench A/B (FORY_ROWFMT_STREAMSIZES
# 1 = fused, 0 = index_frames + decode_sizes), two alternating rounds, and a kernel trace.
set -o pipefail
O=gpurun_out/r06i
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
hostname > $O/host.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_frames.py > $O/pytest_frames.log 2>&1 || { tail -40 $O/pytest_frames.log; exit 1; }
tail -1 $O/pytest_frames.log
for r in 1 2; do
  for k in 1 0; do
    FORY_ROWFMT_STREAMSIZES=$k timeout -k 10 300 python -u bench.py --config mixed40 --frame --no-cpu-baseline \
      > $O/mixed_frame_k${k}_$r.json 2> $O/mixed_frame_k${k}_$r.err || exit $?
    python3 -c "import json;d=json.load(open('$O/mixed_frame_k${k}_$r.json'));print('mixed frame k$k r$r', d['value'], d['kernels_ms'])"
  done
done
timeout -k 10 300 python -u bench.py --config nested --frame --no-cpu-baseline > $O/nested_frame.json 2> $O/nested_frame.err || exit $?
python3 -c "import json;d=json.load(open('$O/nested_frame.json'));print('nested frame', d['value'], d['kernels_ms'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r06i_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config mixed40 --frame --no-cpu-baseline --steps 5 > /tmp/r06i_prof.log 2>&1 || { tail -20 /tmp/r06i_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
find /tmp/r06i_prof -name "*kernel_stats.csv" -exec cp {} $O/mixed_frame_kernel_stats.csv \;
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/r06i/mixed_frame_kernel_stats.csv")):
    print(r["Name"][:90], r["Calls"], r["AverageNs"])
PY
