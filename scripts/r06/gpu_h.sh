#!/bin/bash
# Round 6, call H: the coalesced frame-index write pass (frames tests, Mixed / Nested frame
# benches); the two-rank shard test with and without rocprofv3 (its spawned ranks crashed
# in __cxa_finalize under the traced suite); the encode A/B on this box.
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
hostname > $O/host.txt
timeout -k 10 240 scripts/microbench/bin/enc_ab 67108864 2 > $O/enc_ab.jsonl 2>&1 || exit $?
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_frames.py tests/test_gpu_windows.py > $O/pytest_frames.log 2>&1 || { tail -30 $O/pytest_frames.log; exit 1; }
tail -1 $O/pytest_frames.log
B="python3 -u bench.py --no-cpu-baseline --extras 0 --steps 10 --warmup 3"
timeout -k 10 300 $B --config mixed40 --frame > $O/mixed_frame.json 2>$O/mixed_frame.err || exit 1
timeout -k 10 300 $B --config nested --frame > $O/nested_frame.json 2>$O/nested_frame.err || exit 1
timeout -k 10 300 $T tests/test_gpu_shard.py > $O/pytest_shard.log 2>&1 || { tail -30 $O/pytest_shard.log; exit 1; }
tail -1 $O/pytest_shard.log
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/shardtrace -o shard --output-format csv -- $T tests/test_gpu_shard.py > $O/pytest_shard_rocprof.log 2>&1
echo "shard under rocprofv3 exit $?" >> $O/pytest_shard_rocprof.log
grep -a "passed\|failed\|SIGSEGV\|exit" $O/pytest_shard_rocprof.log | grep -v correlation | tail -4
for f in $O/*_frame.json; do echo "$f $(python3 -c "import json; d=json.load(open('$f')); print(d.get('value'), d.get('kernels_ms'))")"; done
