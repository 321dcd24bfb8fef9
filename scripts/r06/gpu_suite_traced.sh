#!/bin/bash
# Round 6: the full GPU suite in one process under rocprofv3 kernel + memory-copy trace
# (no counters), so that an asynchronous fault names the last kernels / copies before it
# (ADVICE r5); then smoke(). The traces stay on the box (/tmp); their
# summaries and, on a failure, their last records come back.
set -o pipefail
O=gpurun_out/r06_suite
T=/tmp/r06trace
mkdir -p $O $T
export TMPDIR=/tmp PYTHONUNBUFFERED=1
# (first, on the same box: the Struct104 encode's write-side A/B)
hostname > $O/host.txt
timeout -k 10 240 scripts/microbench/bin/enc_ab 67108864 2 > $O/enc_ab.jsonl 2>&1 || exit $?
timeout -k 10 1000 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $T -o suite --output-format csv -- \
  python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_shard.py::test_two_rank_device_shards_concatenate_to_the_whole_batch > $O/pytest_gpu.log 2>&1
rc=$?
echo "suite exit $rc" >> $O/pytest_gpu.log
tail -3 $O/pytest_gpu.log
find $T -name "*stats*.csv" -exec cp {} $O/ \;
if [ $rc -ne 0 ]; then
  for f in $(find $T -name "*kernel_trace.csv" -o -name "*memory_copy_trace.csv"); do
    (head -1 $f; tail -200 $f) > $O/tail_$(basename $f)
  done
  exit $rc
fi
# the two-rank shard test outside the tracer (under it, one traced suite saw both spawned
# ranks segfault in __cxa_finalize after their work; alone under the tracer it passes)
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_shard.py > $O/pytest_shard.log 2>&1 || exit $?
tail -1 $O/pytest_shard.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
