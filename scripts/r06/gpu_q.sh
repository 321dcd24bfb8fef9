#!/bin/bash
# Round 6, call Q: the null-stream arena memset race (host.cpp context creation).
# 1. scripts/microbench/memset_race.hip: hipMemset (null stream) behind a busy null stream,
#    then an H2D on a non-blocking stream: are the copied bytes zeroed by the late fill?
# 2. tests/test_gpu_host.py::test_host_fresh_context_while_the_null_stream_is_busy (a ~1 s spin
#    on torch's default stream, the null stream) against the
#    library with the old hipMemset (fury_amd/lib/ab_oldmemset), expected to fail on wrong
#    bytes, no fault;
# 3. the same test and the whole host file against the fixed library.
set -o pipefail
O=gpurun_out/${1:-r06q}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 120 scripts/microbench/bin/memset_race 5 100000000 > $O/memset_race.jsonl 2>&1 || { cat $O/memset_race.jsonl; exit 1; }
cat $O/memset_race.jsonl
FORY_ROWFMT_LIB=$PWD/fury_amd/lib/ab_oldmemset/libfory_rowfmt.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_host.py -k "fresh_context" > $O/pytest_oldlib.log 2>&1
rc=$?
echo "old library: pytest exit $rc"; tail -3 $O/pytest_oldlib.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
grep -q -i "illegal\|aborted\|core dumped" $O/pytest_oldlib.log && { echo "fault on the old library: stop"; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_host.py > $O/pytest_host.log 2>&1 || { tail -30 $O/pytest_host.log; exit 1; }
tail -1 $O/pytest_host.log
