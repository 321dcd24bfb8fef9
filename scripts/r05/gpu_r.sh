#!/bin/bash
# Round-5 step R: repeat the pageable fixed-width host encode that failed once in the
# closing suite (r05final_a) and describe any mismatch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05r}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python scripts/r05/dbg_pageable.py 30 8192 > $O/dbg_8192.log 2>&1
rc=$?; tail -12 $O/dbg_8192.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/r05/dbg_pageable.py 15 1024 > $O/dbg_1024.log 2>&1
rc=$?; tail -6 $O/dbg_1024.log; exit $rc
