#!/bin/bash
# Round 6, call G: after the traced suite's fault in the varlen call-scoped registration test
# (registration moved to the calling thread, verify read-back through pinned memory): the
# whole GPU suite untraced, smoke, then the host-inclusive pageable rates again.
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
HOST_MEM=pageable timeout -k 10 300 python -u scripts/host_native.py > $O/host_fixed_pageable.json || exit $?
HOST_MEM=pageable timeout -k 10 300 python -u scripts/host_native_var.py > $O/host_var_pageable.json || exit $?
cat $O/host_*.json
