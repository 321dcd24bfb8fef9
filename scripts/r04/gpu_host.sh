#!/bin/bash
# Host-inclusive rates through the C-ABI host path, registered and pageable
# (staged) host buffers: Struct104 8Mi (fixed, chunk pipeline) and Mixed / Nested 8Mi
# (varlen: pipelined encode, two-call and one-call decode). Never bench `value`.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04host
mkdir -p $O
export PYTHONUNBUFFERED=1
for mem in registered pageable; do
  HOST_MEM=$mem timeout -k 10 300 python scripts/host_native.py 8388608 1048576 > $O/host_fixed_$mem.json 2> $O/host_fixed_$mem.err
  rc=$?; echo "fixed $mem exit $rc"; cat $O/host_fixed_$mem.json; [ $rc -eq 0 ] || exit $rc
  HOST_MEM=$mem timeout -k 10 400 python scripts/host_native_var.py 8388608 > $O/host_var_$mem.json 2> $O/host_var_$mem.err
  rc=$?; echo "var $mem exit $rc"; cat $O/host_var_$mem.json; [ $rc -eq 0 ] || exit $rc
done
