#!/bin/bash
# Round-5 step W: the prefetching decode values pass (lib_ab/pf1) sized for two workgroups
# per CU (data-fitted image without growth, 2 KiB staging slots: FORY_ROWFMT_VARFIT=1,
# FORY_ROWFMT_VARSTG=2048), against the closing library; VARDIAG prints the residency.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=$PWD/gpurun_out/${1:-r05w}
mkdir -p $O
export PYTHONUNBUFFERED=1
PF=$PWD/fury_amd/lib_ab/pf1/libfory_rowfmt.so
for r in 1 2; do
  for cfg in mixed40 nested; do
    for v in default pf1fit; do
      unset FORY_ROWFMT_LIB FORY_ROWFMT_VARFIT FORY_ROWFMT_VARSTG FORY_ROWFMT_VARDIAG
      if [ $v = pf1fit ]; then export FORY_ROWFMT_LIB=$PF FORY_ROWFMT_VARFIT=1 FORY_ROWFMT_VARSTG=2048; fi
      [ $r = 1 ] && export FORY_ROWFMT_VARDIAG=1
      timeout -k 10 200 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $O/${cfg}_${v}_$r.json 2> $O/${cfg}_${v}_$r.err
      rc=$?; echo "$cfg $v $r: $(python3 -c "import json; d=json.load(open('$O/${cfg}_${v}_$r.json')); k=d['kernels_ms']; print(d['value'], k['encode_call_avg'], k['decode_call_avg'], k['decode_avg'])")"; [ $rc -eq 0 ] || exit $rc
      [ $r = 1 ] && grep -m3 "decode tile kernel" $O/${cfg}_${v}_$r.err
    done
  done
done
exit 0
