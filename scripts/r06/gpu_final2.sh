#!/bin/bash
# Round 6: the whole GPU suite and smoke on the final library (after the small-kernel and
# host drain changes), then quick Nested A/B of two existing launch knobs (waves per tile,
# XCD tile runs) against the defaults, two alternating rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06final2
mkdir -p $O
export PYTHONUNBUFFERED=1
bash scripts/r06/gpu_box.sh || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
sha256sum fury_amd/lib/libfory_rowfmt.so | cut -c1-16 > $O/lib_sha16.txt
for r in 1 2; do
  for knobs in "" "FORY_ROWFMT_VARNW=4" "FORY_ROWFMT_VARXCD=-1" "FORY_ROWFMT_VARXCD=8"; do
    tag=$(echo "default $knobs" | tr ' =' '__')
    env $knobs timeout -k 10 300 python -u bench.py --config nested --no-cpu-baseline > $O/nested_${tag}_$r.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('$O/nested_${tag}_$r.json'));k=d['kernels_ms'];print('nested $knobs r$r', d['value'], k['encode_call_avg'], k['decode_call_avg'])"
  done
done
