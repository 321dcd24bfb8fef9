#!/bin/bash
# Round 3: the overlap probe (Mixed / Nested), then the columnar-engine check (gpu_r03_f.sh).
set -o pipefail
bash scripts/gpu_r03_e.sh || exit $?
bash scripts/gpu_r03_f.sh
