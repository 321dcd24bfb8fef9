#!/bin/bash
# Profiles for both fixed-width kernel variants (pipelined = default, one-tile = FORY_ROWFMT_PIPE=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export EXTRA_PMC="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_LDS,SQ_WAIT_INST_LDS TA_BUSY_avr,TA_TA_BUSY_sum,TCP_TCC_READ_REQ_sum,TCP_TCC_WRITE_REQ_sum"
OUT=gpurun_out/prof_pipe1 bash scripts/profile.sh || exit $?
FORY_ROWFMT_PIPE=0 OUT=gpurun_out/prof_pipe0 EXTRA_PMC="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_BUSY_CYCLES" bash scripts/profile.sh
