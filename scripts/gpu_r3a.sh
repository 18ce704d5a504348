#!/bin/bash
# round 3, first box: new reference-module fixture tests, counter list, PMC
# passes on the update-operator GEMMs and altcorr.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_net_fixtures.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/fixtures.log 2>&1
rc=$?; echo "fixtures rc=$rc"; grep -E "passed|failed|rms|Error" gpurun_out/fixtures.log | tail -30
[ $rc -le 1 ] || exit $rc
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 rocprofv3 -L > "$REPO/gpurun_out/counters_list.txt" 2>&1; echo "list rc=$?"
cd "$REPO"
KREGEX='rowgemm3|rowchain|corr_mfma|rowadd_ln' PASSES='FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT;SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE TA_BUSY_avr TA_BUSY_max;TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT' TAG=r3a bash scripts/gpu_pmc.sh
