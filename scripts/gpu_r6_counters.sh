#!/bin/bash
# Round-6 counter record: FETCH_SIZE / WRITE_SIZE / TA_BUSY passes over the C3
# bench (altcorr + update-operator kernels) -> profiles/counters_c3.json.
set -u
cd "$(dirname "$0")/.."
KREGEX='corr_mfma_kernel|edge_hist_kernel|edge_scatter_kernel|rowgemm|rowchain|rowadd_ln|sa_reduce_csr|nb_csr' \
PASSES='FETCH_SIZE;WRITE_SIZE;TA_BUSY_avr GRBM_GUI_ACTIVE' TAG=${1:-r6} bash scripts/gpu_pmc.sh || exit $?
python scripts/counters_json.py gpurun_out/pmc_${1:-r6} 95424 gpurun_out/counters_c3_${1:-r6}.json
