#!/bin/bash
# Staged GPU test pass: each -k group in its own pytest run, stopping at the
# first failure of any kind (a fault must not be followed by more GPU work).
#   STAGES="corr_mfma|rowgemm|updateop" bash scripts/gpu_stage.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS='|' read -ra ST <<< "${STAGES:?}"
n=0
for k in "${ST[@]}"; do
  n=$((n + 1))
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "$k" \
      > "gpurun_out/stage_$n.log" 2>&1
  rc=$?
  echo "stage $n [$k] rc=$rc"; grep -E "passed|failed|rror" "gpurun_out/stage_$n.log" | tail -6
  [ $rc -eq 0 ] || exit $rc
done
