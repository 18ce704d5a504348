#!/bin/bash
# timing experiment: corr_mfma with full-line tile loads (wrong results) vs the
# real kernel, kernel-trace of a short C3 bench each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
export TMPDIR=/tmp
for V in real fullline; do
  cd /tmp
  if [ $V = fullline ]; then export DPVO_CM_DBG=fullline; else unset DPVO_CM_DBG; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$REPO/gpurun_out/cm_$V" -o run -- python "$REPO/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --e2e-frames 0 > "$REPO/gpurun_out/cm_$V.log" 2>&1
  echo "$V rc=$?"
  cd "$REPO"
  python scripts/kstats.py gpurun_out/cm_$V 3
done
