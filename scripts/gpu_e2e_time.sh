#!/bin/bash
# e2e wall time vs per-frame GPU busy time (kernel trace), deferred and immediate keyframes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in 1 0; do
  cd /tmp
  DEFER=$d timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$REPO/gpurun_out/e2e_tr_$d" -o run -- python "$REPO/scripts/e2e_gpu_time.py" run > "$REPO/gpurun_out/e2e_tr_$d.json" 2> "$REPO/gpurun_out/e2e_tr_$d.err" || exit 1
  cd "$REPO"
  python scripts/e2e_gpu_time.py report "$(ls gpurun_out/e2e_tr_$d/*kernel_trace.csv | head -1)" 32 <(tail -1 gpurun_out/e2e_tr_$d.json) | tee gpurun_out/e2e_time_$d.json
done
