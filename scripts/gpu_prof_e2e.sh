#!/bin/bash
# rocprofv3 kernel trace + stats of the end-to-end tracker benchmark -> gpurun_out/prof_e2e_$TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/prof_e2e_${TAG:-x}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- python "$REPO/scripts/bench_e2e.py" --frames 20 --warmup 4 > "$OUT/log.txt" 2>&1
rc=$?; echo "e2e trace rc=$rc"; tail -1 "$OUT/log.txt"
exit $rc
