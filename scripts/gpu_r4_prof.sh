#!/bin/bash
# Kernel-trace profile of the C3 bench, then PMC passes on the update
# operator's chain kernels (LDS bank conflicts, wave-cycle split).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
TAG=${TAG:-r4}
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$REPO/gpurun_out/trace_$TAG" -o run -- python "$REPO/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --e2e-frames 0 > "$REPO/gpurun_out/trace_$TAG.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$REPO"
python scripts/kstats.py gpurun_out/trace_$TAG 30
if [ -n "${PASSES:-}" ]; then
  KREGEX="${KREGEX:-rowchain}" PASSES="$PASSES" TAG=$TAG bash scripts/gpu_pmc.sh
fi
