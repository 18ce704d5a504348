#!/bin/bash
# GEMM1 deep prefetch (DPVO_RC_DBG=2048): bit-identity, then c1-chain timing A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
timeout -k 10 120 python scripts/check_rc_dbg_equal.py || exit 1
export TMPDIR=/tmp
cd /tmp
RC_VARIANTS=0,2048,1,2049,0,2048 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$REPO/gpurun_out/deep_ab" -o run -- python "$REPO/scripts/bench_rc_dbg.py" > "$REPO/gpurun_out/deep_ab.log" 2>&1 || exit 1
cd "$REPO"
python scripts/kstats.py gpurun_out/deep_ab 6
