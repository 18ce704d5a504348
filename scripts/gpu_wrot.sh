#!/bin/bash
# W-stage k-order rotation timing experiment (DPVO_RC_DBG 1024 / 1025, wrong
# results): does the chain k-loop speed up when the CUs of an XCD stop
# requesting the same W block from L2 at the same time?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
RC_VARIANTS=0,1024,1,1025,0,1024 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$REPO/gpurun_out/wrot_ab" -o run -- python "$REPO/scripts/bench_rc_dbg.py" > "$REPO/gpurun_out/wrot_ab.log" 2>&1 || exit 1
cd "$REPO"
python scripts/kstats.py gpurun_out/wrot_ab 8
