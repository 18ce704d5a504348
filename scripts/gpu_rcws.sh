#!/bin/bash
# rowchain_ws (warp-specialised 64-row chains, DPVO_RCWS=1) vs the 128-row
# chain kernel: the chain tests with both, the C3 bench with each, a kernel
# trace, and the DPVO_RCWS_DBG timing variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
DPVO_RCWS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_rowgemm.py tests/test_gpu_net_fixtures.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_rcws.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_rcws.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/t_rcws.log | head -30; exit $rc; }
for v in 1 0 1; do
  DPVO_RCWS=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --e2e-frames 0 > gpurun_out/b_rcws_$v.json 2> gpurun_out/b_rcws_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b_rcws_$v.json'));print('RCWS=$v',d['value'],d['ms_per_step'],d['breakdown_ms'])"
done
export TMPDIR=/tmp
cd /tmp
DPVO_RCWS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$REPO/gpurun_out/trace_rcws" -o run -- python "$REPO/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --e2e-frames 0 > "$REPO/gpurun_out/trace_rcws.log" 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$REPO/gpurun_out/rcws_dbg" -o run -- python "$REPO/scripts/bench_rcws_dbg.py" > "$REPO/gpurun_out/rcws_dbg.log" 2>&1 || exit 1
cd "$REPO"
python scripts/kstats.py gpurun_out/trace_rcws 12
python scripts/kstats.py gpurun_out/rcws_dbg 7
