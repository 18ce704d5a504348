#!/bin/bash
# ping-pong chain k-loops (rowchain_kernel, PP) -- the chain / operator tests, the c1
# chain A/B (DPVO_RC_DBG 0 = ping-pong, 512 = the waves in step), the C3
# bench and its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rowgemm.py tests/test_gpu_net_fixtures.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_pp.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_pp.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/t_pp.log | head -30; exit $rc; }
export TMPDIR=/tmp
cd /tmp
RC_VARIANTS=0,512,1,513,0,512 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$REPO/gpurun_out/pp_ab" -o run -- python "$REPO/scripts/bench_rc_dbg.py" > "$REPO/gpurun_out/pp_ab.log" 2>&1 || exit 1
cd "$REPO"
python scripts/kstats.py gpurun_out/pp_ab 5
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --e2e-frames 0 > gpurun_out/b_pp.json 2> gpurun_out/b_pp.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/b_pp.json'));print(d['value'],d['ms_per_step'],d['breakdown_ms'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$REPO/gpurun_out/trace_pp" -o run -- python "$REPO/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --e2e-frames 0 > "$REPO/gpurun_out/trace_pp.log" 2>&1 || exit 1
cd "$REPO"
python scripts/kstats.py gpurun_out/trace_pp 12
