#!/bin/bash
# Round-3 final record: the tracker tests touched last, the PMC counter
# record + C3 bench line + kernel trace (gpu_r3_measure.sh), the C2 line, and
# the end-to-end wall vs GPU-busy time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tracker.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_final.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_final.log; [ $rc -eq 0 ] || exit $rc
TAG=r3final timeout -k 10 900 bash scripts/gpu_r3_measure.sh || exit 1
timeout -k 10 400 python bench.py --config C2 --e2e-frames 0 > gpurun_out/bench_r3final_c2.json 2> gpurun_out/bench_r3final_c2.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_r3final_c2.json'));print('C2',d['value'],d['ms_per_step'],d['breakdown_ms'],d.get('fastba_us_per_iteration'))"
timeout -k 10 600 bash scripts/gpu_e2e_time.sh || exit 1
