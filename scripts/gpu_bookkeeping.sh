#!/bin/bash
# tracker bookkeeping kernels: parity tests, C3 bench line (with end-to-end), e2e GPU-time traces
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_encoder.py tests/test_gpu_tracker.py > gpurun_out/t_bk.log 2>&1 || { tail -30 gpurun_out/t_bk.log; exit 1; }
tail -3 gpurun_out/t_bk.log
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_bk.json 2> gpurun_out/bench_bk.err || { tail -20 gpurun_out/bench_bk.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_bk.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], json.dumps(d.get('end_to_end')))"
bash scripts/gpu_e2e_time.sh
