#!/bin/bash
# the PMC counter record + C3 bench line + kernel trace, the C2 line, end-to-end vs GPU-busy time
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r3close timeout -k 10 700 bash scripts/gpu_r3_measure.sh || exit 1
timeout -k 10 300 python bench.py --config C2 --e2e-frames 0 > gpurun_out/bench_r3close_c2.json 2> gpurun_out/bench_r3close_c2.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_r3close_c2.json'));print('C2',d['value'],d['ms_per_step'],d['breakdown_ms'],d.get('fastba_us_per_iteration'))"
timeout -k 10 400 bash scripts/gpu_e2e_time.sh || exit 1
