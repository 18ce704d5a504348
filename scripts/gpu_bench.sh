#!/bin/bash
# bench.py on the GPU box; output line -> gpurun_out/bench.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json
exit $rc
