#!/bin/bash
# bench.py on the GPU box; output line -> gpurun_out/${OUT:-bench}.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=${OUT:-bench}
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/$O.json 2> gpurun_out/$O.err
rc=$?; echo "bench $O rc=$rc"; tail -5 gpurun_out/$O.err; cat gpurun_out/$O.json
exit $rc
