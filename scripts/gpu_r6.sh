#!/bin/bash
# Round-6 GPU record: tests (TESTS= pytest targets, default the whole -m gpu
# suite), C3 / C2 bench lines, kernel trace of the C3 bench.  SKIP_TESTS=1,
# SKIP_BENCH=1, SKIP_PROF=1 drop steps.  Stops at the first step that ends in
# a fault, abort, kill or timeout.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
tag=${1:-r6}
step() {   # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/${tag}_${name}.log" 2>&1
  local rc=$?
  tail -4 "gpurun_out/${tag}_${name}.log"
  case $rc in 0|1|5) return 0 ;; *) echo "step $name rc=$rc: stopping"; exit $rc ;; esac
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step tests 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  step bench_c3 600 python -u bench.py --steps 20 --warmup 5
  step bench_c2 600 python -u bench.py --config C2 --steps 20 --warmup 5 --no-cpu-baseline --e2e-frames 0
fi
if [ "${SKIP_PROF:-0}" != 1 ]; then
  export TMPDIR=/tmp
  step prof_c3 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --e2e-frames 0
fi
echo done
