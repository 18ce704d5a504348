#!/bin/bash
# quick iteration: the given GPU test files, then a short C3 (and C2) bench
# and a kernel-trace profile of the C3 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
TAG=${TAG:-q}
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests_$TAG.log
  [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/tests_$TAG.log | head -20; exit $rc; }
fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --e2e-frames 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print(d['value'],d['ms_per_step'],d['breakdown_ms'])"
[ $rc -eq 0 ] || exit $rc
if [ "${C2:-0}" = "1" ]; then
  timeout -k 10 300 python bench.py --config C2 --steps 30 --warmup 5 --no-cpu-baseline --e2e-frames 0 > gpurun_out/bench_${TAG}_c2.json 2> gpurun_out/bench_${TAG}_c2.err
  python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_c2.json'));print('C2',d['value'],d['ms_per_step'],d['breakdown_ms'])"
fi
if [ "${TRACE:-1}" = "1" ]; then
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$REPO/gpurun_out/trace_$TAG" -o run -- python "$REPO/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --e2e-frames 0 > "$REPO/gpurun_out/trace_$TAG.log" 2>&1
  echo "trace rc=$?"
  cd "$REPO"
  python scripts/kstats.py gpurun_out/trace_$TAG 25
fi
