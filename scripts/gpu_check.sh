#!/bin/bash
# One GPU-box pass: GPU parity tests, then smoke.  Stops at the first
# abnormal exit (signal / timeout); ordinary test failures (exit 1) are logged
# and the next step still runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
KARGS=()
[ -n "${PYTEST_K:-}" ] && KARGS=(-k "$PYTEST_K")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "${KARGS[@]}" \
    ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; grep -E "passed|failed|error|drift" gpurun_out/gpu_tests.log | tail -20
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
exit $rc
