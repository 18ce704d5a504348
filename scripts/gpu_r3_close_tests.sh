#!/bin/bash
# every GPU test + smoke
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all2.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/t_all2.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/t_all2.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke2.log 2>&1 || { tail -20 gpurun_out/smoke2.log; exit 1; }
tail -1 gpurun_out/smoke2.log
