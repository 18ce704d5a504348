#!/bin/bash
# PMC counter record (FETCH / WRITE / TA busy) of altcorr + the update
# operator, reduced to profiles/counters_c3.json (copied to gpurun_out/), then
# the C3 bench line (which reads it) and a kernel-trace profile of the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
TAG=${TAG:-r3}
mkdir -p gpurun_out
if [ "${SKIP_PMC:-0}" != "1" ]; then
  KREGEX='corr_mfma|edge_hist|edge_scatter|rowgemm|rowchain|rowadd_ln|sa_reduce|nb_csr' \
  PASSES='FETCH_SIZE;WRITE_SIZE;TA_BUSY_avr GRBM_GUI_ACTIVE' TAG=$TAG bash scripts/gpu_pmc.sh > gpurun_out/pmc_$TAG.log 2>&1
  rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_$TAG.log; exit $rc; }
  python scripts/counters_json.py gpurun_out/pmc_$TAG 95424 profiles/counters_c3.json > gpurun_out/counters_$TAG.log 2>&1 || exit 1
  cp profiles/counters_c3.json gpurun_out/counters_c3.json
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$TAG.err; exit $rc; }
if [ "${TRACE:-1}" = "1" ]; then
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$REPO/gpurun_out/trace_$TAG" -o run -- python "$REPO/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --e2e-frames 0 > "$REPO/gpurun_out/trace_$TAG.log" 2>&1
  rc=$?; echo "trace rc=$rc"
fi
exit 0
