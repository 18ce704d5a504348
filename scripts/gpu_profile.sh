#!/bin/bash
# rocprofv3 kernel-trace/stats of a short bench run, then two PMC passes
# (FETCH_SIZE, WRITE_SIZE -- separate passes, gfx950 slot limits) on the
# fused altcorr kernel.  Outputs under gpurun_out/prof_<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
TAG=${TAG:-r1}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${PROF_ARGS:---steps 10 --warmup 2 --no-cpu-baseline}
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python "$REPO/bench.py" $ARGS > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; tail -3 "$OUT/trace.log"
[ $rc -eq 0 ] || exit $rc
[ "${PMC:-1}" = "1" ] || exit 0
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "${KREGEX:-corr_mfma}" -f csv -d "$OUT/pmc_$C" -o run -- python "$REPO/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --e2e-frames 0 > "$OUT/pmc_$C.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc"; tail -2 "$OUT/pmc_$C.log"
  [ $rc -eq 0 ] || exit $rc
done
cd "$REPO"
python scripts/traffic_json.py "$OUT/pmc_FETCH_SIZE" "$OUT/pmc_WRITE_SIZE" 95424 "$OUT/altcorr_traffic.json"
