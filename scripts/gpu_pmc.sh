#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over a short bench run.
#   KREGEX='corr_sfast' PASSES='SQ_WAVES SQ_BUSY_CYCLES;SQ_INSTS_VALU' TAG=x bash scripts/gpu_pmc.sh
# Each pass holds <= 8 SQ counters (gfx950 slot limits); stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/pmc_${TAG:-x}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
IFS=';' read -ra GROUPS_ <<< "$PASSES"
for G in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex "${KREGEX}" -f csv -d "$OUT/p$i" -o run -- python "$REPO/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --e2e-frames 0 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($G) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done
cd "$REPO"
python scripts/pmc_summary.py "$OUT" > "$OUT/summary.txt"; cat "$OUT/summary.txt"
