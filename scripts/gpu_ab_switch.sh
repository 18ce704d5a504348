#!/bin/bash
# Same-box A/B of a class-level switch of dpvo.net.Update (SWITCH=NAME, e.g.
# FUSE_GRU_RES): scripts/exp_update_time.py with NAME=1 and NAME=0, three
# rounds interleaved, then one kernel trace each (PAT= the summary filter).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/ab_${SWITCH}.log
: > "$out"
for r in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 300 python -u scripts/exp_update_time.py --set ${SWITCH}=$v >> "$out" 2>&1 || exit $?
    tail -1 "$out"
  done
done
for v in 1 0; do
  rm -rf gpurun_out/prof_sw_$v
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_sw_$v -o run -- python3 scripts/exp_update_time.py \
    --set ${SWITCH}=$v > gpurun_out/sw_$v.log 2>&1 || exit $?
  python3 scripts/kstats_db.py gpurun_out/prof_sw_$v "${PAT:-}" > gpurun_out/sw_${SWITCH}_$v.txt
  rm -rf gpurun_out/prof_sw_$v
  echo "$SWITCH=$v"; cat gpurun_out/sw_${SWITCH}_$v.txt
done
