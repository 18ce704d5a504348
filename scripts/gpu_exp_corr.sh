#!/bin/bash
# A/B of altcorr experiment builds (scripts/build_exp.sh) at C3, interleaved twice.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/${TAG:-exp_corr}.log
: > "$out"
for r in 1 2; do
  for lib in product ${LIBS:-l2exp1 l2exp2 l2exp3}; do
    if [ "$lib" = product ]; then
      timeout -k 10 300 python -u scripts/exp_corr_time.py --tag product >> "$out" 2>&1 || exit $?
    else
      DPVO_DIAG=1 DPVO_HOT_LIB=exp/$lib/libdpvo_hot.so timeout -k 10 300 python -u scripts/exp_corr_time.py --tag $lib >> "$out" 2>&1 || exit $?
    fi
    tail -1 "$out"
  done
done
