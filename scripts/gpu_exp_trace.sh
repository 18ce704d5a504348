#!/bin/bash
# Kernel-trace A/B of experiment builds (scripts/build_exp.sh): TIMER= a
# scripts/exp_*_time.py driver, LIBS= the exp/<name> builds (plus the product),
# PAT= the kernel-name filter of the summary.  One rocprofv3 --kernel-trace per
# build; summaries in gpurun_out/${TAG}_<lib>.txt.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in product ${LIBS}; do
  if [ "$lib" = product ]; then unset DPVO_HOT_LIB DPVO_DIAG; else export DPVO_HOT_LIB=exp/$lib/libdpvo_hot.so DPVO_DIAG=1; fi
  rm -rf gpurun_out/prof_${TAG}_$lib
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_${TAG}_$lib -o run -- python3 scripts/${TIMER} --tag $lib \
    > gpurun_out/${TAG}_$lib.log 2>&1 || exit $?
  python3 scripts/kstats_db.py gpurun_out/prof_${TAG}_$lib "${PAT:-}" > gpurun_out/${TAG}_$lib.txt
  rm -rf gpurun_out/prof_${TAG}_$lib   # (the traces would exceed the copy-back cap)
  grep '^{' gpurun_out/${TAG}_$lib.log | tail -1
  cat gpurun_out/${TAG}_$lib.txt
done
