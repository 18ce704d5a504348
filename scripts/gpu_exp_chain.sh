#!/bin/bash
# A/B of update-operator experiment builds (scripts/build_exp.sh) at C3's
# shape: the GEMM tests and the whole-update pins on each build, then timings
# interleaved twice (TIMER= the timing script: exp_chain_time.py, c1 / c2's
# chain, or exp_pair_time.py, SoftAgg's GEMM pairs).  LIBS= the exp/<name>
# builds, TESTS=0 skips tests.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/${TAG:-exp_chain}.log
: > "$out"
if [ "${TESTS:-1}" = 1 ]; then
  for lib in ${LIBS:-c64}; do
    DPVO_DIAG=1 DPVO_HOT_LIB=exp/$lib/libdpvo_hot.so timeout -k 10 600 python -u -m pytest -x -q -m gpu \
      --timeout 300 --timeout-method thread -p no:cacheprovider \
      tests/test_gpu_rowgemm.py tests/test_gpu_update_step.py tests/test_gpu_update_async.py \
      > gpurun_out/${TAG:-exp_chain}_tests_$lib.log 2>&1 || { echo "tests $lib rc=$?"; tail -20 gpurun_out/${TAG:-exp_chain}_tests_$lib.log; exit 1; }
    tail -1 gpurun_out/${TAG:-exp_chain}_tests_$lib.log
  done
fi
for r in 1 2; do
  for lib in product ${LIBS:-c64}; do
    if [ "$lib" = product ]; then
      timeout -k 10 300 python -u scripts/${TIMER:-exp_chain_time.py} --tag product >> "$out" 2>&1 || exit $?
    else
      DPVO_DIAG=1 DPVO_HOT_LIB=exp/$lib/libdpvo_hot.so timeout -k 10 300 python -u scripts/${TIMER:-exp_chain_time.py} --tag $lib >> "$out" 2>&1 || exit $?
    fi
    tail -1 "$out"
  done
done
