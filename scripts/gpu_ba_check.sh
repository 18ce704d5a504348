# fastba parity tests + C3 / C2 BA timing (bench lines under gpurun_out/)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fastba.py tests/test_gpu_configs.py tests/test_gpu_tracker.py tests/test_gpu_global_ba.py tests/test_gpu_update_async.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ba_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ba_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in C3 C2; do
  timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --e2e-frames 0 > gpurun_out/ba_$cfg.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ba_$cfg.json')); print('$cfg', d['value'], d['ms_per_step'], d.get('fastba_us_per_iteration'))"
done
