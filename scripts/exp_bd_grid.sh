cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for cfg in C3 C2; do for g in 256 512 768 1024 2048; do
  DPVO_BD_GRID=$g timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --e2e-frames 0 > gpurun_out/bd_$cfg_$g.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/bd_$cfg_$g.json')); print('$cfg', $g, d['ms_per_step'], d.get('fastba_us_per_iteration'), d['breakdown_ms']['fastba'])"
done; done
