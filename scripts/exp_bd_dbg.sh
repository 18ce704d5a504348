# fastba patch-kernel timing split (DPVO_BD_DBG variants; results invalid except 0)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for cfg in C3 C2; do for d in 0 1 2 3 7; do
  DPVO_BD_DBG=$d timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --e2e-frames 0 > gpurun_out/bdd.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/bdd.json')); print('$cfg dbg $d', d['ms_per_step'], d.get('fastba_us_per_iteration'))"
done; done
