#!/bin/bash
# Same-box A/B of two source trees: the current one and ab/<tag> (a git-archive
# copy with its own built library), C3 bench lines interleaved.
#   [EXTRA='--config C2'] bash scripts/ab_trees.sh <tag> [rounds]
set -u
cd "$(dirname "$0")/.."
tag=$1; n=${2:-2}
mkdir -p gpurun_out
for r in $(seq 1 "$n"); do
  for t in cur "$tag"; do
    d=.; [ "$t" = cur ] || d=ab/$t
    timeout -k 10 200 python -u $d/bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-frames 0 ${EXTRA:-} > gpurun_out/ab_${t}_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$t round $r rc=$rc"; tail -5 gpurun_out/ab_${t}_$r.log; exit $rc; }
    grep '^{' gpurun_out/ab_${t}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown_ms']; print('$t', $r, d['value'], 'us/it', d.get('fastba_us_per_iteration'), 'corr', d['roofline']['avg_launch_ms'], 'upd', b['update_op'], 'ba', b['fastba'])"
  done
done
