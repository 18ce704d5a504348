#!/bin/bash
# C2 / C3: eager launches vs update() replayed from a HIP graph
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in C2 C3; do
  for g in "" "--graph"; do
    timeout -k 10 300 python bench.py --config $cfg --steps 30 --warmup 5 --e2e-frames 0 --no-cpu-baseline $g > gpurun_out/b_$cfg$g.json 2> gpurun_out/b_$cfg$g.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/b_$cfg$g.json'));print('$cfg','$g',d['value'],d['ms_per_step'])"
  done
done
