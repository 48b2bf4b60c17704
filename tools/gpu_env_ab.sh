#!/bin/bash
# Whole-model A/B of an environment switch in one GPU run (alternating bench.py runs without extras).
# Usage: tools/gpu_env_ab.sh "VAR=VALUE" [rounds]   (A = the switch set, B = default)
E=$1; N=${2:-2}
for i in $(seq $N); do
  for arm in A B; do
    if [ $arm = A ]; then ENV="$E"; else ENV=""; fi
    env $ENV timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 3 > gpurun_out/envab.log 2>&1 || { tail -5 gpurun_out/envab.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/envab.log').read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" "$arm:${ENV:-default}"
  done
done
