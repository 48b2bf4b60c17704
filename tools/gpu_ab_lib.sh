#!/bin/bash
# A/B two builds of libathd.so in one GPU run (alternating, bench.py without extras).  Usage: tools/gpu_ab_lib.sh A.so B.so [rounds]
A=$1; B=$2; N=${3:-2}
for i in $(seq $N); do
  for L in $A $B; do
    ATHD_LIB=$(realpath $L) timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 3 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $L
  done
done
