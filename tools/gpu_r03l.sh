#!/bin/bash
# dual-output LayerNorm: parity + sites; then 1 vs 2 concurrent forward pipelines (alternating runs)
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_sites_check.sh ln2 || exit 1
for i in 1 2; do
  for P in 2 1; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 2 --pipelines $P > $O/bp${P}_$i.log 2>&1 || { tail -5 $O/bp${P}_$i.log; exit 1; }
    echo "pipelines=$P $(tail -1 $O/bp${P}_$i.log | cut -c80-200)"
  done
done
