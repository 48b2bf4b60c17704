#!/bin/bash
# A/B of the round-3 forward changes (temporary env toggles) + residual-ring kbench (depth 3 vs 1)
O=gpurun_out
mkdir -p $O
run() { env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 2 > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }; echo "$* $(python -c "import json; d=json.loads(open('$O/ab.log').read().strip().splitlines()[-1]); print(d['value'])")"; }
for i in 1 2; do
  run X=all
  run ATHD_X_NOMOVE=1
  run ATHD_X_NODSGN=1
  run ATHD_X_NOMOVE=1 ATHD_X_NODSGN=1
done
timeout -k 10 300 python tools/kbench.py res > $O/kb_rd3.log 2>&1; grep -v amdgpu.ids $O/kb_rd3.log | cut -c1-130
KB_LIB=libkbench_v.so timeout -k 10 300 python tools/kbench.py res > $O/kb_rd1.log 2>&1; grep -v amdgpu.ids $O/kb_rd1.log | cut -c1-130
