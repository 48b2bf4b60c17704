#!/bin/bash
# residual L2 prefetch in gemm5: kbench residual GEMMs, then parity + bench sites
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/kbench.py res > $O/kbench_res.log 2>&1 || { tail -5 $O/kbench_res.log; exit 1; }
grep -v amdgpu.ids $O/kbench_res.log | cut -c1-200
bash tools/gpu_sites_check.sh rpf
