#!/bin/bash
# kernel micro-bench then parity/bench/profile
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/kbench.py attn > gpurun_out/kbench.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/kbench.log | tail -12
if [ $rc -ne 0 ]; then exit $rc; fi
exec_rc=0
bash ./tools/gpu_job1.sh
