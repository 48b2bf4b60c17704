#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python tools/kbench.py "$@" > gpurun_out/kbench.log 2>&1
rc=$?; cat gpurun_out/kbench.log | grep -v amdgpu.ids; exit $rc
