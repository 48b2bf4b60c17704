#!/bin/bash
# attention A/B micro-bench + the parity tests that exercise the transformer
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/kbench.py attn > gpurun_out/kbench_attn.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/kbench_attn.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -rA -p no:cacheprovider --timeout 200 --timeout-method thread -k "sharp or golden or 6s or ragged" > gpurun_out/pytest_attn.log 2>&1
rc=$?; grep -E "passed|failed|Error" gpurun_out/pytest_attn.log | tail -5; exit $rc
