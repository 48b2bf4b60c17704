#!/bin/bash
# gemm5 (persistent, early restage) vs gemm4: kernel bench, whole-model A/B, parity with gemm5 in the product
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python tools/kbench.py g5 > $O/kbench_g5b.log 2>&1 || { tail -20 $O/kbench_g5b.log; exit 1; }
grep -v amdgpu.ids $O/kbench_g5b.log
timeout -k 10 400 bash tools/gpu_ab_lib.sh audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_g5.so 2 || exit 1
ATHD_LIB=$(realpath ablibs/libathd_g5.so) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_r03c.log 2>&1
rc=$?; tail -3 $O/pytest_r03c.log; exit $rc
