#!/bin/bash
# fenc_row0 statistics on all lanes + multi-row LayerNorm: parity tests, then whole-model A/Bs:
# previous commit vs ln1 (statistics change only), ln1 vs ln4, ln2 vs ln4 (rows per wave of the LayerNorm)
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_r03f.log 2>&1
rc=$?; tail -3 $O/pytest_r03f.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest_r03f.log | head -20; exit $rc; }
timeout -k 10 400 bash tools/gpu_ab_lib.sh ablibs/libathd_prev.so ablibs/libathd_ln1.so 2 || exit 1
timeout -k 10 400 bash tools/gpu_ab_lib.sh ablibs/libathd_ln1.so ablibs/libathd_ln4.so 2 || exit 1
timeout -k 10 400 bash tools/gpu_ab_lib.sh ablibs/libathd_ln2.so ablibs/libathd_ln4.so 2 || exit 1
