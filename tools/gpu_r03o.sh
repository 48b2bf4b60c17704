#!/bin/bash
# Round 3: attention row sums on the MFMA (ones block) - bf16 parity + chunk tests, then A/B against HEAD.
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_r03o.log 2>&1
rc=$?; tail -3 $O/pytest_r03o.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_lib.sh abtmp/libA.so abtmp/libB.so 3
