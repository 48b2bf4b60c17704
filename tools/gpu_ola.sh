#!/bin/bash
# parity tests of the forward + quick bench/profile
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_par.log 2>&1 || { tail -30 $O/pytest_par.log; exit 1; }
tail -2 $O/pytest_par.log
bash tools/gpu_prof_quick.sh 40
