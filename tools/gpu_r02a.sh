#!/bin/bash
# Round-2 check: the full -m gpu suite, then the default bench line.
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu.log | tail -3
if [ $rc -gt 1 ]; then tail -30 $O/pytest_gpu.log; exit $rc; fi
timeout -k 10 400 python bench.py > $O/bench_full.log 2>&1 || { tail -20 $O/bench_full.log; exit 1; }
tail -1 $O/bench_full.log
