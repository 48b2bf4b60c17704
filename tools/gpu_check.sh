#!/bin/bash
# Quick GPU check: parity tests, then the default bench line (with CPU baseline and extras).  Usage: tools/gpu_check.sh
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu.log | tail -2
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit $rc; fi
cp $O/parity_report.json $O/parity_report_check.json 2>/dev/null
timeout -k 10 600 python bench.py ${BENCH_ARGS} > $O/bench_full.log 2>&1 || { tail -20 $O/bench_full.log; exit 1; }
tail -1 $O/bench_full.log
