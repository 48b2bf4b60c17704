#!/bin/bash
# Round 3: GPU tests, then a bench line (with the dataset pass of configs[3] at one rank's size)
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
rm -f $O/parity_report.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rA -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_r03a.log 2>&1
rc=$?; grep -E "passed|failed|Error" $O/pytest_r03a.log | tail -8
if [ $rc -ne 0 ]; then tail -60 $O/pytest_r03a.log; exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu-baseline --segments 750 > $O/bench_r03a.log 2>&1 || { tail -20 $O/bench_r03a.log; exit 1; }
tail -2 $O/bench_r03a.log | cut -c1-600
