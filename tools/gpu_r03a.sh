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
# FETCH_SIZE / WRITE_SIZE calibration per access width (tools/pmc_calib.hip), one pass per counter
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/calib_fetch -o run -- tools/pmc_calib > $O/calib_fetch.log 2>&1 || { tail -5 $O/calib_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/calib_write -o run -- tools/pmc_calib > $O/calib_write.log 2>&1 || { tail -5 $O/calib_write.log; exit 1; }
python tools/pmc_calib.py $O/calib_fetch $O/calib_write -o $O/pmc_calib.json
# GEMM v5 (staggered groups) vs v4 on the transformer shapes
timeout -k 10 180 python tools/kbench.py g5 > $O/kbench_g5.log 2>&1; rc=$?; grep -v amdgpu.ids $O/kbench_g5.log | tail -14; exit $rc
