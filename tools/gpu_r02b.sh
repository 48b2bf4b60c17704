#!/bin/bash
# full -m gpu suite, default bench, rocprofv3 kernel trace (serial branches) of a short bench
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu.log | tail -3
if [ $rc -gt 1 ]; then tail -30 $O/pytest_gpu.log; exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_full.log 2>&1 || { tail -20 $O/bench_full.log; exit 1; }
tail -1 $O/bench_full.log | cut -c1-600
ATHD_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $O/prof_b.log 2>&1 || { tail -20 $O/prof_b.log; exit 1; }
python tools/prof_summary.py $O/prof_b > $O/prof_b_summary.txt 2>&1; head -30 $O/prof_b_summary.txt
