#!/bin/bash
# first GPU round: parity tests, bench, rocprof kernel stats
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -rA -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then tail -30 gpurun_out/pytest_gpu.log; exit $rc; fi
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6 -o run -- python bench.py --steps 2 --warmup 1 --batch 16 --no-cpu-baseline > gpurun_out/prof1.log 2>&1
echo "rocprof rc=$?"
