#!/bin/bash
# Iteration loop on the GPU box: parity tests, bench (no CPU baseline), kernel-trace profile of the bench config.
# Usage: tools/gpu_quick.sh <tag> [pytest -k expr]
TAG=${1:-q}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rA -p no:cacheprovider --timeout 120 --timeout-method thread ${2:+-k "$2"} > $O/pytest_$TAG.log 2>&1
rc=$?; grep -E "passed|failed|Error" $O/pytest_$TAG.log | tail -8
if [ $rc -ne 0 ]; then tail -40 $O/pytest_$TAG.log; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$TAG.log 2>&1 || { tail -20 $O/bench_$TAG.log; exit 1; }
tail -1 $O/bench_$TAG.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_$TAG.log 2>&1 || { tail -20 $O/prof_$TAG.log; exit 1; }
python tools/prof_sections.py $O/prof_$TAG
