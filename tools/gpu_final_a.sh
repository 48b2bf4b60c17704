#!/bin/bash
# Round-end GPU pass, part A: the full GPU test suite, smoke(), the default bench (driver protocol: --steps 20
# --warmup 5, CPU baseline included) and the per-call-site kernel profile.  $1 = tag
TAG=${1:-r05}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
set -o pipefail
echo "== pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
grep -E "passed|failed" $O/pytest_gpu.log | tail -1
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.txt 2>&1 || { tail -20 $O/smoke_$TAG.txt; exit 1; }
grep smoke $O/smoke_$TAG.txt
echo "== bench"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_full.log 2>&1 || { tail -20 $O/bench_full.log; exit 1; }
tail -1 $O/bench_full.log | cut -c1-300
echo "== sites"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --dump-kernels $O/kernels_$TAG.json > $O/bench_kernels_$TAG.log 2>&1 || { tail -20 $O/bench_kernels_$TAG.log; exit 1; }
tail -1 $O/bench_kernels_$TAG.log | cut -c1-200
