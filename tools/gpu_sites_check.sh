#!/bin/bash
# GPU parity tests (all, or the -k expression in $2), then the bench with per-call-site kernel times -> gpurun_out/k_$1_sites.json
TAG=${1:-x}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread "${K[@]}" > $O/pytest_$TAG.log 2>&1
rc=$?; tail -3 $O/pytest_$TAG.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest_$TAG.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 2 --dump-kernels $O/k_$TAG.json > $O/b_$TAG.log 2>&1 || { tail -5 $O/b_$TAG.log; exit 1; }
tail -1 $O/b_$TAG.log | cut -c1-110
