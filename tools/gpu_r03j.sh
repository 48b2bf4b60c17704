#!/bin/bash
# HIP-graph replay vs eager launches: the graph parity test, then the bench both ways (alternating)
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "graph or bench_batch" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_r03j.log 2>&1
rc=$?; tail -3 $O/pytest_r03j.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest_r03j.log | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 2 > $O/bg_$i.log 2>&1 || { tail -5 $O/bg_$i.log; exit 1; }
  tail -1 $O/bg_$i.log | cut -c1-110
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 2 --eager > $O/be_$i.log 2>&1 || { tail -5 $O/be_$i.log; exit 1; }
  tail -1 $O/be_$i.log | cut -c1-110
done
