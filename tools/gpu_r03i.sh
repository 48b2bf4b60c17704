#!/bin/bash
# iSTFT balanced split: parity tests, bench with per-site kernel times; gemm5 A-prefetch kbench
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_r03i.log 2>&1
rc=$?; tail -3 $O/pytest_r03i.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest_r03i.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels $O/k_r03i.json > $O/b_r03i.log 2>&1 || { tail -5 $O/b_r03i.log; exit 1; }
tail -1 $O/b_r03i.log | cut -c1-120
python tools/sites_diff.py profiles/r03_sites.json $O/k_r03i_sites.json --top 12
timeout -k 10 600 python tools/kbench.py g5pf > $O/kbench_g5pf.log 2>&1; rc=$?; grep -v amdgpu.ids $O/kbench_g5pf.log; exit $rc
