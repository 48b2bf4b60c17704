#!/bin/bash
# fenc_row VALU folds (levels 0 and 1): parity tests, then per-call-site kernel times, previous commit vs this tree
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_r03h.log 2>&1
rc=$?; tail -3 $O/pytest_r03h.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest_r03h.log | head -20; exit $rc; }
for i in 1 2; do
  for L in prev cur; do
    [ $L = prev ] && LIB=ablibs/libathd_prev.so || LIB=audio-to-sheet-music_amd/athd/libathd.so
    ATHD_LIB=$(realpath $LIB) timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 5 --warmup 2 --dump-kernels $O/k_${L}_$i.json > $O/b_${L}_$i.log 2>&1 || { tail -5 $O/b_${L}_$i.log; exit 1; }
    tail -1 $O/b_${L}_$i.log | cut -c1-80
  done
done
python tools/sites_diff.py $O/k_prev_1_sites.json $O/k_cur_1_sites.json --top 8
python tools/sites_diff.py $O/k_prev_2_sites.json $O/k_cur_2_sites.json --top 8
