#!/bin/bash
# residual-epilogue GEMM kbench (gemm5 vs gemm3 tiles) + per-call-site kernel times, previous commit vs this tree
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/kbench.py res > $O/kb_res.log 2>&1 || { tail -5 $O/kb_res.log; exit 1; }
grep RES $O/kb_res.log | cut -c1-400
for i in 1 2; do
  for L in prev cur; do
    [ $L = prev ] && LIB=ablibs/libathd_prev.so || LIB=audio-to-sheet-music_amd/athd/libathd.so
    ATHD_LIB=$(realpath $LIB) timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 5 --warmup 2 --dump-kernels $O/k_${L}_$i.json > $O/b_${L}_$i.log 2>&1 || { tail -5 $O/b_${L}_$i.log; exit 1; }
  done
done
python tools/sites_diff.py $O/k_prev_1_sites.json $O/k_cur_1_sites.json --top 12
python tools/sites_diff.py $O/k_prev_2_sites.json $O/k_cur_2_sites.json --top 12
