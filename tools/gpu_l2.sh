#!/bin/bash
# L2 hit rate per kernel over a 1-step bench (one PMC pass: TCC_HIT_sum, TCC_MISS_sum).  $1 = tag
O=gpurun_out/l2_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > $O/p.log 2>&1 || { tail -5 $O/p.log; exit 1; }
python tools/pmc_l2.py $O/p --top 40 > $O/l2.txt 2>&1; cat $O/l2.txt
