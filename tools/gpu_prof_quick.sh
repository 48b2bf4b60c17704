#!/bin/bash
# bench line (no CPU baseline / extras) + serial-branch kernel trace summary
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > $O/bench_q.log 2>&1 || { tail -20 $O/bench_q.log; exit 1; }
tail -1 $O/bench_q.log | cut -c1-300
ATHD_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_q -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $O/prof_q.log 2>&1 || { tail -20 $O/prof_q.log; exit 1; }
python tools/prof_summary.py $O/prof_q > $O/prof_q_summary.txt 2>&1; head -${1:-30} $O/prof_q_summary.txt
