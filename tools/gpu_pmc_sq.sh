#!/bin/bash
# One PMC pass of SQ counters over a 1-step bench (per-kernel rows in gpurun_out/pmc_sq_<tag>/).
# Usage: tools/gpu_pmc_sq.sh <tag> "<counters>"
TAG=${1:-sq}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc $2 --output-format csv -d $O/pmc_sq_$TAG -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_sq_$TAG.log 2>&1
rc=$?; tail -3 $O/pmc_sq_$TAG.log; exit $rc
