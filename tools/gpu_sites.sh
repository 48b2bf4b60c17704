#!/bin/bash
# per-call-site kernel profile of the bench config: gpurun_out/sites.json
mkdir -p gpurun_out
ATHD_PROF_SITES=1 timeout -k 10 600 python bench.py --steps 2 --warmup 2 --no-cpu-baseline --dump-kernels gpurun_out/sites.json > gpurun_out/bench_sites.log 2>&1
rc=$?; tail -1 gpurun_out/bench_sites.log; exit $rc
