#!/bin/bash
# Full GPU pass: parity tests, bench (with CPU baseline), kernel-trace profile at the bench config, HBM traffic from
# two PMC passes, and a final bench line carrying the measured traffic.  Usage: tools/gpu_round.sh <tag>
# (SKIP_PYTEST=1: no tests / default bench; SKIP_TRACE=1: no kernel traces - e.g. when tools/gpu_run.sh prof:<tag> ran)
TAG=${1:-r01}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1"; }
if [ -z "$SKIP_PYTEST" ]; then
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu.log | tail -2
if [ $rc -gt 1 ]; then tail -30 $O/pytest_gpu.log; exit $rc; fi
step bench
timeout -k 10 600 python bench.py > $O/bench_full.log 2>&1 || { tail -20 $O/bench_full.log; exit 1; }
tail -1 $O/bench_full.log
fi
if [ -z "$SKIP_TRACE" ]; then
step kernel-trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $O/prof_$TAG.log 2>&1 || { tail -20 $O/prof_$TAG.log; exit 1; }
tail -1 $O/prof_$TAG.log
python tools/timeline.py $O/prof_$TAG --last-steps 2 > $O/timeline_$TAG.txt 2>&1; cat $O/timeline_$TAG.txt
step kernel-trace-serial
ATHD_SERIAL=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${TAG}_serial -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $O/prof_${TAG}_serial.log 2>&1 || { tail -20 $O/prof_${TAG}_serial.log; exit 1; }
tail -1 $O/prof_${TAG}_serial.log | cut -c1-200
fi
step pmc-fetch
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$TAG -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > $O/pmc_fetch_$TAG.log 2>&1 || { tail -20 $O/pmc_fetch_$TAG.log; exit 1; }
step pmc-write
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$TAG -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > $O/pmc_write_$TAG.log 2>&1 || { tail -20 $O/pmc_write_$TAG.log; exit 1; }
timeout -k 10 600 python bench.py --no-cpu-baseline --no-extras --dump-kernels $O/kernels_$TAG.json > $O/bench_kernels_$TAG.log 2>&1 || { tail -20 $O/bench_kernels_$TAG.log; exit 1; }
python tools/pmc_traffic.py $O/pmc_fetch_$TAG $O/pmc_write_$TAG --batch 64 --dtype bf16 --calib profiles/pmc_calib.json --kernels $O/kernels_$TAG.json -o $O/pmc_traffic.json || exit 1
step pmc-sq
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sqa_$TAG -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > $O/pmc_sqa_$TAG.log 2>&1 || { tail -20 $O/pmc_sqa_$TAG.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU SQ_INSTS_MFMA SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sqb_$TAG -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > $O/pmc_sqb_$TAG.log 2>&1 || { tail -20 $O/pmc_sqb_$TAG.log; exit 1; }
python tools/pmc_sq.py $O/pmc_sqa_$TAG $O/pmc_sqb_$TAG -o $O/pmc_sq_$TAG.json --top 40 > $O/pmc_sq_$TAG.txt 2>&1 || exit 1
step bench-with-traffic
ATHD_PMC_TRAFFIC=$O/pmc_traffic.json timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench_traffic.log 2>&1 || { tail -20 $O/bench_traffic.log; exit 1; }
tail -1 $O/bench_traffic.log
