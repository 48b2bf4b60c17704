#!/bin/bash
# One GPU job as a list of steps, run in order; the job stops at the first step that fails (each step has its own
# time limit).  Replaces the per-experiment one-off scripts of rounds 2-3.
#   bash tools/gpu_run.sh STEP [STEP ...]
# Steps (arguments separated by ':'):
#   pytest[:K]              -m gpu tests (optionally -k K)              -> gpurun_out/pytest_<n>.log
#   bench[:ARGS]            bench.py --no-cpu-baseline ARGS (ARGS: ',' for spaces)
#   full                    bench.py with the CPU baseline (the driver's default line)
#   sites:TAG               bench + per-call-site kernel times           -> gpurun_out/k_TAG.json / k_TAG_sites.json
#   ab:A.so:B.so[:ROUNDS]   whole-model A/B of two library builds, alternating runs (tools/gpu_ab_lib.sh)
#   kbench:MODE[:LIB]       tools/kbench.py MODE (kernel micro-benchmarks; tools/libkbench.so or tools/LIB)
#   prof:TAG                rocprofv3 kernel trace of a short bench, both streams and serialised (ATHD_SERIAL=1)
#   sq:TAG                  two SQ counter passes + summary                -> gpurun_out/pmc_sq_TAG.txt
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  IFS=: read -r name a1 a2 a3 <<< "$step"
  echo "== [$n] $step"
  case $name in
    pytest)
      K=(); [ -n "$a1" ] && K=(-k "$a1")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA -p no:cacheprovider --timeout 120 --timeout-method thread "${K[@]}" > $O/pytest_$n.log 2>&1
      rc=$?; grep -E "passed|failed" $O/pytest_$n.log | tail -2
      if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $O/pytest_$n.log | head -20; exit $rc; fi ;;
    bench)
      timeout -k 10 400 python bench.py --no-cpu-baseline ${a1//,/ } > $O/bench_$n.log 2>&1 || { tail -20 $O/bench_$n.log; exit 1; }
      tail -2 $O/bench_$n.log | cut -c1-700 ;;
    full)
      timeout -k 10 600 python bench.py > $O/bench_full.log 2>&1 || { tail -20 $O/bench_full.log; exit 1; }
      tail -1 $O/bench_full.log | cut -c1-700 ;;
    sites)
      timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 2 --dump-kernels $O/k_$a1.json > $O/b_$a1.log 2>&1 || { tail -5 $O/b_$a1.log; exit 1; }
      tail -1 $O/b_$a1.log | cut -c1-160 ;;
    ab)
      timeout -k 10 900 bash tools/gpu_ab_lib.sh "$a1" "$a2" "${a3:-2}" || exit 1 ;;
    kbench)
      KB_LIB=${a2:-libkbench.so} timeout -k 10 600 python tools/kbench.py $a1 > $O/kbench_$n.log 2>&1; rc=$?
      grep -v amdgpu.ids $O/kbench_$n.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$a1 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $O/prof_$a1.log 2>&1 || { tail -20 $O/prof_$a1.log; exit 1; }
      python tools/timeline.py $O/prof_$a1 --last-steps 2 > $O/timeline_$a1.txt 2>&1; head -20 $O/timeline_$a1.txt
      ATHD_SERIAL=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${a1}_serial -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $O/prof_${a1}_serial.log 2>&1 || { tail -20 $O/prof_${a1}_serial.log; exit 1; }
      python tools/prof_sections.py $O/prof_${a1}_serial > $O/sections_$a1.txt 2>&1; head -40 $O/sections_$a1.txt ;;
    sq)
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sqa_$a1 -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > $O/pmc_sqa_$a1.log 2>&1 || { tail -20 $O/pmc_sqa_$a1.log; exit 1; }
      timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU SQ_INSTS_MFMA SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sqb_$a1 -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > $O/pmc_sqb_$a1.log 2>&1 || { tail -20 $O/pmc_sqb_$a1.log; exit 1; }
      python tools/pmc_sq.py $O/pmc_sqa_$a1 $O/pmc_sqb_$a1 -o $O/pmc_sq_$a1.json --top 40 > $O/pmc_sq_$a1.txt 2>&1 || exit 1
      head -30 $O/pmc_sq_$a1.txt ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
exit 0
