# store-then-MFMA (WAR) hazard probe; one bench line with the new defaults (ATHD_NT=0)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 tools/hazard/mfma_war > gpurun_out/r6h_war.txt 2>&1 || { cat gpurun_out/r6h_war.txt; exit 1; }
cat gpurun_out/r6h_war.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r6h_bench.log 2>&1 || { tail -5 gpurun_out/r6h_bench.log; exit 1; }
tail -1 gpurun_out/r6h_bench.log | cut -c1-400
