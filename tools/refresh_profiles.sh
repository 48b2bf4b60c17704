#!/bin/bash
# Copy the summaries of a tools/gpu_round.sh <tag> run (merged back into gpurun_out/) into profiles/.
TAG=${1:-r01}
O=gpurun_out
P=profiles
set -e
cp $O/prof_$TAG/run_kernel_stats.csv $P/${TAG}_kernel_stats.csv
python tools/prof_summary.py $O/prof_$TAG > $P/${TAG}_kernel_summary.txt
python tools/prof_sections.py $O/prof_$TAG > $P/${TAG}_sections.txt
cp $O/prof_${TAG}_serial/run_kernel_stats.csv $P/${TAG}_kernel_stats_serial.csv
python tools/prof_summary.py $O/prof_${TAG}_serial > $P/${TAG}_kernel_summary_serial.txt
python tools/prof_sections.py $O/prof_${TAG}_serial > $P/${TAG}_sections_serial.txt
cp $O/pmc_traffic.json $P/pmc_traffic.json
python tools/pmc_traffic.py $O/pmc_fetch_$TAG $O/pmc_write_$TAG --batch 64 --dtype bf16 --calib $P/pmc_calib.json --kernels $O/kernels_$TAG.json -o /tmp/pmc_traffic.json > $P/${TAG}_pmc_traffic_top.txt
[ -f $O/bench_full.log ] && tail -1 $O/bench_full.log > $P/${TAG}_bench.json
tail -1 $O/bench_traffic.log | sed 's#gpurun_out/pmc_traffic.json#profiles/pmc_traffic.json#' > $P/${TAG}_bench_traffic.json
[ -f $O/timeline_$TAG.txt ] && cp $O/timeline_$TAG.txt $P/${TAG}_timeline.txt
[ -f $O/kernels_${TAG}_sites.json ] && cp $O/kernels_${TAG}_sites.json $P/${TAG}_sites.json
[ -f $O/pmc_sq_$TAG.txt ] && cp $O/pmc_sq_$TAG.txt $P/pmc_sq_$TAG.txt && cp $O/pmc_sq_$TAG.json $P/pmc_sq_$TAG.json
true
