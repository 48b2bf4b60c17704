#!/bin/bash
# PMC passes over a short bench (one rocprofv3 --pmc pass per counter group, each its own run):
# SQ stall/busy + MFMA busy, SQ instruction mix, FETCH_SIZE, WRITE_SIZE.  $1 = output tag (e.g. r02)
T=${1:-r02}
O=gpurun_out/pmc_$T
mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras"
run() { timeout -s KILL 240 rocprofv3 --pmc $2 --output-format csv -d $O/$1 -o run -- $B > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }; }
run sqa "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
run sqb "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU SQ_INSTS_MFMA SQ_BUSY_CYCLES"
run fetch "FETCH_SIZE"
run write "WRITE_SIZE"
python tools/pmc_sq.py $O/sqa $O/sqb -o $O/pmc_sq.json --top 30 > $O/pmc_sq.txt 2>&1
python tools/pmc_traffic.py $O/fetch $O/write --batch 64 --dtype bf16 -o $O/pmc_traffic.json > $O/pmc_traffic_top.txt 2>&1
cat $O/pmc_sq.txt | cut -c1-150; cat $O/pmc_traffic_top.txt
