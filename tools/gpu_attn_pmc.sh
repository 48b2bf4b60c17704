#!/bin/bash
# SQ counters of the attention variants (one rocprofv3 --pmc pass per counter group) on the kbench attn1 shape
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc_avail.txt 2>&1
grep -oE "SQ_[A-Z_0-9]+" gpurun_out/pmc_avail.txt | sort -u > gpurun_out/pmc_sq_names.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc_attn1 -o run -- python tools/kbench.py attn1 > gpurun_out/pmc_attn1.log 2>&1
rc=$?; tail -3 gpurun_out/pmc_attn1.log; exit $rc
