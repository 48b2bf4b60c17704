set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_g6
mkdir -p $O
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/sqa -o run -- $B > $O/sqa.log 2>&1 || { tail -5 $O/sqa.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU SQ_INSTS_MFMA SQ_BUSY_CYCLES --output-format csv -d $O/sqb -o run -- $B > $O/sqb.log 2>&1 || { tail -5 $O/sqb.log; exit 1; }
python tools/pmc_sq.py $O/sqa $O/sqb -o $O/pmc_sq.json --top 40 > $O/pmc_sq.txt 2>&1
head -1 $O/pmc_sq.txt; grep -E "gemm6|gemm5" $O/pmc_sq.txt | cut -c1-160
