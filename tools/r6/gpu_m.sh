# SQ counters: attn32_kernel vs attn_pp_kernel<0> (two passes each, 1-step bench)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_r6m
mkdir -p $O
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras"
run() { timeout -s KILL 240 rocprofv3 --pmc $2 --output-format csv -d $O/$1 -o run -- $B > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }; }
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
Bc="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES SQ_INST_CYCLES_VMEM"
run a0 "$A" && run b0 "$Bc"
export ATHD_ATTN_PP=2
run a2 "$A" && run b2 "$Bc"
unset ATHD_ATTN_PP
python tools/pmc_sq.py $O/a0 $O/b0 -o $O/sq0.json --top 8 > $O/sq0.txt 2>&1
python tools/pmc_sq.py $O/a2 $O/b2 -o $O/sq2.json --top 8 > $O/sq2.txt 2>&1
cat $O/sq0.txt $O/sq2.txt
python - <<'PY'
import json
for f in ("gpurun_out/pmc_r6m/sq0.json", "gpurun_out/pmc_r6m/sq2.json"):
    d = json.load(open(f))
    for k, v in d.items():
        if "attn" in k:
            print(k, {c: round(x) for c, x in v["counters"].items()})
PY
