#!/bin/bash
# SQ counter pass over a short bench for kernels matching $1 (regex), summary to stdout.  $2 = tag
O=gpurun_out/pmck_${2:-x}
mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras"
timeout -s KILL 240 rocprofv3 --kernel-include-regex "$1" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/a -o run -- $B > $O/a.log 2>&1 || { tail -5 $O/a.log; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-include-regex "$1" --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA --output-format csv -d $O/b -o run -- $B > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
python tools/pmc_sq.py $O/a $O/b -o $O/sq.json > $O/sq.txt 2>&1; cat $O/sq.txt | cut -c1-160
python - "$O/sq.json" <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
for k,v in d.items():
    c=v['counters']; w=c.get('SQ_WAVES',0) or 1
    print(k[:60], {x: round(c[x]/w) for x in c if x.startswith('SQ_') and x!='SQ_WAVES'})
PY
