#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) + SQ summary of the kernels matching $1 over a 1-step bench
O=gpurun_out/pmckt_${2:-x}
mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras"
timeout -s KILL 240 rocprofv3 --kernel-include-regex "$1" --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- $B > $O/f.log 2>&1 || { tail -5 $O/f.log; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-include-regex "$1" --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- $B > $O/w.log 2>&1 || { tail -5 $O/w.log; exit 1; }
python - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for tag in ("f", "w"):
    agg = collections.defaultdict(lambda: [0.0, 0])
    for fn in glob.glob(f"{o}/{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            k = r["Kernel_Name"][:70]
            agg[(k, r["Dispatch_Id"])][0] += float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for (k, _), v in agg.items(): per[k].append(v[0])
    for k, v in per.items(): print(tag, k, "n=%d" % len(v), "avg %.1f MB (raw counter x1024)" % (sum(v) / len(v) * 1024 / 1e6))
PY
bash tools/gpu_pmc_k.sh "$1" ${2:-x}
