#!/bin/bash
# gemm5 ablation probes + the hipBLASLt kernels' names/times on the same shapes (rocprofv3 kernel trace)
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/kbench.py g5probe > $O/kbench_g5probe.log 2>&1 || { tail -20 $O/kbench_g5probe.log; exit 1; }
grep -v amdgpu.ids $O/kbench_g5probe.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_g5 -o run -- python tools/kbench.py g5probe > $O/prof_g5.log 2>&1 || { tail -20 $O/prof_g5.log; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_g5/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us x{r["Calls"]:>4}  {r["Name"][:200]}')
PY
