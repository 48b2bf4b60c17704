#!/bin/bash
# A/B of kernel variants selected by environment: for each "NAME=VALUE" argument (or "base"), one short serial-branch
# bench under rocprofv3 --kernel-trace; prints the summary lines matching $AB_RE (default: all, top 12)
O=gpurun_out/ab
mkdir -p $O
export TMPDIR=/tmp
RE=${AB_RE:-.}
for v in "$@"; do
  tag=$(echo "$v" | tr '=' '_')
  if [ "$v" = base ]; then E=""; else E="$v"; fi
  env $E ATHD_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  echo "== $v: $(tail -1 $O/$tag.log | cut -c80-200)"
  python tools/prof_summary.py $O/$tag > $O/$tag.txt 2>&1
  grep -E "$RE" $O/$tag.txt | head -12 | cut -c1-150
done
