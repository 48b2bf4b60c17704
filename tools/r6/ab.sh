# A/B of libathd builds in one GPU run, bench.py without extras (driver protocol steps), alternating;
# per build: whole-step segments/s and the per-site times of the kernels matching $AB_GREP.
# usage: tools/r6/ab.sh TAG ROUNDS LIB1 LIB2 ...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; N=$2; shift 2
for i in $(seq $N); do
  for L in "$@"; do
    n=$(basename $L .so)
    ATHD_LIB=$(realpath $L) timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 --dump-kernels gpurun_out/${TAG}_k_${n}_$i.json > gpurun_out/${TAG}_b_${n}_$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_b_${n}_$i.log; exit 1; }
    python - "$n" gpurun_out/${TAG}_k_${n}_${i}_sites.json gpurun_out/${TAG}_b_${n}_$i.log "${AB_GREP:-attn}" <<'PY'
import json, sys
n, kf, bf, pat = sys.argv[1:5]
ks = json.load(open(kf))
d = json.loads(open(bf).read().strip().splitlines()[-1])
sel = [(k['kernel'][:60], round(k['ms'], 3)) for k in ks if any(p in k['kernel'] for p in pat.split(','))]
print(n, d['value'], d['ms_per_step'], 'sum', round(sum(k['ms'] for k in ks), 3), sel)
PY
  done
done
