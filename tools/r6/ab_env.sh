# A/B of environment settings on the default library, alternating; usage: tools/r6/ab_env.sh TAG ROUNDS "ENV=V ..." "ENV=V ..."
set -o pipefail
export TMPDIR=/tmp
TAG=$1; N=$2; shift 2
for i in $(seq $N); do
  k=0
  for E in "$@"; do
    k=$((k+1))
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 --dump-kernels gpurun_out/${TAG}_k_${k}_$i.json > gpurun_out/${TAG}_b_${k}_$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_b_${k}_$i.log; exit 1; }
    python - "$E" gpurun_out/${TAG}_k_${k}_${i}_sites.json gpurun_out/${TAG}_b_${k}_$i.log "${AB_GREP:-attn}" <<'PY'
import json, sys
n, kf, bf, pat = sys.argv[1:5]
ks = json.load(open(kf))
d = json.loads(open(bf).read().strip().splitlines()[-1])
sel = [(k['kernel'][:60], round(k['ms'], 3)) for k in ks if any(p in k['kernel'] for p in pat.split(','))]
print(n, d['value'], d['ms_per_step'], 'sum', round(sum(k['ms'] for k in ks), 3), sel)
PY
  done
done
