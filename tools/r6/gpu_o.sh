# linear1 tile order (ATHD_G5_ORD=1) and NT: bit-identity, timing A/B, PMC fetch/write
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r6/same_env.py "ATHD_G5_ORD=0" "ATHD_G5_ORD=1" 2>&1 | grep -v amdgpu.ids
AB_GREP=linear1 bash tools/r6/ab_env.sh r6o 2 "ATHD_G5_ORD=0" "ATHD_G5_ORD=1" "ATHD_NT=1"
O=gpurun_out/pmc_r6o
mkdir -p $O
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras"
run() { timeout -s KILL 240 rocprofv3 --pmc $2 --output-format csv -d $O/$1 -o run -- $B > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }; }
run f0 FETCH_SIZE && run w0 WRITE_SIZE
export ATHD_G5_ORD=1; run f1 FETCH_SIZE && run w1 WRITE_SIZE; unset ATHD_G5_ORD
export ATHD_NT=1; run f2 FETCH_SIZE && run w2 WRITE_SIZE; unset ATHD_NT
for k in 0 1 2; do
  python tools/pmc_traffic.py $O/f$k $O/w$k --batch 64 --dtype bf16 -o $O/t$k.json > $O/t$k.txt 2>&1
  python -c "import json; d=json.load(open('$O/t$k.json'))['kernels']; [print($k, n, {a: round(v[a],3) for a in ('fetch_kib','write_kib','traffic_over_algorithmic') if a in v}) for n, v in d.items() if n.startswith('gemm5')]"
done
