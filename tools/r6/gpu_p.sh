# non-temporal whole-line epilogue stores (ATHD_NT=1: linear1, 2: + QKV/Q/KV): identity, timing, PMC traffic
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r6/same_env.py "ATHD_NT=0" "ATHD_NT=2" 2>&1 | grep -v amdgpu.ids
AB_GREP=linear1,qkv,kv bash tools/r6/ab_env.sh r6p 2 "ATHD_NT=0" "ATHD_NT=1" "ATHD_NT=2"
O=gpurun_out/pmc_r6p
mkdir -p $O
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras"
run() { timeout -s KILL 240 rocprofv3 --pmc $2 --output-format csv -d $O/$1 -o run -- $B > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }; }
export ATHD_NT=2; run f2 FETCH_SIZE && run w2 WRITE_SIZE; unset ATHD_NT
python tools/pmc_traffic.py $O/f2 $O/w2 --batch 64 --dtype bf16 -o $O/t2.json > $O/t2.txt 2>&1
python -c "import json; d=json.load(open('$O/t2.json'))['kernels']; [print(n, {a: round(v[a],3) for a in ('fetch_kib','write_kib','traffic_over_algorithmic') if a in v}) for n, v in d.items() if n.startswith('gemm5')]"
