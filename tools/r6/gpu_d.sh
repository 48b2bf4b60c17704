# split-K tail of linear2 + non-temporal linear1 stores: parity (split == unsplit, reproducible, vs oracle; bench
# config), then A/B of ATHD_SK / ATHD_NT
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 180 --timeout-method thread -k "splitk or bench_batch or sharp or reproducible or golden_fixture" > gpurun_out/r6d_pytest.log 2>&1 || { tail -30 gpurun_out/r6d_pytest.log; exit 1; }
tail -2 gpurun_out/r6d_pytest.log
python -c "import json; d=json.load(open('gpurun_out/parity_report.json')); print(d.get('splitk_tail'), d.get('sharp_attention'))"
AB_GREP=linear,sk_reduce,attn32,4225 bash tools/r6/ab_env.sh r6d 2 "ATHD_SK=1 ATHD_NT=1" "ATHD_SK=0 ATHD_NT=1" "ATHD_SK=1 ATHD_NT=0"
