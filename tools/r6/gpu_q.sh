# split-K reduce rewrite: parity tests + timing
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -rf -p no:cacheprovider --timeout 240 --timeout-method thread -k "splitk or reproducible or bench_batch" > gpurun_out/r6q_pytest.log 2>&1 || { tail -30 gpurun_out/r6q_pytest.log; exit 1; }
tail -1 gpurun_out/r6q_pytest.log
AB_GREP=linear2 bash tools/r6/ab_env.sh r6q 2 "ATHD_SK=1" "ATHD_SK=0"
