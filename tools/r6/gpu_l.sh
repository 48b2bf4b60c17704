# attn_pp_kernel: bit-identity (3 prio modes), A/B of the modes against attn32_kernel
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 1 2 3; do
  ATHD_PP_TEST_MODE=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -rf -p no:cacheprovider --timeout 240 --timeout-method thread -k "pingpong" > gpurun_out/r6l_pytest_$m.log 2>&1 || { tail -30 gpurun_out/r6l_pytest_$m.log; exit 1; }
  tail -1 gpurun_out/r6l_pytest_$m.log
done
AB_GREP=attn bash tools/r6/ab_env.sh r6l 2 "ATHD_ATTN_PP=0" "ATHD_ATTN_PP=1" "ATHD_ATTN_PP=2" "ATHD_ATTN_PP=3"
