# text mlp2 + norm_out: rowln.hip's text form (row-major tiles) against gemm3's form (ATHD_RLT=0), 4 pairs
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -k "text_mlp2_ln_forms" 2>&1 | grep -v amdgpu.ids | tail -3
AB_GREP=mlp2 bash tools/r6/ab_env.sh r6z3 4 "ATHD_RLT=0" "ATHD_RLT=1"
