# text mlp2 + norm_out: rowln.hip's text form (default) against gemm3's (ATHD_RLT=0)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -k "text_mlp2_ln_forms or rowln_off or bench_batch_one_chunk" 2>&1 | grep -v amdgpu.ids | tail -15
timeout -k 10 300 python -u tools/r6/same_env.py "ATHD_RLT=0" "ATHD_RLT=1" 2>&1 | grep -v amdgpu.ids
AB_GREP=mlp2,rowln bash tools/r6/ab_env.sh r6z 3 "ATHD_RLT=0" "ATHD_RLT=1"
