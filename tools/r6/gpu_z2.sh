# text mlp2 + norm_out, per-item tiles with the prompts of a segment adjacent: against gemm3's form (ATHD_RLT=0)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -k "text_mlp2_ln_forms or bench_batch_one_chunk" 2>&1 | grep -v amdgpu.ids | tail -4
AB_GREP=mlp2 bash tools/r6/ab_env.sh r6z2 3 "ATHD_RLT=0" "ATHD_RLT=1"
