# attn_pp_kernel: bit-identity test, then an A/B of ATHD_ATTN_PP (whole step + attention sites); tdec pad 3 vs 0
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -rf -p no:cacheprovider --timeout 240 --timeout-method thread -k "pingpong or reproducible" > gpurun_out/r6k_pytest.log 2>&1 || { tail -30 gpurun_out/r6k_pytest.log; exit 1; }
tail -2 gpurun_out/r6k_pytest.log
python -c "import json; d=json.load(open('gpurun_out/parity_report.json')); print(d.get('attn_pingpong'), d.get('bf16_reproducible'))"
AB_GREP=attn bash tools/r6/ab_env.sh r6k 2 "ATHD_ATTN_PP=0" "ATHD_ATTN_PP=1"
timeout -k 10 300 python -u tools/diag_det4.py ablibs/libathd_pad3.so ablibs/libathd_pad0.so > gpurun_out/r6k_det.log 2>&1 || { tail -20 gpurun_out/r6k_det.log; exit 1; }
cat gpurun_out/r6k_det.log
