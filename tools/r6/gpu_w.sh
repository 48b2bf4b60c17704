# bf16 encoder-level stage test (fused vs unfused narrow levels)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread -k "encoder_levels" > gpurun_out/r6w_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r6w_pytest.log
python -c "import json; d=json.load(open('gpurun_out/parity_report.json')); [print(k, {a: round(b,1) for a, b in v.items()}) for k, v in d.items() if 'encoder_levels' in k]"
exit $rc
