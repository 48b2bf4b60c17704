# deterministic fdec1 Gram statistics: parity + reproducibility tests, run-to-run SDR vs the previous library, sites
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "fdec1 or reproducible or golden_fixture or full_segment or bench_batch or ragged or prompts" > gpurun_out/r5p_pytest.log 2>&1 || { tail -30 gpurun_out/r5p_pytest.log; exit 1; }
tail -1 gpurun_out/r5p_pytest.log
python -c "import json; d=json.load(open('gpurun_out/parity_report.json')); print({k: v for k, v in d.items() if 'fdec1' in k or 'reprod' in k})"
timeout -k 10 300 python tools/diag_det.py ablibs/libathd_prev.so > gpurun_out/r5p_det.log 2>&1 || { tail -5 gpurun_out/r5p_det.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5p_det.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels gpurun_out/k_b.json > gpurun_out/b_b.log 2>&1 || exit 1
python -c "import json,sys; [print(k['kernel'][:60], round(k['ms'],3)) for k in json.load(open('gpurun_out/k_b_sites.json')) if 'gram' in k['kernel']]"
tail -1 gpurun_out/b_b.log | cut -c1-200
