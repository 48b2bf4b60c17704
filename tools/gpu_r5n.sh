# gemm6 (constant waits) vs gemm5: parity with ATHD_G6=1, then serialised kernel sites of both
set -o pipefail
export TMPDIR=/tmp
ATHD_G6=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden_fixture or full_segment or bench_batch or transformer" > gpurun_out/r5n_pytest.log 2>&1 || { tail -30 gpurun_out/r5n_pytest.log; exit 1; }
tail -1 gpurun_out/r5n_pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels gpurun_out/k_a.json > gpurun_out/b_a.log 2>&1 || exit 1
ATHD_G6=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels gpurun_out/k_b.json > gpurun_out/b_b.log 2>&1 || exit 1
python tools/sites_diff.py gpurun_out/k_a_sites.json gpurun_out/k_b_sites.json -n 10
tail -1 gpurun_out/b_a.log; tail -1 gpurun_out/b_b.log
