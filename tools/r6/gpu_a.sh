# round 6, first pass: the whole -m gpu suite (incl. the new decoder-stage pin and ATHD_ROWLN=0 tests), then the
# driver's bench protocol with the per-site kernel dump
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r6a_pytest.log 2>&1 || { tail -30 gpurun_out/r6a_pytest.log; exit 1; }
tail -3 gpurun_out/r6a_pytest.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --dump-kernels gpurun_out/r6a_k.json > gpurun_out/r6a_bench.log 2>&1 || { tail -20 gpurun_out/r6a_bench.log; exit 1; }
tail -1 gpurun_out/r6a_bench.log | cut -c1-400
