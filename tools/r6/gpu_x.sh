# decoder tail in parts (ATHD_TAIL_SPLIT): identity vs one part, tests, A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r6/same_env.py "ATHD_TAIL_SPLIT=1" "ATHD_TAIL_SPLIT=2" 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/r6/same_env.py "ATHD_TAIL_SPLIT=1" "ATHD_TAIL_SPLIT=4" 2>&1 | grep -v amdgpu.ids
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -rf -p no:cacheprovider --timeout 240 --timeout-method thread -k "chunks or reproducible or graph_replay or bench_batch or golden or intermediates" > gpurun_out/r6x_pytest.log 2>&1 || { tail -30 gpurun_out/r6x_pytest.log; exit 1; }
tail -1 gpurun_out/r6x_pytest.log
AB_GREP=istft,fdec_tail bash tools/r6/ab_env.sh r6x 3 "ATHD_TAIL_SPLIT=1" "ATHD_TAIL_SPLIT=2" "ATHD_TAIL_SPLIT=4"
