# fenc_row0 as 8-wave workgroups: bf16 output vs the 6-wave library, parity tests, A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r6/same_env.py "ATHD_LIB=$(realpath ablibs/libathd_f6.so)" "ATHD_X=1" 2>&1 | grep -v amdgpu.ids
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -rf -p no:cacheprovider --timeout 240 --timeout-method thread -k "golden or full_segment or reproducible or bench_batch or ragged" > gpurun_out/r6t_pytest.log 2>&1 || { tail -30 gpurun_out/r6t_pytest.log; exit 1; }
tail -1 gpurun_out/r6t_pytest.log
python -c "import json; d=json.load(open('gpurun_out/parity_report.json')); print({k: v for k, v in d.items() if 'bf16' in k})"
AB_GREP=fenc_row bash tools/r6/ab.sh r6t 3 audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_f6.so
