# attention V reads by inline asm (no compiler vmcnt(0) before them): parity + A/B against the builtin reads
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -rf -p no:cacheprovider --timeout 240 --timeout-method thread -k "sharp or pingpong or reproducible or golden or bench_batch" > gpurun_out/r6s_pytest.log 2>&1 || { tail -30 gpurun_out/r6s_pytest.log; exit 1; }
tail -1 gpurun_out/r6s_pytest.log
python -c "import json; d=json.load(open('gpurun_out/parity_report.json')); print(d.get('sharp_attention'), d.get('attn_pingpong'))"
AB_GREP=attn bash tools/r6/ab.sh r6s 3 audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_va0.so
