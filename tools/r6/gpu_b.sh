# attention round-6 form: parity (sharp attention, fixtures, bench config, reproducibility), then A/B vs the round-5 form
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k "sharp or golden_fixture or full_segment or bench_batch or reproducible or intermediates or ragged" > gpurun_out/r6b_pytest.log 2>&1 || { tail -30 gpurun_out/r6b_pytest.log; exit 1; }
tail -2 gpurun_out/r6b_pytest.log
python -c "import json; d=json.load(open('gpurun_out/parity_report.json')); print(d.get('sharp_attention'))"
AB_GREP=attn bash tools/r6/ab.sh r6b 2 audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_a5.so
