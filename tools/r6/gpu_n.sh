# iSTFT time-branch prefetch A/B (libathd vs libathd_sph = previous spectral.o); decode chunk 256 vs 128 items; full -m gpu
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r6n_pytest.log 2>&1 || { tail -30 gpurun_out/r6n_pytest.log; exit 1; }
tail -2 gpurun_out/r6n_pytest.log
AB_GREP=istft bash tools/r6/ab.sh r6n 3 audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_sph.so
for i in 1 2; do for di in 256 128; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 --decode-items $di > gpurun_out/r6n_di_${di}_$i.log 2>&1 || { tail -5 gpurun_out/r6n_di_${di}_$i.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/r6n_di_${di}_$i.log').read().strip().splitlines()[-1]); print('decode_items', $di, d['value'], d['ms_per_step'])"
done; done
