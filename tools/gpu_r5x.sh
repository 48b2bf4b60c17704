# iSTFT at 4 workgroups per CU (resize computed per bin, 128 VGPRs with 14 spilled, 34.8 KB LDS) vs 3
set -o pipefail
export TMPDIR=/tmp
V=$(realpath ablibs/libathd_is.so)
ATHD_LIB=$V timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden_fixture or full_segment or ragged or reproducible" > gpurun_out/r5x_pytest.log 2>&1 || { tail -30 gpurun_out/r5x_pytest.log; exit 1; }
tail -1 gpurun_out/r5x_pytest.log
for L in audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_is.so audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_is.so; do
  n=$(basename $L .so)
  ATHD_LIB=$(realpath $L) timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 --dump-kernels gpurun_out/k_$n.json > gpurun_out/b_$n.log 2>&1 || exit 1
  python -c "import json,sys; [print(sys.argv[1], k['kernel'][:50], round(k['ms'],3)) for k in json.load(open(sys.argv[2])) if 'istft_ola' in k['kernel']]; d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'])" $n gpurun_out/k_${n}_sites.json gpurun_out/b_$n.log
done
