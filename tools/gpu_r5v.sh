# convt4_walk_kernel row-segment count sweep (ATHD_CW_SEG 7 / 10 / 14 / 20): parity of one variant, fdec2 site times
set -o pipefail
export TMPDIR=/tmp
ATHD_LIB=$(realpath ablibs/libathd_s7.so) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden_fixture or full_segment" > gpurun_out/r5v_pytest.log 2>&1 || { tail -30 gpurun_out/r5v_pytest.log; exit 1; }
tail -1 gpurun_out/r5v_pytest.log
for L in audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_s7.so ablibs/libathd_s10.so ablibs/libathd_s20.so audio-to-sheet-music_amd/athd/libathd.so; do
  n=$(basename $L .so)
  ATHD_LIB=$(realpath $L) timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels gpurun_out/k_$n.json > gpurun_out/b_$n.log 2>&1 || exit 1
  python -c "import json,sys; [print(sys.argv[1], k['kernel'][:50], round(k['ms'],3)) for k in json.load(open(sys.argv[2])) if 'walk' in k['kernel']]; d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'])" $n gpurun_out/k_${n}_sites.json gpurun_out/b_$n.log
done
