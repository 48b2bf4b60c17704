# LDS trims: istft without the 16-KB resize table (51.2 -> 34.8 KB), tdec_tail 96-B rows (29.6 -> 25.3 KB)
set -o pipefail
export TMPDIR=/tmp
V=$(realpath ablibs/libathd_lds.so)
ATHD_LIB=$V timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden_fixture or full_segment or intermediates or reproducible or ragged or prompts" > gpurun_out/r5t_pytest.log 2>&1 || { tail -30 gpurun_out/r5t_pytest.log; exit 1; }
tail -1 gpurun_out/r5t_pytest.log
for L in audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_lds.so audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_lds.so; do
  n=$(basename $L .so)
  ATHD_LIB=$(realpath $L) timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels gpurun_out/k_$n.json > gpurun_out/b_$n.log 2>&1 || exit 1
  python -c "import json,sys; [print(sys.argv[1], k['kernel'][:50], round(k['ms'],3)) for k in json.load(open(sys.argv[2])) if any(x in k['kernel'] for x in ('istft','tdec_tail','dconv_apply'))]; d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'])" $n gpurun_out/k_${n}_sites.json gpurun_out/b_$n.log
done
