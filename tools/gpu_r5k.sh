set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden_fixture or full_segment or bench_batch or ragged or attention or transformer" > gpurun_out/r5k_pytest.log 2>&1 || { tail -30 gpurun_out/r5k_pytest.log; exit 1; }
tail -1 gpurun_out/r5k_pytest.log
LIBS="ablibs/libathd_prev.so ablibs/libathd_tail.so audio-to-sheet-music_amd/athd/libathd.so"
for L in $LIBS; do
  n=$(basename $L .so)
  ATHD_LIB=$(realpath $L) timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels gpurun_out/k_$n.json > gpurun_out/b_$n.log 2>&1 || exit 1
  python -c "import json,sys; [print(sys.argv[1], k['kernel'][:60], round(k['ms'],3)) for k in json.load(open(sys.argv[2])) if 'attn32' in k['kernel'] or 'tail' in k['kernel']]" $n gpurun_out/k_${n}_sites.json
done
for i in 1 2; do for L in $LIBS; do
  ATHD_LIB=$(realpath $L) timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $L
done; done
