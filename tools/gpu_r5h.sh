set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden_fixture or full_segment or bench_batch or ragged or graph_replay" > gpurun_out/r5h_pytest.log 2>&1 || { tail -30 gpurun_out/r5h_pytest.log; exit 1; }
tail -1 gpurun_out/r5h_pytest.log
ATHD_LIB=$(realpath ablibs/libathd_ct2.so) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "full_segment or bench_batch" > gpurun_out/r5h_pytest2.log 2>&1 || { tail -30 gpurun_out/r5h_pytest2.log; exit 1; }
tail -1 gpurun_out/r5h_pytest2.log
for L in ablibs/libathd_prev.so audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_ct2.so; do
  n=$(basename $L .so)
  ATHD_LIB=$(realpath $L) timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels gpurun_out/k_$n.json > gpurun_out/b_$n.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/b_$n.log $n
  python -c "import json,sys; [print(sys.argv[1], k['kernel'], round(k['ms'],3)) for k in json.load(open(sys.argv[2])) if 'convt4' in k['kernel']]" $n gpurun_out/k_${n}_sites.json
done
timeout -k 10 900 bash tools/gpu_ab_lib.sh ablibs/libathd_prev.so audio-to-sheet-music_amd/athd/libathd.so 2 || exit 1
