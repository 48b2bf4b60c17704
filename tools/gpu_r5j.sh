set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden_fixture or full_segment or bench_batch or ragged" > gpurun_out/r5j_pytest.log 2>&1 || { tail -30 gpurun_out/r5j_pytest.log; exit 1; }
tail -1 gpurun_out/r5j_pytest.log
for L in ablibs/libathd_prev.so audio-to-sheet-music_amd/athd/libathd.so; do
  n=$(basename $L .so)
  ATHD_LIB=$(realpath $L) timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels gpurun_out/k_$n.json > gpurun_out/b_$n.log 2>&1 || exit 1
done
python tools/sites_diff.py gpurun_out/k_libathd_prev_sites.json gpurun_out/k_libathd_sites.json -n 6
timeout -k 10 900 bash tools/gpu_ab_lib.sh ablibs/libathd_prev.so audio-to-sheet-music_amd/athd/libathd.so 2 || exit 1
