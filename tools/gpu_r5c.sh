set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden_fixture or full_segment or bench_batch or prompts_long or ragged" > gpurun_out/r5c_pytest.log 2>&1 || { tail -30 gpurun_out/r5c_pytest.log; exit 1; }
tail -1 gpurun_out/r5c_pytest.log
for lv in 1 0; do FR_LEVEL=$lv ATHD_LIB=$(realpath ablibs/libathd_frstamp.so) timeout -k 10 300 python tools/fr_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1; done
timeout -k 10 900 bash tools/gpu_ab_lib.sh ablibs/libathd_prev.so audio-to-sheet-music_amd/athd/libathd.so 2 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels gpurun_out/k_r5c.json > gpurun_out/b_r5c.log 2>&1 || exit 1
python tools/sites_diff.py gpurun_out/k_fr1new_sites.json gpurun_out/k_r5c_sites.json -n 8
