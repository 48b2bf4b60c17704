set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden_fixture or full_segment or bench_batch or prompts_long or ragged or fdec1 or decode_chunks or graph_replay" > gpurun_out/r5d_pytest.log 2>&1 || { tail -30 gpurun_out/r5d_pytest.log; exit 1; }
tail -1 gpurun_out/r5d_pytest.log

timeout -k 10 900 bash tools/gpu_ab_lib.sh ablibs/libathd_prev.so audio-to-sheet-music_amd/athd/libathd.so 2 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels gpurun_out/k_ct4old.json > gpurun_out/b_ct4old.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels gpurun_out/k_ct4new.json > gpurun_out/b_ct4new.log 2>&1 || exit 1
python tools/sites_diff.py gpurun_out/k_ct4old_sites.json gpurun_out/k_ct4new_sites.json -n 10
