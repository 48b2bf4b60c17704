set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden_fixture or full_segment or bench_batch or prompts_long or ragged" > gpurun_out/r5b_pytest.log 2>&1 || { tail -30 gpurun_out/r5b_pytest.log; exit 1; }
tail -1 gpurun_out/r5b_pytest.log
FR_LEVEL=1 ATHD_LIB=$(realpath ablibs/libathd_frstamp.so) timeout -k 10 300 python tools/fr_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/gpu_env_ab.sh ATHD_FR1=0 2 || exit 1
ATHD_FR1=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels gpurun_out/k_fr1old.json > gpurun_out/b_fr1old.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels gpurun_out/k_fr1new.json > gpurun_out/b_fr1new.log 2>&1 || exit 1
python tools/sites_diff.py gpurun_out/k_fr1old_sites.json gpurun_out/k_fr1new_sites.json -n 12
