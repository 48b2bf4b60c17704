# gemm5 persistent grid for the residual + statistics epilogue (linear2): parity with the variant, sites, A/B
set -o pipefail
export TMPDIR=/tmp
V=$(realpath ablibs/libathd_pres.so)
ATHD_LIB=$V timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden_fixture or full_segment or intermediates or reproducible or transformer or bench_batch" > gpurun_out/r5u_pytest.log 2>&1 || { tail -30 gpurun_out/r5u_pytest.log; exit 1; }
tail -1 gpurun_out/r5u_pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels gpurun_out/k_a.json > gpurun_out/b_a.log 2>&1 || exit 1
ATHD_LIB=$V timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --dump-kernels gpurun_out/k_b.json > gpurun_out/b_b.log 2>&1 || exit 1
python tools/sites_diff.py gpurun_out/k_a_sites.json gpurun_out/k_b_sites.json -n 5
for i in 1 2 3; do for L in ablibs/libathd_pres.so audio-to-sheet-music_amd/athd/libathd.so; do
  ATHD_LIB=$(realpath $L) timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $L
done; done
