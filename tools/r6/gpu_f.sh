# bisect of the bf16 golden-fixture drop (34 dB on b1_t44100_vocals) + the MFMA-chain hazard probe
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 ./tools/hazard/mfma_ds > gpurun_out/r6f_hazard.txt 2>&1; cat gpurun_out/r6f_hazard.txt
run() { rm -f gpurun_out/parity_report.json; timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden_fixture and bf16" > gpurun_out/r6f_$1.log 2>&1; python -c "import json; d=json.load(open('gpurun_out/parity_report.json')); print('$1', {k: round(v['sdr_db'],2) for k, v in d.items() if k.endswith('/bf16') and 'sdr_db' in v})"; }
run default
ATHD_NT=0 run nt0
ATHD_LIB=$(realpath ablibs/libathd_ss0.so) run ss0
ATHD_LIB=$(realpath ablibs/libathd_km.so) run km
ATHD_LIB=$(realpath ablibs/libathd_is5.so) run is5
ATHD_LIB=$(realpath ablibs/libathd_tc5.so) run tc5
