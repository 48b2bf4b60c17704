# full -m gpu suite; tdec_tail pad A/B (bit-reproducibility without the pad); bench A/B of KM / round-5 iSTFT; SK / NT
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r6g_pytest.log 2>&1 || { tail -30 gpurun_out/r6g_pytest.log; exit 1; }
tail -2 gpurun_out/r6g_pytest.log
python -c "import json; d=json.load(open('gpurun_out/parity_report.json')); print(d.get('splitk_tail'), d.get('sharp_attention'), d.get('bf16_reproducible')); print({k: round(v['sdr_db'],2) for k, v in d.items() if k.endswith('/bf16') and isinstance(v, dict) and 'sdr_db' in v})"
cp gpurun_out/parity_report.json gpurun_out/r6g_parity_report.json
for i in 1 2; do ATHD_LIB=$(realpath ablibs/libathd_nopad.so) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider --timeout 180 --timeout-method thread -k reproducible > gpurun_out/r6g_nopad_$i.log 2>&1; python -c "import json; d=json.load(open('gpurun_out/parity_report.json')); print('nopad', d.get('bf16_reproducible'))"; done
AB_GREP=attn32,istft bash tools/r6/ab.sh r6g 2 audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_km.so ablibs/libathd_is5.so
AB_GREP=linear,sk_reduce,4225,4224,qkv,tconv0 bash tools/r6/ab_env.sh r6g 2 "ATHD_SK=1 ATHD_NT=1" "ATHD_SK=0 ATHD_NT=1" "ATHD_SK=1 ATHD_NT=0" "ATHD_SK=1 ATHD_NT=2"
