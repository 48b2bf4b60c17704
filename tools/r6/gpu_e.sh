# MFMA->LDS hazard probe; full -m gpu suite (attention max hazard fix, split-K, NT); A/B of row sums, split-K, NT
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/hazard/mfma_ds > gpurun_out/r6e_hazard.txt 2>&1; cat gpurun_out/r6e_hazard.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r6e_pytest.log 2>&1 || { tail -30 gpurun_out/r6e_pytest.log; exit 1; }
tail -2 gpurun_out/r6e_pytest.log
python -c "import json; d=json.load(open('gpurun_out/parity_report.json')); print(d.get('splitk_tail'), d.get('sharp_attention')); print({k: round(v['sdr_db'],2) for k, v in d.items() if k.endswith('/bf16') and isinstance(v, dict) and 'sdr_db' in v})"
AB_GREP=attn32,istft bash tools/r6/ab.sh r6e 2 audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_ss0.so ablibs/libathd_km.so ablibs/libathd_is5.so
AB_GREP=linear,sk_reduce,4225,4224,qkv,tconv0 bash tools/r6/ab_env.sh r6e 2 "ATHD_SK=1 ATHD_NT=1" "ATHD_SK=0 ATHD_NT=1" "ATHD_SK=1 ATHD_NT=0" "ATHD_SK=1 ATHD_NT=2"
