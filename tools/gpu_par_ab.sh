#!/bin/bash
# forward parity tests (bf16 SDR summary) then a kernel-time A/B: tools/gpu_par_ab.sh "<regex>" [variants...]
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_par.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_par.log
python -c "import json; d=json.load(open('gpurun_out/parity_report.json')); print({k: round(v.get('sdr_db', v.get('sdr_db_vs_oracle', 0)), 1) for k, v in d.items() if 'bf16' in k})"
[ $rc -eq 0 ] || exit $rc
RE="$1"; shift
AB_RE="$RE" bash tools/gpu_ab.sh "${@:-base}"
