#!/bin/bash
# compact level-3 skips + XCD-ordered tdec_tail: parity tests, then a whole-model A/B against the previous commit
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_r03d.log 2>&1
rc=$?; tail -3 $O/pytest_r03d.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest_r03d.log | head -20; exit $rc; }
timeout -k 10 500 bash tools/gpu_ab_lib.sh ablibs/libathd_prev.so audio-to-sheet-music_amd/athd/libathd.so 3 || exit 1
ATHD_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r03d -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $O/prof_r03d.log 2>&1 || { tail -5 $O/prof_r03d.log; exit 1; }
python tools/prof_summary.py $O/prof_r03d | head -30
