#!/bin/bash
# compact level-3 skips + XCD-ordered tdec_tail: parity tests; then whole-model A/Bs: previous commit vs this tree,
# this tree vs (iSTFT without its LDS table at 4 waves/SIMD), vs (that + persistent residual-epilogue GEMMs)
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_r03e.log 2>&1
rc=$?; tail -3 $O/pytest_r03e.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest_r03e.log | head -20; exit $rc; }
CUR=audio-to-sheet-music_amd/athd/libathd.so
timeout -k 10 400 bash tools/gpu_ab_lib.sh ablibs/libathd_prev.so $CUR 2 || exit 1
timeout -k 10 400 bash tools/gpu_ab_lib.sh ablibs/libathd_i.so ablibs/libathd_pi.so 2 || exit 1
