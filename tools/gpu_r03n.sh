#!/bin/bash
# Round 3: iSTFT on the second stream per decode chunk (FO double-buffered) - parity, then the bench at 1, 2 and 4
# decode chunks (ATHD_DECODE_ITEMS 256 / 128 / 64), alternating.
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_r03n.log 2>&1
rc=$?; tail -3 $O/pytest_r03n.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for it in 256 128 64; do
    ATHD_DECODE_ITEMS=$it timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > $O/bn_${it}_$rep.log 2>&1 || { tail -5 $O/bn_${it}_$rep.log; exit 1; }
    echo "items=$it rep=$rep $(tail -1 $O/bn_${it}_$rep.log | cut -c1-170)"
  done
done
