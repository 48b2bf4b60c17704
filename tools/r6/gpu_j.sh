# tdec_tail: the 48-state delay at the kernel start (pad 3) instead of before the z stores; pad 0 again
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_det4.py ablibs/libathd_pad3.so ablibs/libathd_pad0.so ablibs/libathd_pad3.so > gpurun_out/r6j_det.log 2>&1 || { tail -20 gpurun_out/r6j_det.log; exit 1; }
cat gpurun_out/r6j_det.log
