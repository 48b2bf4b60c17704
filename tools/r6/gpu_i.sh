# tdec_tail pad discrimination: pad 0 (none), pad 2 (scheduling fence only), pad 0 with serial branches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_det4.py ablibs/libathd_pad0.so ablibs/libathd_pad2.so > gpurun_out/r6i_det.log 2>&1 || { tail -20 gpurun_out/r6i_det.log; exit 1; }
cat gpurun_out/r6i_det.log
ATHD_SERIAL=1 ATHD_LIB=$(realpath ablibs/libathd_pad0.so) timeout -k 10 200 python -u tools/diag_det4.py run > gpurun_out/r6i_det_serial.log 2>&1 || { tail -20 gpurun_out/r6i_det_serial.log; exit 1; }
echo "pad0 serial:"; cat gpurun_out/r6i_det_serial.log
