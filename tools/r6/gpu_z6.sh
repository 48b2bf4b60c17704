# occupancy bounds: dec_merge_w1 at 4 waves per SIMD (46 VGPRs spilled), fdec_lr_merge3 at 6 (10 spilled)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_GREP=merge,fdec_tail bash tools/r6/ab.sh r6z6 3 ablibs/base.so ablibs/mw1lb4.so ablibs/lr3lb6.so
