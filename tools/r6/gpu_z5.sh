# fdec_tail at 4 waves per SIMD (128 VGPRs, __launch_bounds__) against the compiler's 130 VGPRs (3 waves per SIMD)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_GREP=fdec_tail,istft bash tools/r6/ab.sh r6z5 3 ablibs/base.so ablibs/ftlb4.so
