# rowln residual prefetch depth (RD 1 / 2 default / 3) and fdec_tail rows per chunk (16 / 32 default / 64)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_GREP=rowln,fdec_tail bash tools/r6/ab.sh r6r 2 audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_rl1.so ablibs/libathd_rl3.so ablibs/libathd_ft16.so ablibs/libathd_ft64.so
