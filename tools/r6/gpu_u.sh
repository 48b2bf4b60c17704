# iSTFT: spectrum prefetch at 2 waves per SIMD (is1) / 3 with spills (is2) against the default
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_GREP=istft bash tools/r6/ab.sh r6u 2 audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_is1.so ablibs/libathd_is2.so
