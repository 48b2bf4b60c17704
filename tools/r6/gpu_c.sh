# attention row sums: v_pk_add_f32 (default) vs single v_add_f32 (ATHD_ATTN_SSUM=1)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_GREP=attn32 bash tools/r6/ab.sh r6c 2 audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_ss.so
