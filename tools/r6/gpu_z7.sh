# fdec_tail: two accumulator chains of 6 MFMAs per row (ATHD_FT_CH=2) against one chain of 12
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r6/same_env.py "ATHD_LIB=$PWD/ablibs/base.so" "ATHD_LIB=$PWD/ablibs/ftch2.so" 2>&1 | grep -v amdgpu.ids
AB_GREP=fdec_tail bash tools/r6/ab.sh r6z7 3 ablibs/base.so ablibs/ftch2.so
