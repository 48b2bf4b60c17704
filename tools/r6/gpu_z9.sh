# the frequency branch on a high-priority library stream (ATHD_PRIO=1 build) against the caller's stream
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r6/same_env.py "ATHD_LIB=$PWD/ablibs/base.so" "ATHD_LIB=$PWD/ablibs/prio.so" 2>&1 | grep -v amdgpu.ids
AB_GREP=attn32 bash tools/r6/ab.sh r6z9 3 ablibs/base.so ablibs/prio.so
