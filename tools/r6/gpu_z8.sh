# attention: first tile's scores shifted by the max in registers (ATHD_ATTN_T0SUB=1) against QK^T recomputed
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r6/same_env.py "ATHD_LIB=$PWD/ablibs/base.so" "ATHD_LIB=$PWD/ablibs/t0sub.so" 2>&1 | grep -v amdgpu.ids
AB_GREP=attn32 bash tools/r6/ab.sh r6z8 3 ablibs/base.so ablibs/t0sub.so
