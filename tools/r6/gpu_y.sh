# decoder tail parts: 3/4 + 1/4 split (ATHD_TAIL_SKEW=1) against one part
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r6/same_env.py "ATHD_TAIL_SPLIT=1" "ATHD_TAIL_SPLIT=2 ATHD_TAIL_SKEW=1" 2>&1 | grep -v amdgpu.ids
AB_GREP=istft,fdec_tail bash tools/r6/ab_env.sh r6y 3 "ATHD_TAIL_SPLIT=1" "ATHD_TAIL_SPLIT=2 ATHD_TAIL_SKEW=1"
