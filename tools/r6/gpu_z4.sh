# rowln ablations (K-loop only / no MFMAs) and the text-form A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_GREP=rowln bash tools/r6/ab.sh r6z4 1 ablibs/rlbase.so ablibs/rlprobe1.so ablibs/rlprobe2.so
bash tools/r6/gpu_z3.sh
