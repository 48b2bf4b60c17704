set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for L in libkbench.so libkbench_poly4.so libkbench_poly8.so; do
  echo "== $L"
  ATTN_VARIANTS=0 KB_LIB=$L timeout -k 10 300 python tools/kbench.py attn 2>&1 | grep -v amdgpu.ids || exit 1
done
for lv in 1 0; do
  FR_LEVEL=$lv ATHD_LIB=$(realpath ablibs/libathd_frstamp.so) timeout -k 10 300 python tools/fr_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
done
