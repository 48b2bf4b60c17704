# fenc_row0 hidden-image swizzle (row >> 2) & 3: identity, A/B, LDS conflicts
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r6/same_env.py "ATHD_X=0" "ATHD_LIB=$(realpath ablibs/libathd_sw2.so)" 2>&1 | grep -v amdgpu.ids
AB_GREP=fenc_row0 bash tools/r6/ab.sh r6v 3 audio-to-sheet-music_amd/athd/libathd.so ablibs/libathd_sw2.so
O=gpurun_out/pmc_r6v; mkdir -p $O
ATHD_LIB=$(realpath ablibs/libathd_sw2.so) timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/a -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > $O/a.log 2>&1 || { tail -5 $O/a.log; exit 1; }
python tools/pmc_sq.py $O/a --top 40 > $O/sq.txt 2>&1; grep -E "kernel$|fenc_row" $O/sq.txt
