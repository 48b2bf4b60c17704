# wave occupancy of fenc_row0 with 112-B (51.7 KB LDS) vs 160-B (65.8 KB) residual rows: SQ_WAVES, SQ_WAVE_CYCLES,
# SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE per dispatch (one PMC pass per library)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/occ_a -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/occ_a.log 2>&1 || { tail -5 gpurun_out/occ_a.log; exit 1; }
ATHD_LIB=$(realpath ablibs/libathd_x80.so) timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/occ_b -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/occ_b.log 2>&1 || { tail -5 gpurun_out/occ_b.log; exit 1; }
ls gpurun_out/occ_a gpurun_out/occ_b
