#!/bin/bash
# r4 GPU session 7: the headline's remaining PMC passes (LDS / wait, FETCH_SIZE, WRITE_SIZE; the SQ pass ran in
# session 6), then SQ counters of the occupancy probe at 4 / 3 / 2 / 1 resident waves per SIMD (one short round).
source tools/gpu_session_lib.sh
mkdir -p gpurun_out/prof_r4
SKIP_TRACE=1 SKIP_SQ=1 step profile 900 bash tools/profile_session.sh r4 || exit 1
step occ_pmc 300 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/occ_pmc -o run -- tools/occupancy_probe 8192 200 4 1 || exit 1
step valu 200 tools/valu_probe || exit 1
