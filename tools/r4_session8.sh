#!/bin/bash
# r4 GPU session 8: VALU issue costs of the DPP select forms; SQ counters of the occupancy probe; the headline's PMC
# passes on tools/headline_loop (the library's fwd/inv without python: the python bench crashed the host under --pmc).
source tools/gpu_session_lib.sh
step valu 200 tools/valu_probe || exit 1
step occ_pmc 200 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/occ_pmc -o run -- tools/occupancy_probe 8192 200 4 1 || exit 1
P="--output-format csv -o run -- tools/headline_loop 20"
step pmc_sq 120 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU -d gpurun_out/hl_pmc/pmc_sq $P || exit 1
step pmc_lds 120 timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/hl_pmc/pmc_lds $P || exit 1
step pmc_fetch 120 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/hl_pmc/pmc_fetch $P || exit 1
step pmc_write 120 timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/hl_pmc/pmc_write $P || exit 1
