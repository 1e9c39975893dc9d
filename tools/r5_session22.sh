#!/bin/bash
# r5 GPU session 22: clean per-kernel times of the 3_3 step (one lane, so no two kernels overlap), kernel trace
source tools/gpu_session_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step trace33 300 env MI_PBS_LANES=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace33 -o run -- python3 -u tools/shape_probe.py message_3_carry_3 || exit 1
rm -f gpurun_out/trace33/run_kernel_trace.csv
