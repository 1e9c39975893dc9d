#!/bin/bash
# r5 GPU session 15: the K = 2 rotation pass with its block-twist values loaded once for all levels: large / shape
# parity, the 3_3 / 4_4 legs twice, their kernel trace
source tools/gpu_session_lib.sh
step pytest_large 900 python -u -m pytest tests/test_pbs_large_gpu.py tests/test_pbs_shapes_gpu.py tests/test_blind_rotate_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
step shapes_a 300 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step shapes_b 300 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step shape_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shape_trace15 -o run -- python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
rm -f gpurun_out/shape_trace15/run_kernel_trace.csv
