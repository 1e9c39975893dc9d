#!/bin/bash
# r4 GPU session 22: the large-N blind rotation on two stream lanes: large / shape PBS parity, shape probe A/B
# (MI_PBS_LANES=1: one lane), kernel trace of the two-lane run.
source tools/gpu_session_lib.sh
step pytest_large 600 python -u -m pytest tests/test_pbs_large_gpu.py tests/test_pbs_shapes_gpu.py tests/test_blind_rotate_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step shapes_lanes 300 python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
MI_PBS_LANES=1 step shapes_one 300 python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step shapes_lanes2 300 python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step shape_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shape_trace22 -o run -- python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
