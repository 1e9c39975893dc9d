#!/bin/bash
# r5 GPU session 23: the shape kernels' MAC as 128-bit column sums with one reduction (pbs::Acc128): shape / generic /
# blind-rotation / large parity, then the 1_1 / 3_3 / 4_4 legs twice
source tools/gpu_session_lib.sh
step pytest_shapes 900 python -u -m pytest tests/test_pbs_shapes_gpu.py tests/test_pbs_gpu.py tests/test_blind_rotate_gpu.py tests/test_pbs_large_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
step shapes_a 300 python -u tools/shape_probe.py message_1_carry_1 message_3_carry_3 message_4_carry_4 || exit 1
step shapes_b 300 python -u tools/shape_probe.py message_1_carry_1 message_3_carry_3 message_4_carry_4 || exit 1
