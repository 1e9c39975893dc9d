#!/bin/bash
# r5 GPU session 24: lazy forward windows in the shape kernels (ntt_regs LAZY before the Acc128 MAC): parity,
# then the 1_1 leg twice
source tools/gpu_session_lib.sh
step pytest_shapes 900 python -u -m pytest tests/test_pbs_shapes_gpu.py tests/test_pbs_gpu.py tests/test_blind_rotate_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
step shapes_a 300 python -u tools/shape_probe.py message_1_carry_1 || exit 1
step shapes_b 300 python -u tools/shape_probe.py message_1_carry_1 || exit 1
