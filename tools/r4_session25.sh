#!/bin/bash
# r4 GPU session 25: level-1 shape kernels (pbs_kernels.hip) at 2 waves per SIMD: shape / PBS / ext-product parity,
# 1_1 NTT shape probe.
source tools/gpu_session_lib.sh
step pytest_shapes 900 python -u -m pytest tests/test_pbs_shapes_gpu.py tests/test_pbs_gpu.py tests/test_blind_rotate_gpu.py tests/test_ntt_tw_shapes_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step shapes 300 python3 -u tools/shape_probe.py message_1_carry_1 message_3_carry_3 message_4_carry_4 || exit 1
step shapes2 300 python3 -u tools/shape_probe.py message_1_carry_1 || exit 1
