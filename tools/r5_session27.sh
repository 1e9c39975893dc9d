#!/bin/bash
# r5 GPU session 27: N = 512, k = 4 at level 1 as one wave per ciphertext with eight coefficients per lane (the
# column-wise MAC / inverse / accumulate, pbs_kernels.hip WIDE): shape / blind-rotation parity (both forms), then
# the 1_1 leg A/B by MI_SHAPE_WIDE, twice
source tools/gpu_session_lib.sh
step pytest_shapes 900 python -u -m pytest tests/test_pbs_shapes_gpu.py tests/test_blind_rotate_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
step wide_a 300 env MI_SHAPE_WIDE=1 python -u tools/shape_probe.py message_1_carry_1 || exit 1
step narrow_a 300 env MI_SHAPE_WIDE=0 python -u tools/shape_probe.py message_1_carry_1 || exit 1
step wide_b 300 env MI_SHAPE_WIDE=1 python -u tools/shape_probe.py message_1_carry_1 || exit 1
step narrow_b 300 env MI_SHAPE_WIDE=0 python -u tools/shape_probe.py message_1_carry_1 || exit 1
