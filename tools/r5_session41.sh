#!/bin/bash
# r5 GPU session 41: N = 512, k = 4 level-1 PBS with the MAC's key loads one column at a time (a scheduling barrier:
# 248 VGPRs, no spill, against 256 + 18 spilled; MI_SHAPE_SB=1): shape / blind-rotation parity under it, then the
# 1_1 leg A/B
source tools/gpu_session_lib.sh
step pytest_sb 900 env MI_SHAPE_SB=1 python -u -m pytest tests/test_pbs_shapes_gpu.py tests/test_blind_rotate_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
step sb0_a 300 env MI_SHAPE_SB=0 python -u tools/shape_probe.py message_1_carry_1 || exit 1
step sb1_a 300 env MI_SHAPE_SB=1 python -u tools/shape_probe.py message_1_carry_1 || exit 1
step sb0_b 300 env MI_SHAPE_SB=0 python -u tools/shape_probe.py message_1_carry_1 || exit 1
step sb1_b 300 env MI_SHAPE_SB=1 python -u tools/shape_probe.py message_1_carry_1 || exit 1
