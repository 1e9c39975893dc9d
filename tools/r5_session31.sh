#!/bin/bash
# r5 GPU session 31: the wave-specialised MAC-fused inverse (MI_PBS_WS = two-wave workgroups per CU; producer wave
# forms y into LDS, consumer wave runs the inverse of the unit before): large-N / shape parity under it, then the
# 3_3 / 4_4 legs A/B
source tools/gpu_session_lib.sh
step pytest_ws 900 env MI_PBS_WS=8 python -u -m pytest tests/test_pbs_large_gpu.py tests/test_pbs_shapes_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
step ws0_a 300 env MI_PBS_WS=0 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step ws8_a 300 env MI_PBS_WS=8 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step ws4_a 300 env MI_PBS_WS=4 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step ws0_b 300 env MI_PBS_WS=0 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step ws8_b 300 env MI_PBS_WS=8 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
