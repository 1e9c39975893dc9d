#!/bin/bash
# r5 GPU session 32: the wave-specialised MAC-fused inverse, second form (MI_PBS_WS = two-wave workgroups per CU; the
# producer writes each row to LDS as it is reduced and streams its terms through a 26-deep ring, the consumer's
# transposes have their own region): large-N / shape parity under it, then the 3_3 / 4_4 legs A/B
source tools/gpu_session_lib.sh
step pytest_ws 900 env MI_PBS_WS=6 python -u -m pytest tests/test_pbs_large_gpu.py tests/test_pbs_shapes_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
step ws0_a 300 env MI_PBS_WS=0 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step ws6_a 300 env MI_PBS_WS=6 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step ws4_a 300 env MI_PBS_WS=4 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step ws0_b 300 env MI_PBS_WS=0 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step ws6_b 300 env MI_PBS_WS=6 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
