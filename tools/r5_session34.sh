#!/bin/bash
# r5 GPU session 34: the K <= 3 rotation pass (large_rotdec_top, 3_3's K = 2) with lazy top stages before the block
# twist (MI_ROTDEC_LAZY, default on): large-N / shape parity, then the 3_3 leg A/B
source tools/gpu_session_lib.sh
step pytest_lazy 900 python -u -m pytest tests/test_pbs_large_gpu.py tests/test_pbs_shapes_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
step lazy0_a 300 env MI_ROTDEC_LAZY=0 python -u tools/shape_probe.py message_3_carry_3 || exit 1
step lazy1_a 300 env MI_ROTDEC_LAZY=1 python -u tools/shape_probe.py message_3_carry_3 || exit 1
step lazy0_b 300 env MI_ROTDEC_LAZY=0 python -u tools/shape_probe.py message_3_carry_3 || exit 1
step lazy1_b 300 env MI_ROTDEC_LAZY=1 python -u tools/shape_probe.py message_3_carry_3 || exit 1
