#!/bin/bash
# r4 GPU session 21: one-launch split transform for plain transforms only (the blind rotation back on its separate
# kernels): full GPU suite, split probe, 3_3 / 4_4 shapes.
source tools/gpu_session_lib.sh
step pytest_gpu 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step split_fused 300 python3 -u tools/split_probe.py 20 || exit 1
step shapes 300 python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
