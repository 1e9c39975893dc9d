#!/bin/bash
# r4 GPU session 13: shift twiddles in the register-window engine's compile-time windows (Solinas plans): GPU suite,
# the shape legs (1_1 / 3_3 / 4_4, NTT and f64), the default bench line.
source tools/gpu_session_lib.sh
step pytest_gpu 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step shapes 600 python3 -u tools/shape_probe.py message_1_carry_1 message_3_carry_3 message_4_carry_4 || exit 1
step bench 400 python -u bench.py || exit 1
