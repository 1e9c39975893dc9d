#!/bin/bash
# r4 GPU session 23: two stream lanes in the shape-generic f64 PBS too: f64 generic parity (incl. the two-lane
# determinism test), f64 shape probe A/B (MI_PBS_LANES=1: one lane).
source tools/gpu_session_lib.sh
step pytest_fftg 600 python -u -m pytest tests/test_fft_generic_gpu.py tests/test_fft_blind_rotate_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step fft_lanes 300 python3 -u tools/shape_probe.py --fft message_1_carry_1 message_3_carry_3 message_4_carry_4 || exit 1
MI_PBS_LANES=1 step fft_one 300 python3 -u tools/shape_probe.py --fft message_1_carry_1 message_3_carry_3 message_4_carry_4 || exit 1
step fft_lanes2 300 python3 -u tools/shape_probe.py --fft message_1_carry_1 message_3_carry_3 message_4_carry_4 || exit 1
