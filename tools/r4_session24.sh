#!/bin/bash
# r4 GPU session 24: lane count sweep (MI_PBS_LANES 1-4) on both large-N engines, and the one-launch split forms inside
# the blind rotation (MI_PBS_FUSED=1) combined with lanes; parity of every variant first.
source tools/gpu_session_lib.sh
step pytest_large 600 python -u -m pytest tests/test_pbs_large_gpu.py tests/test_pbs_shapes_gpu.py tests/test_fft_generic_gpu.py tests/test_blind_rotate_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
MI_PBS_FUSED=1 step pytest_fused 600 python -u -m pytest tests/test_pbs_large_gpu.py tests/test_pbs_shapes_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
for n in 1 2 3 4; do
  MI_PBS_LANES=$n step ntt_l$n 300 python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
  MI_PBS_FUSED=1 MI_PBS_LANES=$n step ntt_fused_l$n 300 python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
  MI_PBS_LANES=$n step fft_l$n 300 python3 -u tools/shape_probe.py --fft message_1_carry_1 message_3_carry_3 message_4_carry_4 || exit 1
done
