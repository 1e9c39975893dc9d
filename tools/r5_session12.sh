#!/bin/bash
# r5 GPU session 12: wave-capped (looping) body launches in the large-N blind rotation (MI_PBS_WAVE_CAP waves per SIMD):
# parity with the cap on, then 3_3 / 4_4 over cap 0..3 at two lanes, cap 1 at three and four lanes
source tools/gpu_session_lib.sh
step pytest_large_cap2 600 env MI_PBS_WAVE_CAP=2 python -u -m pytest tests/test_pbs_large_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
for cap in 0 1 2 3; do
  step shapes_cap${cap} 300 env MI_PBS_WAVE_CAP=$cap python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
done
step shapes_cap1_l3 300 env MI_PBS_WAVE_CAP=1 MI_PBS_LANES=3 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step shapes_cap1_l4 300 env MI_PBS_WAVE_CAP=1 MI_PBS_LANES=4 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step shapes_cap0b 300 env MI_PBS_WAVE_CAP=0 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
