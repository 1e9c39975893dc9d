#!/bin/bash
# r5 GPU session 25: full-occupancy looping launches (MI_PBS_WAVE_CAP=4: one generation, each wave two or three units)
# with and without a staggered start of every other round of workgroups (MI_PBS_STAGGER sleeps of ~3.7 us) in the
# MAC-fused inverse; 3_3 / 4_4, baseline (no cap) first and last
source tools/gpu_session_lib.sh
step base_a 300 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step cap4 300 env MI_PBS_WAVE_CAP=4 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
for st in 2 5 10; do
  step cap4_st$st 300 env MI_PBS_WAVE_CAP=4 MI_PBS_STAGGER=$st python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
done
step base_b 300 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
