#!/bin/bash
# r5 GPU session 11: stream-lane count of the large-N blind rotation (MI_PBS_LANES 1..4) with the MAC-fused inverse on
# and off, 3_3 / 4_4 legs
source tools/gpu_session_lib.sh
for lanes in 1 2 3 4; do
  step shapes_l${lanes}_mac1 300 env MI_PBS_LANES=$lanes python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
  step shapes_l${lanes}_mac0 300 env MI_PBS_LANES=$lanes MI_PBS_MAC_FUSED=0 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
done
