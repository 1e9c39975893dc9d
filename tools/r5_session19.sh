#!/bin/bash
# r5 GPU session 19: one-box A/B of the two K = 5 tile asm blocks separately (MI_TILE_ASM bit 0: rotation pass, bit 1:
# accumulating inverse top tile), 4_4 only, rotated order, two rounds
source tools/gpu_session_lib.sh
for r in a b; do
  for m in 0 1 2 3; do
    step shapes_m${m}_$r 300 env MI_TILE_ASM=$m python -u tools/shape_probe.py message_4_carry_4 || exit 1
  done
done
