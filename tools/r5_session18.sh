#!/bin/bash
# r5 GPU session 18: one-box A/B of the K = 5 tile asm (rotation pass forward + accumulating inverse top tile) against
# the compiled stages (MI_TILE_ASM=0), 3_3 / 4_4 legs alternated
source tools/gpu_session_lib.sh
step pytest_large 600 python -u -m pytest tests/test_pbs_large_gpu.py -q -m gpu -x -k "65536 or two_lanes" --timeout 300 --timeout-method thread || exit 1
for r in a b c; do
  step shapes_asm0_$r 300 env MI_TILE_ASM=0 python -u tools/shape_probe.py message_4_carry_4 message_3_carry_3 || exit 1
  step shapes_asm1_$r 300 python -u tools/shape_probe.py message_4_carry_4 message_3_carry_3 || exit 1
done
