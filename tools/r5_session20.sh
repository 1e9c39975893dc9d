#!/bin/bash
# r5 GPU session 20: the inverse top tile's stages-only asm (MI_TILE_ASM bit 2, the untwist compiled beside the row
# loads): 65536 parity with it, then 4_4 at masks 1 / 5 / 1 / 5
source tools/gpu_session_lib.sh
step pytest_large 600 env MI_TILE_ASM=5 python -u -m pytest tests/test_pbs_large_gpu.py tests/test_ntt_gpu.py -q -m gpu -x -k "65536 or two_lanes or split or beyond or all_sizes" --timeout 300 --timeout-method thread || exit 1
for r in a b; do
  for m in 1 5; do
    step shapes_m${m}_$r 300 env MI_TILE_ASM=$m python -u tools/shape_probe.py message_4_carry_4 || exit 1
  done
done
