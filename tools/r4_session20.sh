#!/bin/bash
# r4 GPU session 20: the split transform of N = 2^12 ... 2^14 in one launch (top stages + bodies per workgroup):
# transform and large-PBS parity, A/B of the split probe (MI_SPLIT_FUSED=0: two launches), 3_3 / 4_4 shapes.
source tools/gpu_session_lib.sh
step pytest_split 600 python -u -m pytest tests/test_ntt_gpu.py tests/test_pbs_large_gpu.py tests/test_blind_rotate_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread || exit 1
step split_fused 300 python3 -u tools/split_probe.py 20 || exit 1
MI_SPLIT_FUSED=0 step split_two 300 python3 -u tools/split_probe.py 20 || exit 1
step shapes 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shape_trace20 -o run -- python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
