#!/bin/bash
# r5 GPU session 10: the MAC-fused inverse at 168 VGPRs (a 21-term load ring, 3 waves per SIMD): large parity, the
# 3_3 / 4_4 legs with the fused MAC off and on, a kernel trace of the shape legs
source tools/gpu_session_lib.sh
step pytest_large 900 python -u -m pytest tests/test_pbs_large_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
step shapes_mac0 300 env MI_PBS_MAC_FUSED=0 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step shapes_mac1 300 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step shapes_mac0b 300 env MI_PBS_MAC_FUSED=0 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step shapes_mac1b 300 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step shape_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shape_trace10 -o run -- python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
rm -f gpurun_out/shape_trace10/run_kernel_trace.csv
