#!/bin/bash
# r4 GPU session 18: non-temporal digit stores in the fused rotation + decomposition passes and the gather ordered after the caller stream: GPU suite,
# shape trace.
source tools/gpu_session_lib.sh
step pytest_gpu 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step shapes 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shape_trace18 -o run -- python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
