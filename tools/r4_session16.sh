#!/bin/bash
# r4 GPU session 16 (as 15): the MAC with a compile-time level count (large-N external product / blind rotation): GPU suite, shape probe.
source tools/gpu_session_lib.sh
step pytest_gpu 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step shapes 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shape_trace16 -o run -- python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
