#!/bin/bash
# r4 GPU session 10: the cooperative-tile stage-0 pass (K = 4 / 5: split transform and the large-N blind rotation):
# GPU suite, large-shape trace, split-transform probe.
source tools/gpu_session_lib.sh
step pytest_gpu 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step shape_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shape_trace10 -o run -- python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step split_probe 300 python3 -u tools/split_probe.py || exit 1
