#!/bin/bash
# r4 GPU session 5: GPU suite on the column-fused large-N MAC, the large-shape kernel trace, the default bench line
# (with the default-stream leg), then the headline's kernel trace + PMC passes (tools/profile_session.sh).
source tools/gpu_session_lib.sh
step pytest_gpu 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step shape_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shape_trace5 -o run -- python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step bench 400 python -u bench.py || exit 1
step profile 1100 bash tools/profile_session.sh r4 || exit 1
