#!/bin/bash
# r4 GPU session 6: GPU suite on the shift-twiddle stage-0 top passes and the two-coefficient MAC, the large-shape
# trace, the default bench line, then the headline PMC passes (tools/profile_session.sh, trace skipped: session 5's).
source tools/gpu_session_lib.sh
step pytest_gpu 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step shape_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shape_trace6 -o run -- python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step split_probe 300 python3 -u tools/split_probe.py || exit 1
step bench 400 python -u bench.py || exit 1
SKIP_TRACE=1 step profile 1100 bash tools/profile_session.sh r4 || exit 1
