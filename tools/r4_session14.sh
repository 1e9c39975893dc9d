#!/bin/bash
# r4 GPU session 14: the default bench line (two-stream key conversion added), then the kernel trace of a 3,000-step
# bench run (the headline's timed launches against its own line).
source tools/gpu_session_lib.sh
step bench 400 python -u bench.py || exit 1
step trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace14 -o run -- python3 -u bench.py --steps 3000 --warmup 200 --no-cpu-baseline || exit 1
