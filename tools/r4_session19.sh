#!/bin/bash
# r4 GPU session 19: the round's final library: smoke(), the default bench line, and the kernel trace of a 3,000-step
# bench run.
source tools/gpu_session_lib.sh
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 400 python -u bench.py || exit 1
step trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace19 -o run -- python3 -u bench.py --steps 3000 --warmup 200 --no-cpu-baseline || exit 1
