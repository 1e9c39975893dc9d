#!/bin/bash
# r4 GPU session 26 (the round's final numbers): full GPU suite, smoke, the driver's bench command, and a 3000-step
# kernel trace of the bench for the roofline cross-check.
source tools/gpu_session_lib.sh
step pytest_gpu 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 400 python -u bench.py || exit 1
step trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace26 -o run -- python3 -u bench.py --steps 3000 --warmup 200 --no-cpu-baseline || exit 1
