#!/bin/bash
# r5 GPU session 7: the forward scale plan in the library (tools/tw_scale_plan.py, SCALE_PLAN): the full GPU suite,
# the driver's bench command, smoke, then the rocprofv3 kernel trace of a 3,000-step bench (the headline's launches)
source tools/gpu_session_lib.sh
step pytest_gpu 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
rc=$?
[ $rc -le 1 ] || exit $rc
step bench_default 300 python -u bench.py || exit 1
tail -1 gpurun_out/bench_default.txt > gpurun_out/bench_line.json
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_trace -o run -- python3 -u bench.py --steps 3000 || exit 1
exit $rc
