#!/bin/bash
# r5 GPU session 1: the driver's default bench command (compact final line) and smoke on HEAD's library.
source tools/gpu_session_lib.sh
step bench_default 600 python -u bench.py || exit 1
tail -c 5000 gpurun_out/bench_default.txt | tail -1 > gpurun_out/bench_line.json
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
