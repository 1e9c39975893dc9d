#!/bin/bash
# r5 GPU session 39 (final build): the default bench run (no flags) for the record beside the driver's command
source tools/gpu_session_lib.sh
O=gpurun_out/r5final5
mkdir -p $O
step bench_default 400 python -u bench.py || exit 1
grep '"metric"' gpurun_out/bench_default.txt | tail -1 > $O/bench_line.json
