#!/bin/bash
# r5 GPU session 42 (final build: + the 1_1 MAC one key column at a time): the full
# GPU suite, the driver's bench command and smoke
source tools/gpu_session_lib.sh
O=gpurun_out/r5final6
mkdir -p $O
step pytest_gpu 700 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
rc=$?
[ $rc -le 1 ] || exit $rc
step bench_driver_cmd 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
grep '"metric"' gpurun_out/bench_driver_cmd.txt | tail -1 > $O/bench_line_driver_cmd.json
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
exit $rc
