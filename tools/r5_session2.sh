#!/bin/bash
# r5 GPU session 2: EXEC-masked bodies. One-process A/B of the r4 vs r5 transform bodies, then the full GPU suite,
# the driver's default bench command (compact final line) and smoke.
source tools/gpu_session_lib.sh
step variant_probe 240 ./tools/variant_probe || exit 1
step pytest_gpu 1100 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step bench_default 600 python -u bench.py || exit 1
tail -1 gpurun_out/bench_default.txt > gpurun_out/bench_line.json
cp gpurun_out/bench_full.json gpurun_out/bench_full_session2.json 2>/dev/null
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
