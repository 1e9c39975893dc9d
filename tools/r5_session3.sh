#!/bin/bash
# r5 GPU session 3: the SALU-cost probe (variant_probe: r4 bodies, + independent SALU, + EXEC writes, EXEC-masked
# bodies), the full GPU suite (KS32, Solinas full batch, large N 32768 / 131072), the driver's bench command, smoke.
source tools/gpu_session_lib.sh
step variant_probe 240 ./tools/variant_probe || exit 1
step pytest_gpu 1500 python -u -m pytest tests -q -m gpu --timeout 600 --timeout-method thread
rc=$?
# test failures (rc 1) are read afterwards; a time limit, abort or fault ends the session here
[ $rc -le 1 ] || exit $rc
step bench_default 600 python -u bench.py || exit 1
tail -1 gpurun_out/bench_default.txt > gpurun_out/bench_line.json
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
exit $rc
