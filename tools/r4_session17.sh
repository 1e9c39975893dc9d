#!/bin/bash
# r4 GPU session 17: the MAC with the item's digit loads first and non-temporal digit / product traffic: GPU suite,
# smoke(), shape trace.
source tools/gpu_session_lib.sh
step pytest_gpu 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step shapes 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shape_trace17 -o run -- python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
