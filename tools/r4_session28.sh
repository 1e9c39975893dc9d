#!/bin/bash
# r4 GPU session 28: the final tree (f64 4_4 back to two lanes): full GPU suite and smoke.
source tools/gpu_session_lib.sh
step pytest_gpu 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step shapes_fft 300 python3 -u tools/shape_probe.py --fft message_3_carry_3 message_4_carry_4 || exit 1
