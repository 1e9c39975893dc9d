#!/bin/bash
# r5 GPU session 29: config-3 external products on the persistent grid with a staggered start (MI_EXT_PERSIST=1,
# MI_EXT_STAGGER), parity under the staggered form first, then the A/B
source tools/gpu_session_lib.sh
step pytest_ext 600 env MI_EXT_PERSIST=1 MI_EXT_STAGGER=4 python -u -m pytest tests/test_pbs_gpu.py -q -m gpu -x -k "external_product or cmux or indexed" --timeout 300 --timeout-method thread || exit 1
step base_a 300 python -u tools/ext_probe.py || exit 1
step persist_a 300 env MI_EXT_PERSIST=1 python -u tools/ext_probe.py || exit 1
step st2 300 env MI_EXT_PERSIST=1 MI_EXT_STAGGER=2 python -u tools/ext_probe.py || exit 1
step st4 300 env MI_EXT_PERSIST=1 MI_EXT_STAGGER=4 python -u tools/ext_probe.py || exit 1
step st8 300 env MI_EXT_PERSIST=1 MI_EXT_STAGGER=8 python -u tools/ext_probe.py || exit 1
step base_b 300 python -u tools/ext_probe.py || exit 1
