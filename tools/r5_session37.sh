#!/bin/bash
# r5 GPU session 37: config-3 external products touching the rows of the item that runs on their slot next
# (MI_EXT_PREFETCH = items ahead): external-product parity under it, then the A/B
source tools/gpu_session_lib.sh
step pytest_pf 600 env MI_EXT_PREFETCH=1024 python -u -m pytest tests/test_pbs_gpu.py -q -m gpu -x -k "external_product or cmux or indexed" --timeout 300 --timeout-method thread || exit 1
step pf0_a 300 env MI_EXT_PREFETCH=0 python -u tools/ext_probe.py || exit 1
step pf1024_a 300 env MI_EXT_PREFETCH=1024 python -u tools/ext_probe.py || exit 1
step pf2048_a 300 env MI_EXT_PREFETCH=2048 python -u tools/ext_probe.py || exit 1
step pf512_a 300 env MI_EXT_PREFETCH=512 python -u tools/ext_probe.py || exit 1
step pf0_b 300 env MI_EXT_PREFETCH=0 python -u tools/ext_probe.py || exit 1
step pf1024_b 300 env MI_EXT_PREFETCH=1024 python -u tools/ext_probe.py || exit 1
