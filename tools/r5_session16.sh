#!/bin/bash
# r5 GPU session 16: persistent external-product launches (MI_EXT_PERSIST=1: <= 4 two-wave workgroups per CU looping
# over items): external-product / CMUX parity with it on, then the config-3 leg off / on / off / on
source tools/gpu_session_lib.sh
step pytest_ext 600 env MI_EXT_PERSIST=1 python -u -m pytest tests/test_pbs_gpu.py -q -m gpu -x -k "ext or cmux or external" --timeout 300 --timeout-method thread || exit 1
step ext0 200 python -u tools/ext_probe.py || exit 1
step ext1 200 env MI_EXT_PERSIST=1 python -u tools/ext_probe.py || exit 1
step ext0b 200 python -u tools/ext_probe.py || exit 1
step ext1b 200 env MI_EXT_PERSIST=1 python -u tools/ext_probe.py || exit 1
