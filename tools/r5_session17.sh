#!/bin/bash
# r5 GPU session 17: the inverse K = 5 top tile as generated asm (untwist + GS stages) and the persistent external-product
# launches (MI_EXT_PERSIST=1, A/B): transform / large / external-product parity, the 3_3 / 4_4 legs, the config-3 leg
# off / on / off / on
source tools/gpu_session_lib.sh
step pytest_ntt 600 python -u -m pytest tests/test_ntt_gpu.py tests/test_pbs_large_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
step pytest_ext 600 env MI_EXT_PERSIST=1 python -u -m pytest tests/test_pbs_gpu.py -q -m gpu -x -k "ext or cmux or external" --timeout 300 --timeout-method thread || exit 1
step shapes_a 300 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step shapes_b 300 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step ext0 200 python -u tools/ext_probe.py || exit 1
step ext1 200 env MI_EXT_PERSIST=1 python -u tools/ext_probe.py || exit 1
step ext0b 200 python -u tools/ext_probe.py || exit 1
step ext1b 200 env MI_EXT_PERSIST=1 python -u tools/ext_probe.py || exit 1
