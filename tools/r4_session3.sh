#!/bin/bash
# r4 GPU session 3: the split transform (N = 2^12 ... 2^20 through the 2048 body): parity tests, transform timings
# against the r3 library (window kernels), and the large-N PBS shapes.
source tools/gpu_session_lib.sh
step pytest_split 900 python -u -m pytest tests/test_ntt_gpu.py tests/test_pbs_large_gpu.py tests/test_pbs_shapes_gpu.py tests/test_blind_rotate_gpu.py tests/test_pbs_gpu.py tests/test_golden.py tests/test_ntt_tw_shapes_gpu.py -x -q --timeout 300 --timeout-method thread || exit 1
step split_probe_new 300 python -u tools/split_probe.py 20 || exit 1
step split_probe_r3 300 python -u tools/split_probe.py --lib ab/oldlib/libtfhe_ntt_amd.so 20 || exit 1
step shape_probe 600 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step occupancy 300 tools/occupancy_probe 8192 || exit 1
