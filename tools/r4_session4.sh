#!/bin/bash
# r4 GPU session 4: the whole GPU suite + C++ mirrors on the current tree, the occupancy probe of the transform bodies,
# a kernel trace of the large-N PBS shapes, and the default bench line.
source tools/gpu_session_lib.sh
step pytest_gpu 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step cpp_core 300 tests/cpp/test_core_crypto || exit 1
step cpp_prime64 200 tests/cpp/test_prime64 || exit 1
step occupancy 300 tools/occupancy_probe 8192 || exit 1
step shape_trace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/shape_trace -o run -- python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step bench 400 python -u bench.py || exit 1
