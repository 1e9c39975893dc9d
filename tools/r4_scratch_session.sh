#!/bin/bash
# r4 GPU session: the r3 stale-scratch failure reproduced with the pre-fix library (ab/oldlib: the tree of commit
# a3e1113^ built unchanged) and isolated with tools/scratch_order_probe (each ingredient switched on its own), a
# runtime log and a rocprofv3 kernel + copy + HIP API trace of one failing run; then the current library's C++ mirror
# (null and created streams, plain and serialised) and the GPU test suite.
source tools/gpu_session_lib.sh
SER="AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3"
step old_probe_plain 120 ab/oldlib/fftg_rt_probe_old 1024 12 || exit 1
step old_probe_serial 120 env $SER ab/oldlib/fftg_rt_probe_old 1024 12 || exit 1
step old_probe_serial_8192 120 env $SER ab/oldlib/fftg_rt_probe_old 8192 6 || exit 1
step standalone_plain 180 tools/scratch_order_probe 512 20 0 1 2 3 4 5 6 7 8 9 10 11 || exit 1
step standalone_serial 180 env $SER tools/scratch_order_probe 512 20 0 1 2 3 4 5 6 7 8 9 10 11 || exit 1
step old_log 120 env $SER AMD_LOG_LEVEL=3 ab/oldlib/fftg_rt_probe_old 1024 3 || exit 1
step old_trace 240 env $SER rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d gpurun_out/old_trace -o run -- ab/oldlib/fftg_rt_probe_old 1024 3 || exit 1
step new_probe_serial 120 env $SER tools/fftg_rt_probe 1024 12 || exit 1
step new_probe_serial_8192 120 env $SER tools/fftg_rt_probe 8192 6 || exit 1
step cpp_core_plain 300 tests/cpp/test_core_crypto || exit 1
step cpp_core_serial 400 env $SER tests/cpp/test_core_crypto || exit 1
step cpp_prime64 200 tests/cpp/test_prime64 || exit 1
step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread || exit 1
