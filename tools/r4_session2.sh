#!/bin/bash
# r4 GPU session 2: the pre-fix library's in-place reorder over many serialised reps, with the default memory pool and
# with its release threshold at UINT64_MAX ("keep": pool blocks never go back to the runtime's VM heap), one logged run;
# the current library the same way; then the default bench line.
source tools/gpu_session_lib.sh
SER="AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3"
step old_serial_default_1024 150 env $SER ab/oldlib/fftg_rt_probe_old 1024 60 || exit 1
step old_serial_keep_1024 150 env $SER ab/oldlib/fftg_rt_probe_old 1024 60 keep || exit 1
step old_serial_default_8192 150 env $SER ab/oldlib/fftg_rt_probe_old 8192 30 || exit 1
step old_serial_keep_8192 150 env $SER ab/oldlib/fftg_rt_probe_old 8192 30 keep || exit 1
step old_plain_default_8192 150 ab/oldlib/fftg_rt_probe_old 8192 60 || exit 1
step old_log_default_1024 200 env $SER AMD_LOG_LEVEL=3 ab/oldlib/fftg_rt_probe_old 1024 60 || exit 1
step new_serial_1024 150 env $SER tools/fftg_rt_probe 1024 60 || exit 1
step new_serial_8192 150 env $SER tools/fftg_rt_probe 8192 30 || exit 1
step bench 400 python -u bench.py || exit 1
