#!/bin/bash
# r4 GPU session 27: per-N default lane counts of the f64 engine (4 at N 8192, 3 at N >= 65536): f64 generic parity,
# smoke, the driver's bench command.
source tools/gpu_session_lib.sh
step pytest_fftg 600 python -u -m pytest tests/test_fft_generic_gpu.py tests/test_fft_blind_rotate_gpu.py tests/test_pbs_large_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 400 python -u bench.py || exit 1
