#!/bin/bash
# r5 GPU session 14: the generated forward top-pass asm of the large-N rotation passes (gen_tile_asm.py): large /
# shape parity, the 3_3 / 4_4 legs twice, their kernel trace; the headline's own kernel trace on tools/headline_loop
# (only the config-2 launches, so the per-kernel averages are the headline's)
source tools/gpu_session_lib.sh
step pytest_large 900 python -u -m pytest tests/test_pbs_large_gpu.py tests/test_pbs_shapes_gpu.py tests/test_blind_rotate_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
step shapes_a 300 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
step shapes_b 300 python -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step shape_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shape_trace14 -o run -- python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
rm -f gpurun_out/shape_trace14/run_kernel_trace.csv
step headline_trace 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/headline_trace -o run -- tools/headline_loop 3000 || exit 1
rm -f gpurun_out/headline_trace/run_kernel_trace.csv
