#!/bin/bash
# r5 GPU session 5: kernel-level breakdown of the multi-kernel NTT blind rotation at 3_3 and 4_4 (shape probe under
# rocprofv3 --kernel-trace --stats)
source tools/gpu_session_lib.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step shape_trace 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shape_trace -o run -- python3 -u tools/shape_probe.py message_3_carry_3 message_4_carry_4 || exit 1
