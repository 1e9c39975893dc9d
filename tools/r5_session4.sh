#!/bin/bash
# r5 GPU session 4: EXEC-masked bodies scheduled with a VALU -> SALU mask latency of 6 / 12 / 20 slots vs the r4 bodies
source tools/gpu_session_lib.sh
step variant_probe_lat 240 ./tools/variant_probe || exit 1
