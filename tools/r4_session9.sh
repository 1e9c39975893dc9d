#!/bin/bash
# r4 GPU session 9: the DPP-select transform A/B is rejected (VALU probe); here the large-N PBS at larger batches
# (4 GiB chunk scratch): NTT and f64 engines at 3_3 / 4_4 with 1x, 2x, 4x the bench's batch.
source tools/gpu_session_lib.sh
step shapes_ntt 600 python3 -u tools/shape_probe.py 8192,1,1077,15,2,1024 8192,1,1077,15,2,2048 65536,1,1117,11,3,192 65536,1,1117,11,3,384 65536,1,1117,11,3,768 || exit 1
step shapes_fft 600 python3 -u tools/shape_probe.py --fft 8192,1,1077,15,2,1024 8192,1,1077,15,2,2048 65536,1,1117,11,3,192 65536,1,1117,11,3,384 65536,1,1117,11,3,768 || exit 1
