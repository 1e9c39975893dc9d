#!/bin/bash
# r5 GPU session 30: rehearsal of the driver's multi-rank bench command on the 1-GPU box (two ranks on cuda:0, gloo
# instead of RCCL): the N > 1 path end to end, one compact line from rank 0
source tools/gpu_session_lib.sh
step bench_2rank 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --same-device || exit 1
grep '"metric"' gpurun_out/bench_2rank.txt | tail -1 > gpurun_out/bench_line_2rank.json
