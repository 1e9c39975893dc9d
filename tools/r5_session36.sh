#!/bin/bash
# r5 GPU session 36 (final build): the rocprofv3 kernel trace of a 3,000-step bench (summarised on the box, the raw
# trace deleted: it exceeds the copy-back limit) and the headline's PMC passes on tools/headline_loop (no python under
# --pmc)
source tools/gpu_session_lib.sh
O=gpurun_out/r5final5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 -u bench.py --steps 3000 || exit 1
grep "\"metric\"" gpurun_out/trace.txt | tail -1 > $O/bench_line_under_rocprof.json
python3 tools/summarize_rocpd.py $O/trace/run_kernel_trace.csv $O/trace_sum $O/bench_line_under_rocprof.json > $O/trace_sum.txt 2>&1
rm -f $O/trace/run_kernel_trace.csv
P="--output-format csv -o run -- tools/headline_loop 20"
step pmc_sq 120 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU -d $O/pmc_sq $P || exit 1
step pmc_lds 120 timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $O/pmc_lds $P || exit 1
step pmc_fetch 120 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch $P || exit 1
step pmc_write 120 timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write $P || exit 1
