#!/bin/bash
# One parameterised GPU session (replaces the per-session scripts of rounds 4-5; git history keeps them):
#   bash tools/gpu_session.sh <out-dir> <step>...
# steps, run in order, each under its own time limit, the session stopping at the first failure:
#   suite    pytest -m gpu (whole GPU suite)          bench    the driver's command (bench.py --gpus 1 --steps 20 --warmup 5)
#   smoke    __graft_entry__.smoke()                  trace    rocprofv3 kernel trace + stats of the driver's command
#   probe    tools/variant_probe 8192 (body A/B)      test=<pytest node or -k expr>  one test selection
source tools/gpu_session_lib.sh
O=$1
shift
mkdir -p "$O"
for s in "$@"; do
  case $s in
    suite) step pytest_gpu 900 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread
           rc=$?; cp gpurun_out/pytest_gpu.txt "$O/"; [ $rc -eq 0 ] || exit $rc ;;
    bench) step bench_driver_cmd 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
           cp gpurun_out/bench_full.json "$O/" 2>/dev/null; tail -1 gpurun_out/bench_driver_cmd.txt > "$O/bench_line.json" ;;
    smoke) step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1; cp gpurun_out/smoke.txt "$O/" ;;
    trace) export TMPDIR=/tmp  # the full trace stays on the box (it exceeds gpurun's 64 MiB return); the stats come back
           step trace_driver_cmd 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/mi_trace -o run -- \
             python3 -u bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
           mkdir -p "$O/trace"; cp /tmp/mi_trace/*stats*.csv "$O/trace/"
           grep '^{"metric"' gpurun_out/trace_driver_cmd.txt | tail -1 > "$O/trace/bench_line_under_rocprof.json"
           python3 tools/summarize_rocpd.py /tmp/mi_trace/run_kernel_trace.csv "$O/trace" \
             "$O/trace/bench_line_under_rocprof.json" > "$O/trace/summary.txt" 2>&1 || true ;;
    probe) step variant_probe 240 ./tools/variant_probe 8192 || exit 1; cp gpurun_out/variant_probe.txt "$O/" ;;
    test=*) step pytest_sel 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${s#test=}
            rc=$?; cp gpurun_out/pytest_sel.txt "$O/"; [ $rc -eq 0 ] || exit $rc ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
