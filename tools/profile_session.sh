#!/bin/bash
# rocprofv3 passes for the headline kernel (run on the GPU box).  Each pass is its own process; PMC
# passes never combine with tracing domains (gpurun policy).  The PMC passes skip the other-shape PBS legs
# (--no-shapes): rocprofv3 --pmc segfaults on the host inside the shape-generic f64 engine's launch.  Output under gpurun_out/prof_<tag>.
set -o pipefail
tag=${1:-r1}
out=gpurun_out/prof_$tag
mkdir -p $out
export PYTHONUNBUFFERED=1
run() { local name=$1; shift; echo "=== $name $(date +%T)"; timeout -k 10 300 "$@" > $out/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -2 $out/$name.log; return $rc; }
[ -n "$SKIP_TRACE" ] || run trace rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --steps ${TRACE_STEPS:-3000} --warmup 200 --no-cpu-baseline || exit 1
[ -n "$SKIP_SQ" ] || run pmc_sq rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $out/pmc_sq -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-shapes || exit 1
run pmc_lds rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_lds -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-shapes || exit 1
run pmc_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-shapes || exit 1
run pmc_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-shapes || exit 1
