#!/bin/bash
# One GPU session: every GPU step under its own time limit, chained so that the first failure
# (test failure, fault, abort or timeout) ends the session.  Output goes straight to files under
# gpurun_out/ (unbuffered) so the silence watchdog sees progress.
set -o pipefail
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name secs=$2
  name=$(echo "$1" | tr -c 'A-Za-z0-9_.=-' '_' | cut -c1-60); shift 2
  echo "=== $name ($(date +%T))" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.txt" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(date +%T))" | tee -a gpurun_out/session.log
  tail -3 "gpurun_out/$name.txt"
  return $rc
}
export PYTHONUNBUFFERED=1
n=0
for s in "$@"; do
  case $s in
    pytest) step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 240 || exit 1 ;;
    bench) step bench 300 python -u bench.py --steps 30 --warmup 5 --cpu-seconds 10 || exit 1 ;;
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    prof) step rocprof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline || exit 1 ;;
    *) n=$((n+1)); step "s${n}_$s" 600 bash -c "$s" || exit 1 ;;
  esac
done
