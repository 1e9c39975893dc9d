#!/bin/bash
# step <name> <seconds> <cmd...>: one GPU step under its own time limit, output to gpurun_out/<name>.txt (unbuffered,
# so the silence watchdog sees progress), the exit status returned so a session can stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {
  local name=$1 secs=$2
  shift 2
  echo "=== $name ($(date +%T))" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.txt" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(date +%T))" | tee -a gpurun_out/session.log
  tail -3 "gpurun_out/$name.txt"
  return $rc
}
