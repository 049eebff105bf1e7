#!/bin/bash
# Helper for multi-step GPU calls: `step NAME TIMEOUT CMD...` runs CMD under its own time limit, logs to
# gpurun_out/NAME.log, and stops the whole call after a fault-like exit (timeout / abort / segfault / kill)
# so no further GPU work starts after one (test failures are reported and the next step still runs).
mkdir -p gpurun_out
export PYTHONPATH=$PWD
STEPS_RC=0
step() {
  local name=$1 t=$2
  shift 2
  local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[step] $name rc=$rc $(( $(date +%s) - t0 ))s"
  tail -4 "gpurun_out/$name.log"
  case $rc in
    0) ;;
    124|137|134|139|143) echo "[step] $name: fault-like exit $rc, stopping"; exit $rc ;;
    *) STEPS_RC=$rc ;;
  esac
}
