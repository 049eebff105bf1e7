#!/usr/bin/env bash
# One GPU-box validation pass (used through gpurun): GPU tests, smoke, headline bench.
# Every GPU step has its own time limit; a crash / abort / timeout stops the script (test
# failures, exit 1, do not: the bench still runs so a single failing case does not hide perf).
#   tools/gpu_check.sh [tests|smoke|bench|all] [extra bench args...]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
WHAT=${1:-all}
shift || true
export HSA_ENABLE_IPC_MODE_LEGACY=0

fatal() {  # exit statuses that mean the GPU step crashed or hung
  case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac
}

if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread \
      > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -5 gpurun_out/gpu_tests.log
  if fatal $rc; then echo "gpu tests: fatal rc=$rc"; exit $rc; fi
fi
if [ "$WHAT" = all ] || [ "$WHAT" = smoke ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?
  tail -2 gpurun_out/smoke.log
  if [ $rc -ne 0 ]; then echo "smoke: rc=$rc"; exit $rc; fi
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench.log 2>&1
  rc=$?
  tail -3 gpurun_out/bench.log
  exit $rc
fi
