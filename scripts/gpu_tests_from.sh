#!/bin/bash
# GPU tests of the given files/selection only (pytest args pass through)
set -u
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -q -x --timeout 120 --timeout-method thread "$@" > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
exit $rc
