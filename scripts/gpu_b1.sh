#!/bin/bash
# GPU tests + B=1 bench + B=1 rocprof breakdown + B=512 bench (one gpurun call)
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log
case $rc in 0|1) ;; *) echo "tests fatal rc=$rc"; exit $rc;; esac
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; exit 1; }
timeout -k 10 300 python -u bench.py --concurrency 1 --steps 200 --warmup 10 --no-rtt > gpurun_out/bench_b1.log 2>&1 || exit $?
tail -1 gpurun_out/bench_b1.log
BS=1 bash tools/gpu_prof.sh > gpurun_out/prof.log 2>&1 || { tail -5 gpurun_out/prof.log; exit 1; }
head -16 gpurun_out/prof_b1_breakdown.txt
timeout -k 10 400 python -u bench.py --steps 100 --warmup 10 > gpurun_out/bench_b512.log 2>&1 || exit $?
tail -1 gpurun_out/bench_b512.log
