#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py --concurrency 1 --steps 64 --warmup 8 > gpurun_out/bench_b1.log 2>&1 || { tail -5 gpurun_out/bench_b1.log; exit 1; }
tail -1 gpurun_out/bench_b1.log | cut -c1-700
timeout -k 10 300 python -u bench.py > gpurun_out/bench_b512.log 2>&1 || { tail -5 gpurun_out/bench_b512.log; exit 1; }
tail -1 gpurun_out/bench_b512.log | cut -c1-400
