#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py --concurrency 1 --steps 64 --warmup 8 --no-rtt > gpurun_out/bench_b1.log 2>&1 || { tail -5 gpurun_out/bench_b1.log; exit 1; }
tail -1 gpurun_out/bench_b1.log
timeout -k 10 300 python -u tools/tune_gemv.py --ms 1,2,4,8,16 --out gpurun_out/gemv_tuning.json > gpurun_out/tune_small.out 2>&1 || { tail -5 gpurun_out/tune_small.out; exit 1; }
grep "M=  1" gpurun_out/tune_gemv.log
