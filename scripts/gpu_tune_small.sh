#!/bin/bash
# GEMV kernel tests, re-tune the few-row GEMV table (weights streamed from HBM), then the B=1 bench
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
rm -f gpurun_out/tune_gemv.log
timeout -k 10 900 python -u tools/tune_gemv.py --ms ${MS:-1,2,4,8,16,32,48,64} > gpurun_out/tune.out 2>&1 || { echo "tune rc=$?"; tail -5 gpurun_out/tune.out; exit 1; }
cp nats_llm_studio_amd/ops/gemv_tuning.json gpurun_out/gemv_tuning.json
grep "M=  1 " gpurun_out/tune.out
timeout -k 10 300 python -u bench.py --concurrency 1 --steps 200 --warmup 10 --no-rtt > gpurun_out/bench_b1.log 2>&1 || exit $?
tail -1 gpurun_out/bench_b1.log
