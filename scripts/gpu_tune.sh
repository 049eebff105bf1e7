#!/usr/bin/env bash
# GEMV/GEMM kernel tests, then the launch-config sweep (writes ops/gemv_tuning.json), then the bench.
#   scripts/gpu_tune.sh [Ms (default 128,256,512,2048)] [test file filter]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
MS=${1:-128,256,512,2048}
TESTS=${2:-tests/test_kernels_gpu.py}
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -x --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { echo "tests rc=$rc"; exit $rc; }
rm -f gpurun_out/tune_gemv.log
timeout -k 10 600 python -u tools/tune_gemv.py --ms $MS > gpurun_out/tune.out 2>&1 || { echo "tune rc=$?"; tail -5 gpurun_out/tune.out; exit 1; }
cp nats_llm_studio_amd/ops/gemv_tuning.json gpurun_out/gemv_tuning.json
timeout -k 10 300 python -u bench.py --no-rtt > gpurun_out/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
