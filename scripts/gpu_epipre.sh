#!/bin/bash
# path-A epilogue operand prefetch: GPU tests, then batch-1/8 decode A/B against the previous build
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
K=$PWD/nats_llm_studio_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py > gpurun_out/epipre_tests.log 2>&1 || { tail -30 gpurun_out/epipre_tests.log; exit 1; }
tail -1 gpurun_out/epipre_tests.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 150 --warmup 10 --no-rtt --serve-load 0 $BARGS > gpurun_out/ep_$label.log 2>&1 || { tail -20 gpurun_out/ep_$label.log; exit 1; }
  echo "$label $BARGS $(tail -1 gpurun_out/ep_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for rep in 1 2; do
  for B in 1 8; do
    BARGS="--concurrency $B"
    run b${B}_base NLS_KERNELS_SO=$K/_kernels_base.so
    run b${B}_new NLS_KERNELS_SO=$K/_kernels.so
  done
done
