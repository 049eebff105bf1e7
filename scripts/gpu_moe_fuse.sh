#!/usr/bin/env bash
# Fused MoE norm + router + route: kernel tests, model tests, Mixtral batch-1 A/B.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
    -k "moe" tests/test_model_gpu.py > gpurun_out/moe_fuse_tests.log 2>&1 || { tail -30 gpurun_out/moe_fuse_tests.log; exit 1; }
tail -2 gpurun_out/moe_fuse_tests.log
for v in 4 0 4 0; do
  NLS_MOE_NORM_ROUTE=$v timeout -k 10 420 python -u bench.py --no-rtt --serve-load 0 --model mixtral-8x7b \
      --ftype Q5_K_M --concurrency 1 --steps 100 --warmup 10 > gpurun_out/mix_b1_$v.log 2>&1 || { tail -5 gpurun_out/mix_b1_$v.log; exit 1; }
  echo "NLS_MOE_NORM_ROUTE=$v $(tail -1 gpurun_out/mix_b1_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
