#!/usr/bin/env bash
# fp8 (OCP e4m3) paged KV cache: kernel + model tests, then bf16 vs fp8 decode throughput.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
    -k "rope_kv or attention" tests/test_model_gpu.py > gpurun_out/kv8_tests.log 2>&1 || { tail -30 gpurun_out/kv8_tests.log; exit 1; }
tail -2 gpurun_out/kv8_tests.log
run() {  # tag kvdtype concurrency prompt
  NLS_KV_DTYPE=$2 timeout -k 10 420 python -u bench.py --no-rtt --serve-load 0 --concurrency $3 --prompt-len $4 \
      --steps 100 --warmup 10 > gpurun_out/kv8_$1.log 2>&1 || { tail -5 gpurun_out/kv8_$1.log; exit 1; }
  echo "$1 $(tail -1 gpurun_out/kv8_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
run b512_p128_bf16 bf16 512 128
run b512_p128_fp8 fp8 512 128
run b16_p4096_bf16 bf16 16 4096
run b16_p4096_fp8 fp8 16 4096
run b1_p4096_bf16 bf16 1 4096
run b1_p4096_fp8 fp8 1 4096
