#!/usr/bin/env bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_production_gpu.py -k "lib_gemm" \
    > gpurun_out/qw_tests.log 2>&1 || { tail -20 gpurun_out/qw_tests.log; exit 1; }
tail -1 gpurun_out/qw_tests.log
for v in 1 0; do
  NLS_LIB_GEMM=$v timeout -k 10 420 python -u bench.py --no-rtt --serve-load 0 --steps 40 --warmup 5 --model qwen2.5-7b \
      --concurrency 512 > gpurun_out/qwb.log 2>&1 || { tail -5 gpurun_out/qwb.log; exit 1; }
  echo "qwen B=512 NLS_LIB_GEMM=$v $(tail -1 gpurun_out/qwb.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
