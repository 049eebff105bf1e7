#!/usr/bin/env bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_production_gpu.py \
    -k "lib_gemm" > gpurun_out/lib_prod_tests.log 2>&1 || { tail -20 gpurun_out/lib_prod_tests.log; exit 1; }
tail -2 gpurun_out/lib_prod_tests.log
run() {  # tag concurrency
  timeout -k 10 420 python -u bench.py --no-rtt --serve-load 0 --model llama-3-70b --ftype Q4_K_M \
      --concurrency $2 --steps 20 --warmup 3 > gpurun_out/l70_$1.log 2>&1
  local rc=$?
  echo "$1 rc=$rc $(tail -1 gpurun_out/l70_$1.log | cut -c1-260)"
  [ $rc -eq 0 ] || exit $rc
}
run b128_auto60 128
run b512_auto60 512
