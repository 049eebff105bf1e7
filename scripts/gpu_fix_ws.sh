#!/usr/bin/env bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # tag concurrency prompt steps
  timeout -k 10 300 python -u bench.py --concurrency $2 --prompt-len $3 --steps $4 --warmup 10 --no-rtt \
      --serve-load 0 > gpurun_out/fx_$1.log 2>&1
  local rc=$?
  echo "$1 rc=$rc $(tail -1 gpurun_out/fx_$1.log | python3 -c 'import json,sys
try:
    d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])
except Exception: print("no json")')"
  return $rc
}
run b256_p1024 256 1024 100 && run b64_p1024 64 1024 100 && run b1_p4096 1 4096 100 && run b16_p4096 16 4096 100 \
  && run b512_p128 512 128 100 && run b1_p128 1 128 200 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
    -k "attention" tests/test_model_gpu.py tests/test_production_gpu.py > gpurun_out/fx_tests.log 2>&1 || { tail -20 gpurun_out/fx_tests.log; exit 1; }
tail -1 gpurun_out/fx_tests.log
