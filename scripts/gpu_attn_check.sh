#!/usr/bin/env bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
    -k "attention" tests/test_model_gpu.py > gpurun_out/attn_pol.log 2>&1 || { tail -20 gpurun_out/attn_pol.log; exit 1; }
tail -1 gpurun_out/attn_pol.log
run() {  # tag concurrency prompt
  timeout -k 10 300 python -u bench.py --concurrency $2 --prompt-len $3 --steps 100 --warmup 10 --no-rtt \
      --serve-load 0 > gpurun_out/ap.log 2>&1 || { tail -5 gpurun_out/ap.log; exit 1; }
  echo "$1 $(tail -1 gpurun_out/ap.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
run "b1 p128" 1 128
run "b1 p4096" 1 4096
run "b16 p4096" 16 4096
run "b64 p1024" 64 1024
run "b256 p1024" 256 1024
run "b512 p128" 512 128
