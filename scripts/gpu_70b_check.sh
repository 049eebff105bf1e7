#!/usr/bin/env bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for c in 256 512; do
  timeout -k 10 420 python -u bench.py --no-rtt --serve-load 0 --steps 40 --warmup 5 --model llama-3-70b --concurrency $c \
      > gpurun_out/l70c.log 2>&1 || { tail -5 gpurun_out/l70c.log; exit 1; }
  echo "l70 B=$c $(tail -1 gpurun_out/l70c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
