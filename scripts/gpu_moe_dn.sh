#!/usr/bin/env bash
# Mixtral batch-1 / batch-4: sweep of the MoE decode down-projection GEMV config (NLS_MOE_GEMV_DN).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for c in "" 0,8,1,1 0,8,2,1 0,4,1,1 0,4,2,1 0,8,1,1; do
  NLS_MOE_GEMV_DN=$c timeout -k 10 420 python -u bench.py --no-rtt --serve-load 0 --model mixtral-8x7b \
      --ftype Q5_K_M --concurrency 1 --steps 100 --warmup 10 > gpurun_out/mix_dn.log 2>&1 || { tail -5 gpurun_out/mix_dn.log; exit 1; }
  echo "DN=${c:-default} $(tail -1 gpurun_out/mix_dn.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
