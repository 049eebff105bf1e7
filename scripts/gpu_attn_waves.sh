#!/usr/bin/env bash
# Decode attention: in-wave shuffle merge (both) and 4 vs 8 waves per workgroup.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for w in 4 8; do
  NLS_ATTN_WAVES=$w timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_kernels_gpu.py -k "attention_paged" > gpurun_out/attn_w$w.log 2>&1 || { tail -20 gpurun_out/attn_w$w.log; exit 1; }
  echo "waves=$w $(tail -1 gpurun_out/attn_w$w.log)"
done
run() {  # tag waves kv concurrency prompt
  NLS_ATTN_WAVES=$2 NLS_KV_DTYPE=$3 timeout -k 10 300 python -u bench.py --concurrency $4 --prompt-len $5 --steps 100 \
      --warmup 10 --no-rtt --serve-load 0 > gpurun_out/aw.log 2>&1 || { tail -5 gpurun_out/aw.log; exit 1; }
  echo "$1 $(tail -1 gpurun_out/aw.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for w in 4 8; do
  run "w$w b1 p4096 bf16" $w bf16 1 4096
  run "w$w b1 p4096 fp8" $w fp8 1 4096
  run "w$w b16 p4096 bf16" $w bf16 16 4096
  run "w$w b512 p128 bf16" $w bf16 512 128
  run "w$w b1 p128 bf16" $w bf16 1 128
done
