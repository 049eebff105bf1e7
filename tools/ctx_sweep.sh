#!/usr/bin/env bash
# Long-context decode sweep: Llama-3.1-8B (synthetic Q4_K_M, 128K context) at prompt lengths x batch x
# KV dtype, one bench.py line each (JSONL) -> gpurun_out/ctx_sweep.jsonl
#   CTXS="8192 16384 32768" BATCHES="1 16" KVS="bf16 fp8" bash tools/ctx_sweep.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/ctx_sweep.jsonl
for P in ${CTXS:-8192 16384 32768}; do
  for B in ${BATCHES:-1 16}; do
    for KV in ${KVS:-bf16 fp8}; do
      NLS_KV_DTYPE=$KV timeout -k 10 ${STEP_TIMEOUT:-300} python -u bench.py --model llama-3.1-8b --concurrency $B \
        --prompt-len $P --steps ${STEPS:-50} --warmup 5 --serve-load 0 --no-rtt --tp-leg 0 > gpurun_out/ctx_${P}_${B}_${KV}.log 2>&1
      rc=$?
      line=$(grep '^{' gpurun_out/ctx_${P}_${B}_${KV}.log | tail -1)
      [ $rc -ne 0 ] && { echo "ctx=$P B=$B kv=$KV rc=$rc"; tail -5 gpurun_out/ctx_${P}_${B}_${KV}.log; exit $rc; }
      echo "{\"kv\": \"$KV\", \"ctx\": $P, \"batch\": $B, \"bench\": $line}" >> $out
      echo "ctx=$P B=$B kv=$KV $(echo "$line" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "tok/s", d["ms_per_step"], "ms/step")')"
    done
  done
done
