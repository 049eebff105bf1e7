#!/usr/bin/env bash
# End-of-session validation: full GPU suite, smoke, default bench, batch-1 bench, prefill o/down A/B.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_check.sh all || exit $?
timeout -k 10 300 python -u bench.py --concurrency 1 --steps 200 --warmup 10 --no-rtt --serve-load 0 \
    > gpurun_out/bench_b1.log 2>&1 || exit $?
tail -1 gpurun_out/bench_b1.log | cut -c1-300
timeout -k 10 300 python -u tools/blaslt_ab.py --M 2048 --shapes o,down > gpurun_out/blaslt_ab_2048.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/blaslt_ab_2048.txt
# flash-decoding split cap at long context (batch 1 / 16, 4K-token prompts)
for c in 32 16 8 64; do
  for b in 1 16; do
    NLS_ATTN_SPLIT_CAP=$c timeout -k 10 300 python -u bench.py --concurrency $b --prompt-len 4096 --steps 100 \
        --warmup 10 --no-rtt --serve-load 0 > gpurun_out/cap.log 2>&1 || exit $?
    echo "cap=$c B=$b $(tail -1 gpurun_out/cap.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
