#!/bin/bash
# round 5, call AM: Llama-3-70B on one GPU at B=512: the KV-aware auto policy (no f16 copies) vs forced copies.
source tools/gpu_steps.sh
step r5am_auto 900 python3 -u bench.py --model llama-3-70b --concurrency 512 --steps 10 --warmup 3 --no-rtt --serve-load 0
export NLS_DENSE_WEIGHTS=1
step r5am_copies 600 python3 -u bench.py --model llama-3-70b --concurrency 512 --steps 10 --warmup 3 --no-rtt --serve-load 0
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
