#!/bin/bash
# round 6, call AI: records at the final head -- a 200-step sustained run of the headline config, the other families
# at batch 1 (Llama-3-70B on one GPU, Mixtral-8x7B) and the 70B at 128 requests.
source tools/gpu_steps.sh
step r6ai_b512_200 600 python3 -u bench.py --steps 200 --warmup 5 --no-rtt --serve-load 0
B="python3 -u bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6ai_mx_b1 400 $B --model mixtral-8x7b --concurrency 1
rm -f /tmp/nls_bench/*.gguf
step r6ai_70b_b1 600 $B --model llama-3-70b --concurrency 1
step r6ai_70b_b128 600 $B --model llama-3-70b --concurrency 128
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
