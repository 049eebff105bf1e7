#!/bin/bash
# round 6, call P: fresh rocprofv3 breakdowns of the head (Llama-3-8B B=512 and B=1), and the other families at the head
# (Qwen2.5-7B B=512 / 1, Granite-3.0-2B B=512 / 1, Mixtral-8x7B B=1).
source tools/gpu_steps.sh
BS="512 1" step r6p_prof 700 bash tools/gpu_prof.sh
rm -f /tmp/nls_bench/*.gguf
B="python3 -u bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6p_qwen_b512 400 $B --model qwen2.5-7b
step r6p_qwen_b1 300 $B --model qwen2.5-7b --concurrency 1
rm -f /tmp/nls_bench/*.gguf
step r6p_granite_b512 300 $B --model granite-3.0-2b
step r6p_granite_b1 300 $B --model granite-3.0-2b --concurrency 1
rm -f /tmp/nls_bench/*.gguf
step r6p_mx_b1 400 $B --model mixtral-8x7b --concurrency 1
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
