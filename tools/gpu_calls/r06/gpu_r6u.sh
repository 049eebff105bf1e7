#!/bin/bash
# round 6, call U: long-prompt TTFT at the head (8K / 32K-token prompts, Llama-3.1-8B, chunked MFMA prefill).
source tools/gpu_steps.sh
step r6u_prefill 600 python3 -u tools/prefill_probe.py --lens 8192 32768 --model llama-3.1-8b --reps 2
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
