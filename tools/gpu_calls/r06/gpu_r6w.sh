#!/bin/bash
# round 6, call W: the service burst (512 chat_model requests, half sampled, 256 tokens) with the engine's prefill chunk
# at 2048 (default) / 4096 / 8192 tokens -- larger prefill GEMMs for the 55K-token prompt backlog, TTFT and service tok/s.
source tools/gpu_steps.sh
B="python3 -u bench.py --steps 20 --warmup 5"
step r6w_pf2048 400 $B --prefill-tokens 2048
step r6w_pf4096 400 $B --prefill-tokens 4096
step r6w_pf8192 400 $B --prefill-tokens 8192
step r6w_pf2048b 400 $B --prefill-tokens 2048
rm -f /tmp/nls_bench/*.gguf
BS=1 MODEL=qwen2.5-7b step r6w_qwen_prof 500 bash tools/gpu_prof.sh
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
