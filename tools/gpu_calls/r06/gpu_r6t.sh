#!/bin/bash
# round 6, call T: B=512 decode attention in the 4-wave MFMA form (a workgroup of 4 waves splitting each (token, kv head)'s
# keys; NLS_ATTN_MFMA_BIG above the grid size) vs the default one-wave form, Llama-3-8B and Granite-3.0-2B, back to back.
source tools/gpu_steps.sh
B="python3 -u bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6t_8b_w1 300 $B
NLS_ATTN_MFMA_BIG=100000000 step r6t_8b_w4 300 $B
step r6t_8b_w1b 300 $B
rm -f /tmp/nls_bench/*.gguf
step r6t_gr_w1 300 $B --model granite-3.0-2b
NLS_ATTN_MFMA_BIG=100000000 step r6t_gr_w4 300 $B --model granite-3.0-2b
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
