#!/bin/bash
# round 6, call AA: Q|K|V at decode batches with split-K (RoPE then runs as its own launch) vs unsplit (RoPE in the GEMM
# epilogue): Qwen2.5-7B B=512 ("d:4608:3584:512" [10,8,2,3] vs [10,8,2,1] / [4,16,2,1]), Llama-3-8B and Mixtral B=256
# ("d:6144:4096:256" [4,16,2,2] vs [4,16,2,1]). NLS_TUNING_EXTRA overrides, one box, back to back.
source tools/gpu_steps.sh
B="python3 -u bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6aa_qw_cur 300 $B --model qwen2.5-7b
NLS_TUNING_EXTRA='{"d:4608:3584:512": [10, 8, 2, 1]}' step r6aa_qw_m10 300 $B --model qwen2.5-7b
NLS_TUNING_EXTRA='{"d:4608:3584:512": [4, 16, 2, 1]}' step r6aa_qw_m4 300 $B --model qwen2.5-7b
step r6aa_qw_cur2 300 $B --model qwen2.5-7b
rm -f /tmp/nls_bench/*.gguf
step r6aa_8b256_cur 300 $B --concurrency 256
NLS_TUNING_EXTRA='{"d:6144:4096:256": [4, 16, 2, 1]}' step r6aa_8b256_ks1 300 $B --concurrency 256
rm -f /tmp/nls_bench/*.gguf
step r6aa_mx_cur 400 $B --model mixtral-8x7b --concurrency 256
NLS_TUNING_EXTRA='{"d:6144:4096:256": [4, 16, 2, 1]}' step r6aa_mx_ks1 300 $B --model mixtral-8x7b --concurrency 256
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
