#!/bin/bash
# round 6, call D: f16-copy policy evidence -- quantised-only vs copies for the 8B at B=512 / 256 and the 70B at B=128 / 1.
source tools/gpu_steps.sh
B="python3 -u bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0"
NLS_DENSE_WEIGHTS=0 step r6d_8b_b512_q 400 $B
step r6d_8b_b512_d 400 $B
NLS_DENSE_WEIGHTS=0 step r6d_8b_b256_q 400 $B --concurrency 256
step r6d_8b_b256_d 400 $B --concurrency 256
NLS_DENSE_WEIGHTS=0 step r6d_70b_b128_q 600 $B --model llama-3-70b --concurrency 128
step r6d_70b_b128_d 600 $B --model llama-3-70b --concurrency 128
NLS_DENSE_WEIGHTS=0 step r6d_70b_b1_q 600 $B --model llama-3-70b --concurrency 1
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
