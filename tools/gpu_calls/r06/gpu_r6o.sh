#!/bin/bash
# round 6, call O: the re-tuned quantised large-M entries (mode 3 at 64-row blocks on Q|K|V / o; first Llama-3-70B
# entries at M = 128) in the model: 8B quantised-only B=512 / 256 next to the default (copies), 70B B=128 (quantised
# by the new copy policy).
source tools/gpu_steps.sh
B="python3 -u bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0"
NLS_DENSE_WEIGHTS=0 step r6o_8b_b512_q 300 $B
step r6o_8b_b512_d 300 $B
NLS_DENSE_WEIGHTS=0 step r6o_8b_b256_q 300 $B --concurrency 256
step r6o_8b_b256_d 300 $B --concurrency 256
rm -f /tmp/nls_bench/*.gguf
step r6o_70b_b128 600 $B --model llama-3-70b --concurrency 128
NLS_TUNING_EXTRA='{"12+12+12:10240:8192:128": [2, 8, 2, 3], "12+12+14:10240:8192:128": [2, 8, 2, 3], "12:57344:8192:128": [2, 8, 2, 1], "12:8192:28672:128": [2, 8, 4, 4], "12:8192:8192:128": [2, 8, 2, 4], "14:128256:8192:128": [2, 8, 4, 1], "14:8192:28672:128": [2, 8, 4, 4]}' step r6o_70b_b128_r05cfg 300 $B --model llama-3-70b --concurrency 128
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
