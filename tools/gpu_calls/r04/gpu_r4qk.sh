#!/bin/bash
# round 4: Q|K|V at 256 rows -- split-K slabs + the separate RoPE/KV kernel (table: d:6144:4096:256 = 4,16,2,2) vs
# one launch with RoPE + KV append in the GEMM epilogue (ks 1), Llama-3-8B and Mixtral-8x7B at B=256
source tools/gpu_steps.sh
X='{"d:6144:4096:256": [4, 16, 2, 1]}'
step l8_base 300 python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --concurrency 256 --steps 20 --warmup 5
step l8_ks1 300 env NLS_TUNING_EXTRA="$X" python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --concurrency 256 --steps 20 --warmup 5
step mx_base 400 python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model mixtral-8x7b --ftype Q5_K_M --concurrency 256 --steps 20 --warmup 3
step mx_ks1 400 env NLS_TUNING_EXTRA="$X" python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model mixtral-8x7b --ftype Q5_K_M --concurrency 256 --steps 20 --warmup 3
for f in l8_base l8_ks1 mx_base mx_ks1; do echo "$f $(grep -h '^{' gpurun_out/$f.log | cut -c150-230)"; done
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
