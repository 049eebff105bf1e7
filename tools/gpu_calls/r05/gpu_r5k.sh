#!/bin/bash
# round 5, call K: the driver's default bench (20 steps) with the native pre-tokeniser (service_load tokenize phase),
# batch 1, Mixtral B=256, and the TP rehearsal tests with eager IPC collectives on by default.
source tools/gpu_steps.sh
step r5k_bench20 300 python3 -u bench.py --steps 20 --warmup 5
step r5k_b1 300 python3 -u bench.py --concurrency 1 --steps 100 --warmup 5 --serve-load 0 --no-rtt --tp-leg 0
step r5k_mx 400 python3 -u bench.py --model mixtral-8x7b --ftype Q5_K_M --concurrency 256 --steps 20 --warmup 5 --serve-load 0 --no-rtt --tp-leg 0
grep -h '^{' gpurun_out/r5k_*.log | cut -c1-300
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
