#!/bin/bash
# round 4, last call: the whole GPU suite at the head (router kernel at one token per 8-wave workgroup), smoke,
# the driver's 20-step bench, and Mixtral B=256
source tools/gpu_steps.sh
step gpu_suite 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench20 300 python3 -u bench.py --steps 20 --warmup 5
step mx256 400 python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model mixtral-8x7b --ftype Q5_K_M --concurrency 256 --steps 20 --warmup 3
grep -h '^{' gpurun_out/bench20.log gpurun_out/mx256.log | cut -c150-260
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
