#!/bin/bash
# round 5, call BF: full GPU suite + smoke at the final head (all re-tuned entries, rebuilt library), the driver's bench
# command, and the batch-1 bench.
source tools/gpu_steps.sh
step r5bf_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step r5bf_smoke 120 python3 -u __graft_entry__.py smoke
step r5bf_bench 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
step r5bf_b1 300 python3 -u bench.py --concurrency 1 --steps 100 --warmup 5 --no-rtt --serve-load 0
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
