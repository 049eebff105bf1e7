#!/bin/bash
# round 5, call BB: full GPU suite + smoke at the final head (fp8-conversion dequant + re-tuned batch-1 Q|K|V entry), the driver's bench
# command, and the batch-1 bench.
source tools/gpu_steps.sh
step r5bb_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step r5bb_smoke 120 python3 -u __graft_entry__.py smoke
step r5bb_bench 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
step r5bb_b1 300 python3 -u bench.py --concurrency 1 --steps 100 --warmup 5 --no-rtt --serve-load 0
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
