#!/bin/bash
# round 5, call AJ: bench with the native list_models responder; the engine chat_model RTT phase breakdown.
source tools/gpu_steps.sh
step r5aj_bench 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
