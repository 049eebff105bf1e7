#!/bin/bash
# round 5, call Z: TP=4 one-GPU rehearsal with per-launch completion events: which launch of the late rank lagged.
source tools/gpu_steps.sh
export NLS_TP_TRACE=1 NLS_OP_TIMING=1
step r5z_a 200 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4 --no-ref
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
