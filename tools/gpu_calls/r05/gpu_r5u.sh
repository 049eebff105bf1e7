#!/bin/bash
# round 5, call U: TP=4 on one GPU with sampled requests (candidate gather over 3 peers), traced.
source tools/gpu_steps.sh
export NLS_TP_TRACE=1 NLS_AR_PROBE=1
step r5u_w4_sample 240 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4 --no-ref
step r5u_w4_sample_eager 240 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4 --no-ref --no-graphs
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
