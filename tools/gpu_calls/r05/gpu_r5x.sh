#!/bin/bash
# round 5, call X: TP=4 rehearsal failure with host launch times of the add+norm calls.
source tools/gpu_steps.sh
export NLS_AR_PROBE=1 NLS_TP_TRACE=1
step r5x_rehearsal 240 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4 --no-ref
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
