#!/bin/bash
# round 5, call AD: TP=4 request 9: candidate path off (full-logit gather) -- logits vs candidate logic.
source tools/gpu_steps.sh
export NLS_TP_CANDIDATES=0
step r5ad_full 200 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
