#!/bin/bash
# round 5, call AF: TP=8 / EP=8 rehearsal on one GPU (8 processes).
source tools/gpu_steps.sh
step r5af_tp8 300 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 8
step r5af_ep8 300 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 8 --model mixtral-8x7b-1layer --ep
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
