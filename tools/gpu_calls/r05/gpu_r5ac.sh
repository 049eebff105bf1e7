#!/bin/bash
# round 5, call AC: TP=4 sampled-token (in)stability: ref + TP4 twice, tokens compared.
source tools/gpu_steps.sh
step r5ac_1 200 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4
step r5ac_2 200 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4
step r5ac_w2 200 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 2
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
