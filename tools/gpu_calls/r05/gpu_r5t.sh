#!/bin/bash
# round 5, call T: diagnose the TP=4-on-one-GPU one-shot timeout (eager vs graphs, trace + device-clock probes).
source tools/gpu_steps.sh
export NLS_TP_TRACE=1 NLS_AR_PROBE=1
step r5t_w4_eager 240 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4 --no-ref --greedy-only --no-graphs
step r5t_w4_graph 240 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4 --no-ref --greedy-only
step r5t_w3_graph 240 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 3 --no-ref --greedy-only
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
