#!/bin/bash
# round 5, call Y: TP=4 one-GPU rehearsal (sampled rows) under fewer HW queues per process / no SDMA / default.
source tools/gpu_steps.sh
export GPU_MAX_HW_QUEUES=1; step r5y_q1 200 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4 --no-ref
export GPU_MAX_HW_QUEUES=2; step r5y_q2 200 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4 --no-ref
unset GPU_MAX_HW_QUEUES; export HSA_ENABLE_SDMA=0; step r5y_nosdma 200 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4 --no-ref
unset HSA_ENABLE_SDMA; step r5y_default 200 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4 --no-ref
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
