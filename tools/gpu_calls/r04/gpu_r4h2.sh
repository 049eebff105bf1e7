#!/bin/bash
# round 4, call H2: which row / slice / epoch of the second prefill's fused add+norm one-shot times out
source tools/gpu_steps.sh
step tpw_diag 200 env NLS_TP_TRACE=1 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --no-ref --profile-steps 8
exit $STEPS_RC
