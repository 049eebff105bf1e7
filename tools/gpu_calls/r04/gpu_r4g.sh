#!/bin/bash
# round 4, call G: the greedy TP rehearsal WITH the post-run window (the second prefill, which timed out in
# call E) under: the same conditions, graphs off, one hardware queue per process, every rank idle + barrier
# before the window; then the KV-pressure run with the expected-growth admission
source tools/gpu_steps.sh
R="python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --no-ref --profile-steps 8"
step tpw_base 200 env NLS_TP_TRACE=1 $R
step tpw_nographs 200 env NLS_TP_TRACE=1 $R --no-graphs
step tpw_hwq1 200 env NLS_TP_TRACE=1 GPU_MAX_HW_QUEUES=1 $R
step tpw_barrier 200 env NLS_TP_TRACE=1 NLS_REHEARSAL_BARRIER=1 $R
step kvp 400 python3 -u tools/kv_pressure.py --n 512 --max-tokens 1024 --kv-fraction 0.03
exit $STEPS_RC
