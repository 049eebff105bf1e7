#!/bin/bash
# round 4, call F: which condition makes the second prefill's fused add+norm one-shot time out in the
# 2-process / 1-GPU greedy TP rehearsal: graphs off, one hardware queue per process, a barrier before it
source tools/gpu_steps.sh
R="python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --no-ref"
step tpg_nographs 200 env NLS_TP_TRACE=1 $R --no-graphs
step tpg_hwq1 200 env NLS_TP_TRACE=1 GPU_MAX_HW_QUEUES=1 $R
step tpg_base 200 env NLS_TP_TRACE=1 $R
step attn_b1 200 python3 -u tools/attn_b1_probe.py
step attn_b1_w4 200 env NLS_ATTN_MFMA_WAVES=4 python3 -u tools/attn_b1_probe.py
exit $STEPS_RC
