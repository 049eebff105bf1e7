#!/bin/bash
# round 4, call L: the fused add+norm one-shot under its launch options (consumed-granule re-tag on/off,
# L2 invalidate before every re-poll on/off): simulated ranks per call / row, then the traced greedy rehearsal
source tools/gpu_steps.sh
for r in 0 1; do for i in 0 1; do
  step sim_r${r}_i${i} 120 env NLS_AR_RETAG=$r NLS_AR_POLL_INV=$i python3 -u tools/addnorm_sim_probe.py
  cat gpurun_out/sim_r${r}_i${i}.log | grep '^{'
done; done
for r in 0 1; do
  step reh_r${r}_i1 200 env NLS_TP_TRACE=1 NLS_AR_RETAG=$r NLS_AR_POLL_INV=1 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --profile-steps 8
  grep -h "error words\|timeout_addnorm" gpurun_out/reh_r${r}_i1.log | cut -c1-200 | head -3
done
exit $STEPS_RC
