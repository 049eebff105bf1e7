#!/bin/bash
# round 5, call W: TP=4 rehearsal failure with a 32-deep device-clock history; the add+norm stress with async ranks.
source tools/gpu_steps.sh
export NLS_AR_PROBE=1 NLS_TP_TRACE=1
step r5w_rehearsal 240 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4 --no-ref
unset NLS_TP_TRACE
step r5w_w4_async 200 python3 -u tools/diag/addnorm_ipc_stress.py --world 4 --iters 64 --batch 8
step r5w_w4_jit 200 python3 -u tools/diag/addnorm_ipc_stress.py --world 4 --iters 64 --batch 8 --jitter 20 --gemms 6
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
