#!/bin/bash
# round 5, call V: 4 processes on one GPU, eager add+norm prefill pattern, stop + device-clock history at the first timeout.
source tools/gpu_steps.sh
export NLS_AR_PROBE=1
step r5v_w4 200 python3 -u tools/diag/addnorm_ipc_stress.py --world 4 --iters 60
step r5v_w2 200 python3 -u tools/diag/addnorm_ipc_stress.py --world 2 --iters 60
exit $STEPS_RC
