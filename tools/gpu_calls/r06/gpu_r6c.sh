#!/bin/bash
# round 6, call C: re-tag root cause (NLS_AR_RETAG=0 with the normaliser's x re-check, plain vs agent-scope row reads),
# the GPU kernel suite, the TP/EP rehearsals (EP payload checksums, no PyTorch kernels in decode graphs), the bench.
source tools/gpu_steps.sh
T="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
NLS_AR_RETAG=0 NLS_AR_XCHECK=1 NLS_AR_XPLAIN=1 step r6c_retag0_plain 120 python3 -u tools/diag/addnorm_sim.py 2 16 4096 12
NLS_AR_RETAG=0 NLS_AR_XCHECK=1 step r6c_retag0_agent 120 python3 -u tools/diag/addnorm_sim.py 2 16 4096 12
NLS_AR_RETAG=1 NLS_AR_XCHECK=1 NLS_AR_XPLAIN=1 step r6c_retag1_plain 120 python3 -u tools/diag/addnorm_sim.py 2 16 4096 12
NLS_AR_RETAG=0 NLS_AR_XCHECK=1 step r6c_retag0_agent_w8 120 python3 -u tools/diag/addnorm_sim.py 8 64 8192 12
step r6c_kern 900 $T tests/test_kernels_gpu.py
step r6c_tp 900 $T tests/test_tp_rehearsal_gpu.py
step r6c_bench 400 python3 -u bench.py --steps 20 --warmup 5 --no-rtt --serve-load 0
exit $STEPS_RC
