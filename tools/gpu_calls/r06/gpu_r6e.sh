#!/bin/bash
# round 6, call E: the fence-free stage-handoff gate (tools/diag/fencefree_chain.py), the one-shot kernel tests with
# the re-tag OFF (agent-scope normaliser reads = default, then the r05 plain reads), the kernel suite, the TP/EP
# rehearsals (no PyTorch kernels in decode graphs, EP payload checksums).
source tools/gpu_steps.sh
T="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
step r6e_chain 180 python3 -u tools/diag/fencefree_chain.py 64 20
NLS_AR_RETAG=0 NLS_AR_XCHECK=1 step r6e_retag0_agent 300 $T tests/test_kernels_gpu.py -k oneshot
NLS_AR_RETAG=0 NLS_AR_XCHECK=1 NLS_AR_XPLAIN=1 step r6e_retag0_plain 300 $T tests/test_kernels_gpu.py -k oneshot
step r6e_kern 900 $T tests/test_kernels_gpu.py
step r6e_tp 900 $T tests/test_tp_rehearsal_gpu.py
exit $STEPS_RC
