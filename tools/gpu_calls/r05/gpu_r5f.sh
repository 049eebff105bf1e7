#!/bin/bash
# round 5, call F: the fused add+norm on a bounded grid (<= 128 workgroups, every item pushed before any poll).
# (1) one-shot kernel tests, re-tag on and off; (2) the 2-process eager rehearsal that timed out (re-tag on / off,
# probe timings kept); (3) the TP rehearsal tests with eager one-shot calls.
source tools/gpu_steps.sh
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
step r5f_kern 300 $T tests/test_kernels_gpu.py tests/test_oneshot_ipc_gpu.py -k "oneshot"
step r5f_kern_noretag 300 env NLS_AR_RETAG=0 $T tests/test_kernels_gpu.py -k "oneshot"
R="python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --profile-steps 4 --no-ref"
step r5f_eager 200 env NLS_TP_TRACE=1 NLS_REHEARSAL_WAVES=1 NLS_ONESHOT_EAGER=1 NLS_AR_PROBE=1 $R
step r5f_eager_noretag 200 env NLS_TP_TRACE=1 NLS_REHEARSAL_WAVES=1 NLS_ONESHOT_EAGER=1 NLS_AR_PROBE=1 NLS_AR_RETAG=0 $R
step r5f_tp 600 env NLS_ONESHOT_EAGER=1 $T tests/test_tp_rehearsal_gpu.py
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
