#!/bin/bash
# round 4, call H: the fused add+norm one-shot with coherent epoch counters and a row-independent
# workgroup -> XCD map: the greedy TP rehearsal with its post-run window (timed out in calls E and G),
# then the one-shot kernel tests and the TP rehearsal tests
source tools/gpu_steps.sh
step tpw_fix 200 env NLS_TP_TRACE=1 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --profile-steps 8
step tpw_mixed 200 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --no-ref --profile-steps 8
step os_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "oneshot" tests/test_oneshot_ipc_gpu.py
step tp_tests 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_rehearsal_gpu.py
exit $STEPS_RC
