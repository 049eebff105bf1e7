#!/bin/bash
# round 4, call K: XCD-aligned fused add+norm grid + slot-block epochs everywhere + per-kernel timeout
# diagnostics: one-shot kernel tests, traced greedy rehearsals (70B TP2, Mixtral EP2), TP rehearsal tests
source tools/gpu_steps.sh
step os_tests 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "oneshot or sample" tests/test_oneshot_ipc_gpu.py
step tpk_70b 200 env NLS_TP_TRACE=1 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --profile-steps 8
step tpk_mix 200 env NLS_TP_TRACE=1 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --model mixtral-8x7b-1layer --ep --greedy-only --profile-steps 8
step tp_tests 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_tp_rehearsal_gpu.py
exit $STEPS_RC
