#!/bin/bash
# round 4, call A: TP rehearsal + IPC kernels, prefill kernel tests, prefill TTFT (new vs v1 kernel)
source tools/gpu_steps.sh
step tp_tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_oneshot_ipc_gpu.py tests/test_tp_rehearsal_gpu.py
step prefill_tests 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attention_prefill
step pf_v2 500 python -u tools/prefill_probe.py --lens 8192 32768 --reps 2
step pf_v1 500 env NLS_PREFILL_V1=1 python -u tools/prefill_probe.py --lens 8192 32768 --reps 1
exit $STEPS_RC
