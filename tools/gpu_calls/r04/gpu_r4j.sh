#!/bin/bash
# round 4, call J: slot-block epochs (no consumed-tag rewrite) in every one-shot kernel: kernel tests,
# IPC tests, the TP/EP rehearsals incl. the second-prefill regression, and the eager kernel list of a TP
# decode step (the sequence the graph captures) for the no-RCCL evidence
source tools/gpu_steps.sh
step os_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "oneshot" tests/test_oneshot_ipc_gpu.py
step tp_tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_rehearsal_gpu.py
step tp_kernels 200 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --no-ref --no-graphs --profile-steps 4
exit $STEPS_RC
