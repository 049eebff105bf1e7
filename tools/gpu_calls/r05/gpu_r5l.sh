#!/bin/bash
# round 5, call L: the expert-parallel decode exchange (ep_exchange.hip): the 2-process IPC test (random routing,
# bit-exact rows), then the TP / EP rehearsal tests (Mixtral EP2 tokens vs TP=1, graph node lists).
source tools/gpu_steps.sh
T="python3 -u -m pytest -x -q --timeout 200 --timeout-method thread"
step r5l_ipc 200 $T tests/test_oneshot_ipc_gpu.py
step r5l_tp 600 $T tests/test_tp_rehearsal_gpu.py
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
