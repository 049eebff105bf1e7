#!/bin/bash
# round 5, call S: 4 ranks on one GPU (TP4 70B-2layer, Mixtral EP4) vs TP=1.
source tools/gpu_steps.sh
step r5s_tp4 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_tp_rehearsal_gpu.py -k tp4
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
