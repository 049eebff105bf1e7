#!/bin/bash
# round 5, call AE: TP=4 / EP=4 and TP=8 / EP=8 one-GPU rehearsal tests.
source tools/gpu_steps.sh
step r5ae_tp4 700 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_tp_rehearsal_gpu.py -k "tp4_tp8"
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
