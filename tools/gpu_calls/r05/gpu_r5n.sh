#!/bin/bash
# round 5, call N: long-prompt TP prefill (row-parallel chunks, one-shot all-reduce on the comm side stream) vs TP=1.
source tools/gpu_steps.sh
step r5n_long 300 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_tp_rehearsal_gpu.py -k long_prompt
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
