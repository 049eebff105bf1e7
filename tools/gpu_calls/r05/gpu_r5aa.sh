#!/bin/bash
# round 5, call AA: TP=4 / EP=4 on one GPU with polling grids sized for co-resident ranks.
source tools/gpu_steps.sh
step r5aa_tp4 700 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_tp_rehearsal_gpu.py -k "tp4"
step r5aa_rep1 200 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4 --no-ref
step r5aa_rep2 200 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4 --no-ref
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
