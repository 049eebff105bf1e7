#!/bin/bash
# round 5, call AB: TP=4 / EP=4 rehearsal tests, and the world-4 rehearsal with the old 128-workgroup grid forced.
source tools/gpu_steps.sh
step r5ab_tp4 700 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_tp_rehearsal_gpu.py -k "tp4"
export NLS_AR_NORM_WGS=128
step r5ab_old1 200 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4 --no-ref
step r5ab_old2 200 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --world 4 --no-ref
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
