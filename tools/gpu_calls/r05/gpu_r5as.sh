#!/bin/bash
# round 5, call AS: Mixtral-8x7B B=256 kernel breakdown (rocprofv3) at the head.
source tools/gpu_steps.sh
export BS=256 MODEL=mixtral-8x7b FTYPE=Q5_K_M
step r5as_prof 900 bash tools/gpu_prof.sh
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
