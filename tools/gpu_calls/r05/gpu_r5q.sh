#!/bin/bash
# round 5, call Q: per-launch cost of a batch-1 graph chain; B=512 and B=1 kernel traces of the head.
source tools/gpu_steps.sh
step r5q_launch 200 python3 -u tools/diag/launch_cost.py
export BS="512 1"; step r5q_prof 900 bash tools/gpu_prof.sh
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
