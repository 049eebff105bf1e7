#!/bin/bash
# round 6, call AL: Mixtral-8x7B batch 1 (and 4) with the MoE norm + router + route folded into the o projection's last
# workgroup (NLS_MOE_FOLD_ROUTE=1) vs its own launch (default; r03 measured the fold slower), one box, back to back.
source tools/gpu_steps.sh
B="python3 -u bench.py --steps 50 --warmup 3 --no-rtt --serve-load 0 --model mixtral-8x7b"
step r6al_b1_sep 300 $B --concurrency 1
NLS_MOE_FOLD_ROUTE=1 step r6al_b1_fold 300 $B --concurrency 1
step r6al_b1_sep2 300 $B --concurrency 1
NLS_MOE_FOLD_ROUTE=1 step r6al_b1_fold2 300 $B --concurrency 1
step r6al_b4_sep 300 $B --concurrency 4
NLS_MOE_FOLD_ROUTE=1 step r6al_b4_fold 300 $B --concurrency 4
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
