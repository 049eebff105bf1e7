#!/bin/bash
# round 5, call AK: short single-prompt prefill (chat_model RTT case): host launch time vs GPU time of the forward.
source tools/gpu_steps.sh
step r5ak_pf 300 python3 -u tools/diag/prefill_small.py --tokens 21 --reps 8 --cprofile
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
