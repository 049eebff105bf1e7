#!/bin/bash
# round 6, call AP: decode attention K/V rate vs context at B=512 (the bench's timed steps sit at ~135-155 keys):
# tools/attn_layout_probe.py at ctx 128 / 144 / 192 / 256 / 512, contiguous and churned block placement.
source tools/gpu_steps.sh
for c in 128 144 192 256 512; do
  step r6ap_ctx$c 120 python3 -u tools/attn_layout_probe.py --B 512 --ctx $c
done
step r6ap_ctx144_perm 120 python3 -u tools/attn_layout_probe.py --B 512 --ctx 144 --perm
exit $STEPS_RC
