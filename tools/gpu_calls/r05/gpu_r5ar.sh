#!/bin/bash
# round 5, call AR: decode attention at B=512 with K staged through LDS in whole-row loads (NLS_ATTN_KLDS=1) vs the
# 16-rows-x-64-byte K loads: time and the attention kernel tests under each.
source tools/gpu_steps.sh
for kl in 0 1; do
  export NLS_ATTN_KLDS=$kl
  step r5ar_probe256_$kl 120 python3 -u tools/attn_layout_probe.py --B 512 --ctx 256
  step r5ar_probe150_$kl 120 python3 -u tools/attn_layout_probe.py --B 512 --ctx 150
  step r5ar_probe1k_$kl 120 python3 -u tools/attn_layout_probe.py --B 128 --ctx 1024
  step r5ar_tests_$kl 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention and not prefill"
done
exit $STEPS_RC
