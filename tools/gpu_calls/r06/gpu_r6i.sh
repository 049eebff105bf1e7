#!/bin/bash
# round 6, call I: Mixtral-8x7B B=256 down-projection config A/B in the model (mode 3 split 4 / split 2 / mode 2
# unsplit, gate|up on mode 3 in all), then Llama-3-70B on one GPU: quantised-only vs the default policy at B=128, and
# B=1 without (new default) / with the 139 GB of f16 copies.
source tools/gpu_steps.sh
B="python3 -u bench.py --model mixtral-8x7b --concurrency 256 --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6i_mx_dn3ks4 600 $B
NLS_MOE_QCFG_DN=2,8,4 NLS_MOE_KS_DN=1 step r6i_mx_dn2 300 $B
NLS_MOE_KS_DN=2 step r6i_mx_dn3ks2 300 $B
rm -f /tmp/nls_bench/*.gguf
B="python3 -u bench.py --model llama-3-70b --steps 20 --warmup 3 --no-rtt --serve-load 0"
NLS_DENSE_WEIGHTS=0 step r6i_70b_b128_q 600 $B --concurrency 128
step r6i_70b_b128_d 400 $B --concurrency 128
step r6i_70b_b1_d 300 $B --concurrency 1
NLS_DENSE_WEIGHTS=1 step r6i_70b_b1_copies 300 $B --concurrency 1
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
