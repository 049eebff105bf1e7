#!/bin/bash
# round 6, call F: Mixtral grouped expert GEMM occupancy / split-K sweep (tools/diag/moe_probe.py, B=256), then the
# f16-copy policy evidence (call D's steps): quantised-only vs copies for the 8B at B=512 / 256, the 70B at B=128 / 1.
source tools/gpu_steps.sh
P="python3 -u tools/diag/moe_probe.py --T 256 --iters 20"
for c in 2,8,4,1 2,8,2,1 2,8,1,1; do step r6f_moe_gu_${c//,/_} 120 $P --proj gateup --cfg $c; done
for c in 2,8,4,1 2,8,4,2 2,8,4,4 2,8,2,2 2,8,1,1 2,8,1,2 2,8,1,4; do step r6f_moe_dn_${c//,/_} 120 $P --proj down --cfg $c; done
B="python3 -u bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0"
NLS_DENSE_WEIGHTS=0 step r6d_8b_b512_q 400 $B
step r6d_8b_b512_d 400 $B
NLS_DENSE_WEIGHTS=0 step r6d_8b_b256_q 400 $B --concurrency 256
step r6d_8b_b256_d 400 $B --concurrency 256
NLS_DENSE_WEIGHTS=0 step r6d_70b_b128_q 600 $B --model llama-3-70b --concurrency 128
step r6d_70b_b128_d 600 $B --model llama-3-70b --concurrency 128
NLS_DENSE_WEIGHTS=0 step r6d_70b_b1_q 600 $B --model llama-3-70b --concurrency 1
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
