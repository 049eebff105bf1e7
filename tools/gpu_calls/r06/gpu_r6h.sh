#!/bin/bash
# round 6, call H: Mixtral-8x7B B=256 with the mapped LDS-DMA expert GEMMs (new default) vs the r05 configs, its
# rocprofv3 breakdown; then the 8B f16-copy A/B (quantised-only vs copies) at B=512 / 256.
source tools/gpu_steps.sh
B="python3 -u bench.py --model mixtral-8x7b --concurrency 256 --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6h_mx_new 600 $B
NLS_MOE_DMA=0 NLS_MOE_KS_DN=1 step r6h_mx_old 400 $B
BS=256 MODEL=mixtral-8x7b FTYPE=Q5_K_M step r6h_mx_prof 500 bash tools/gpu_prof.sh
rm -f /tmp/nls_bench/*.gguf
B="python3 -u bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0"
NLS_DENSE_WEIGHTS=0 step r6h_8b_b512_q 300 $B
step r6h_8b_b512_d 300 $B
NLS_DENSE_WEIGHTS=0 step r6h_8b_b256_q 300 $B --concurrency 256
step r6h_8b_b256_d 300 $B --concurrency 256
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
