#!/bin/bash
# round 6, call K: the mode-3 96-row blocks skipping their padding tiles (NLS_DMA_NA=1, default build) vs multiplying
# all six (the _kernels_nona.so variant): mapped-MoE kernel tests, the isolated gate|up launch, and the Mixtral B=256 step.
source tools/gpu_steps.sh
T="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
step r6k_mapped_tests 300 $T tests/test_kernels_gpu.py -k "mapped_moe"
[ $STEPS_RC -ne 0 ] && exit $STEPS_RC
P="python3 -u tools/diag/moe_probe.py --T 256 --iters 20 --proj gateup --cfg 3,4,6,1"
step r6k_gu_na 120 $P
NLS_KERNELS_SO=$PWD/nats_llm_studio_amd/_kernels_nona.so step r6k_gu_nona 120 $P
step r6k_gu_na2 120 $P
B="python3 -u bench.py --model mixtral-8x7b --concurrency 256 --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6k_mx_na 600 $B
NLS_KERNELS_SO=$PWD/nats_llm_studio_amd/_kernels_nona.so step r6k_mx_nona 300 $B
step r6k_mx_na2 300 $B
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
