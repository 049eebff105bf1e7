#!/bin/bash
# round 6, call AM: moe_norm_route_kernel with the router rows loaded before the norm's reduction (once for all tokens)
# vs the previous kernel (_kernels_mnrold.so): kernel test, Mixtral-8x7B batch 1 / 4 A/B, one box.
source tools/gpu_steps.sh
step r6am_tests 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "moe_norm_route or moe_route or router"
B="python3 -u bench.py --steps 50 --warmup 3 --no-rtt --serve-load 0 --model mixtral-8x7b"
OLD=$PWD/nats_llm_studio_amd/_kernels_mnrold.so
step r6am_b1_new 300 $B --concurrency 1
NLS_KERNELS_SO=$OLD step r6am_b1_old 300 $B --concurrency 1
step r6am_b1_new2 300 $B --concurrency 1
NLS_KERNELS_SO=$OLD step r6am_b1_old2 300 $B --concurrency 1
step r6am_b4_new 300 $B --concurrency 4
NLS_KERNELS_SO=$OLD step r6am_b4_old 300 $B --concurrency 4
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
