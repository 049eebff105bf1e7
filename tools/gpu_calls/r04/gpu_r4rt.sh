#!/bin/bash
# round 4: the MoE router kernel (ops.router_logits): kernel test, Mixtral GPU tests (model, rehearsal), then
# Mixtral-8x7B Q5_K_M at B=256 and B=1 with it and with the GEMV router (NLS_ROUTER_KERNEL=0)
source tools/gpu_steps.sh
step rt_tests 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "router or moe"
step mx_tests 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_tp_rehearsal_gpu.py -k "mixtral"
run() { local n=$1 c=$2; shift 2; step mxr_$n 400 env "$@" python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model mixtral-8x7b --ftype Q5_K_M --concurrency $c --steps 20 --warmup 3; }
run b256_kernel 256 NLS_X=0
run b256_gemv 256 NLS_ROUTER_KERNEL=0
run b1_kernel 1 NLS_X=0
run b1_gemv 1 NLS_ROUTER_KERNEL=0
for f in b256_kernel b256_gemv b1_kernel b1_gemv; do echo "$f $(grep -h '^{' gpurun_out/mxr_$f.log | cut -c150-230)"; done
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
