#!/bin/bash
# round 4: Mixtral-8x7B prefill TTFT (one 8K-token prompt, 2048-token chunks) with the E-row router kernel and
# with the GEMV router
source tools/gpu_steps.sh
step mxpf_kernel 400 python3 -u tools/prefill_probe.py --model mixtral-8x7b --lens 8192 --reps 2
step mxpf_gemv 400 env NLS_ROUTER_KERNEL=0 python3 -u tools/prefill_probe.py --model mixtral-8x7b --lens 8192 --reps 2
grep -h '^{' gpurun_out/mxpf_kernel.log gpurun_out/mxpf_gemv.log
rm -rf /tmp/nls_bench
exit $STEPS_RC
