#!/bin/bash
# round 4: Mixtral-8x7B B=256, expert down projection split over K (NLS_MOE_KS_DN = 1 default, 2, 3)
source tools/gpu_steps.sh
run() { local n=$1; shift; step mxks_$n 400 env "$@" python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model mixtral-8x7b --ftype Q5_K_M --concurrency 256 --steps 20 --warmup 3; }
run 1 NLS_MOE_KS_DN=1
run 2 NLS_MOE_KS_DN=2
run 3 NLS_MOE_KS_DN=3
for f in 1 2 3; do echo "ks_dn=$f $(grep -h '^{' gpurun_out/mxks_$f.log | cut -c150-230)"; done
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
