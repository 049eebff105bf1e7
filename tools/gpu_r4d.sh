#!/bin/bash
# round 4, call D: batch-1 A/B of the XL GEMV weight prefetch depth at two row tiles per wave (gate|up)
source tools/gpu_steps.sh
for v in "" d3 d4; do
  so=nats_llm_studio_amd/_kernels${v:+_$v}.so
  step b1_${v:-base} 240 env NLS_KERNELS_SO=$PWD/$so python3 -u bench.py --concurrency 1 --steps 100 --warmup 10 --serve-load 0 --no-rtt --tp-leg 0
  grep '^{' gpurun_out/b1_${v:-base}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], 'ms/token')"
done
exit $STEPS_RC
