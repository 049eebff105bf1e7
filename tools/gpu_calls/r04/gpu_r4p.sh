#!/bin/bash
# round 4, call P: batch-1 gate|up weight stream -- 7 waves x one 16-row tile (256 workgroups) vs 4 x 2 (224)
# and 8 x 1, at XL prefetch depths 8 (default) / 4 / 2 for one-tile waves; then the B=1 step with the winner
source tools/gpu_steps.sh
C='[[1,4,2,1],[1,7,1,1],[1,8,1,1]]'
for v in "" x4 x2; do
  so=$PWD/nats_llm_studio_amd/_kernels${v:+_$v}.so
  step gu_${v:-base} 120 env NLS_KERNELS_SO=$so python3 -u tools/l3_warm_probe.py --shape gateup --cfgs "$C"
  grep -h '^{' gpurun_out/gu_${v:-base}.log | cut -c1-200
done
for v in "" x4; do
  so=$PWD/nats_llm_studio_amd/_kernels${v:+_$v}.so
  step b1w7_${v:-base} 120 env NLS_KERNELS_SO=$so NLS_TUNING_EXTRA='{"12:28672:4096:1": [1, 7, 1, 1]}' python3 -u bench.py --concurrency 1 --steps 100 --warmup 10 --serve-load 0 --no-rtt --tp-leg 0
  grep -h '^{' gpurun_out/b1w7_${v:-base}.log | cut -c1-160
done
step b1_base 120 python3 -u bench.py --concurrency 1 --steps 100 --warmup 10 --serve-load 0 --no-rtt --tp-leg 0
grep -h '^{' gpurun_out/b1_base.log | cut -c1-160
exit $STEPS_RC
