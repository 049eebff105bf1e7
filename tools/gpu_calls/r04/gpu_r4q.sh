#!/bin/bash
# round 4, call Q: in-model batch-1 A/B of gate|up at XL depth 2 for one-tile waves: 8 x 1 and 7 x 1 vs 4 x 2
source tools/gpu_steps.sh
so=$PWD/nats_llm_studio_amd/_kernels_x2.so
for c in "1, 8, 1, 1" "1, 7, 1, 1" "1, 4, 2, 1"; do
  n=$(echo $c | tr -d ' ,')
  step b1q_$n 120 env NLS_KERNELS_SO=$so NLS_TUNING_EXTRA="{\"12:28672:4096:1\": [$c]}" python3 -u bench.py --concurrency 1 --steps 100 --warmup 10 --serve-load 0 --no-rtt --tp-leg 0
  grep -h '^{' gpurun_out/b1q_$n.log | cut -c150-230
done
step b1q_base 120 python3 -u bench.py --concurrency 1 --steps 100 --warmup 10 --serve-load 0 --no-rtt --tp-leg 0
grep -h '^{' gpurun_out/b1q_base.log | cut -c150-230
exit $STEPS_RC
