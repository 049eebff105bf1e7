#!/bin/bash
# round 4, call D: TP rehearsal with the control-op trace (profile window), the rehearsal tests again, and a
# batch-1 A/B of the XL GEMV weight prefetch depth at two row tiles per wave (gate|up), then the B=512 decode
# headline with the r04 dense-tune table
source tools/gpu_steps.sh
step tp_trace 300 env NLS_TP_TRACE=1 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --no-ref --profile-steps 8
step tp_tests 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_rehearsal_gpu.py
for v in "" d3 d4; do
  so=nats_llm_studio_amd/_kernels${v:+_$v}.so
  step b1_${v:-base} 240 env NLS_KERNELS_SO=$PWD/$so python3 -u bench.py --concurrency 1 --steps 100 --warmup 10 --serve-load 0 --no-rtt --tp-leg 0
  grep '^{' gpurun_out/b1_${v:-base}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], 'ms/token')"
done
step b512 400 python3 -u bench.py --steps 100 --warmup 10 --serve-load 0 --no-rtt --tp-leg 0
exit $STEPS_RC
