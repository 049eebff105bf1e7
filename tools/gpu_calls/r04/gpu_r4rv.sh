#!/bin/bash
# round 4: re-check of the router kernel at the committed head (router / MoE kernel tests, every MoE GPU test incl.
# the EP all-to-all rehearsal, Mixtral B=256)
source tools/gpu_steps.sh
step rt_tests 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "router or moe"
step moe_tests 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_tp_rehearsal_gpu.py tests/test_production_gpu.py
step mx256 400 python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model mixtral-8x7b --ftype Q5_K_M --concurrency 256 --steps 20 --warmup 3
grep -h '^{' gpurun_out/mx256.log | cut -c150-230
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
