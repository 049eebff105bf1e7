#!/bin/bash
# round 4, call T: 4-wave dense GEMM tiles (64 x 64 per wave): kernel tests, then the dense tune of the
# Llama-3-8B projections at 256 / 512 rows with them among the candidates
source tools/gpu_steps.sh
step dense_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "hgemm_dense"
step dt4 600 python3 -u tools/dense_tune.py --model llama-3-8b --M 256,512,1024,2048 --roles qkv,o,down --emit
grep -h "EMIT" gpurun_out/dt4.log | cut -c1-600
exit $STEPS_RC
