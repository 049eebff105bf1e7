#!/bin/bash
# round 4, call C: mode-10 BN=128 correctness, then hand-written large-M GEMM configs vs hipBLASLt for every
# dense shape of the three families
source tools/gpu_steps.sh
step h10_tests 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "hgemm10 or qkv_rope_kv_dense"
[ $STEPS_RC -ne 0 ] && exit $STEPS_RC
step dt_8b 400 python3 -u tools/dense_tune.py --model llama-3-8b --M 256,512,1024,2048 --rounds 3 --emit
step dt_70b 420 python3 -u tools/dense_tune.py --model llama-3-70b --M 256,512,1024,2048 --rounds 3 --emit
step dt_qwen 300 python3 -u tools/dense_tune.py --model qwen2.5-7b --M 256,512,1024,2048 --rounds 3 --emit
exit $STEPS_RC
