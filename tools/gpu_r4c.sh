#!/bin/bash
# round 4, call C: hand-written large-M GEMM configs vs hipBLASLt for every dense shape of the three families
source tools/gpu_steps.sh
step dt_8b 300 python3 -u tools/dense_tune.py --model llama-3-8b --M 256,512,1024,2048 --emit
step dt_70b 420 python3 -u tools/dense_tune.py --model llama-3-70b --M 256,512,1024,2048 --emit
step dt_qwen 300 python3 -u tools/dense_tune.py --model qwen2.5-7b --M 256,512,1024,2048 --emit
exit $STEPS_RC
